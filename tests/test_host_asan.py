"""Host code under AddressSanitizer + UBSan (SURVEY.md s5 "race detection / sanitizers"): the engine's
host graph preparation (csrc/host_graph.cpp) and the drop-in header's threaded flatten / KeyIndex /
materialisation (include/ppr/grank.h), compiled with g++ -fsanitize=address,undefined
(build.build_host_asan, tests/cpp/host_asan_test.cc). Every run must be clean (any sanitizer report
aborts the driver) and produce the production library's results. No device code is involved."""
import os
import subprocess

import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr

FNV0 = 1469598103934665603


def fnv(b: bytes, h: int = FNV0) -> int:
    for x in b:
        h ^= x
        h = (h * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.fixture(scope="module")
def asan():
    from approximated_personalized_pagerank_amd import build
    return build.build_host_asan(force=True)


def run(binary, *args):
    env = dict(os.environ, ASAN_OPTIONS="halt_on_error=1:abort_on_error=1:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    p = subprocess.run([binary, *map(str, args)], capture_output=True, text=True, env=env, timeout=300)
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-4000:]
    assert p.returncode == 0, p.stderr[-4000:]
    import json
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("scale,seed", [(10, 1), (12, 5)])
def test_graph_prep_sanitized_matches_library(asan, scale, seed):
    d = run(asan, "graph", scale, seed)
    g = ppr.rmat(scale, seed=seed)
    assert d["n"] == g.n and d["m"] == g.m
    csr = fnv(np.ascontiguousarray(g.col, dtype=np.int32).tobytes(),
              fnv(np.ascontiguousarray(g.row_ptr, dtype=np.int64).tobytes()))
    assert d["csr"] == f"{csr:016x}"
    assert d["part"] == f"{fnv(g.partitions().astype(np.uint8).tobytes()):016x}"
    assert d["order"] == f"{fnv(g.execution_order().astype(np.int32).tobytes()):016x}"


def test_flatten_and_materialise_sanitized(asan):
    assert run(asan, "flatten", 16)["bad"] == 0


def test_flatten_sparse_keys_sanitized(asan):
    """keys far apart take the KeyIndex hash (dense ids take its direct array)"""
    assert run(asan, "flatten_sparse", 14)["bad"] == 0


def test_csv_import_sanitized(asan, tmp_path):
    path = tmp_path / "g.csv"
    rng = np.random.default_rng(3)
    e = rng.integers(0, 500, size=(4000, 2))
    path.write_text("".join(f"{a},{b}\r\n" for a, b in e))
    d = run(asan, "csv", str(path))
    g = ppr.import_edge_csv(str(path))
    assert d["n"] == g.n and d["m"] == g.m
    csr = fnv(np.ascontiguousarray(g.col, dtype=np.int32).tobytes(),
              fnv(np.ascontiguousarray(g.row_ptr, dtype=np.int64).tobytes()))
    assert d["csr"] == f"{csr:016x}"
