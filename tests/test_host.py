"""CPU-only checks of the product library's host side and ABI (no device calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr
from approximated_personalized_pagerank_amd import _lib
from helpers import all_names, load

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "ppr_hip.h")).read()
    return sorted(set(re.findall(r"\b(ppr_[a-z0-9_]+)\s*\(", src)))


def test_abi_exports_every_declared_symbol():
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 15
    for s in syms:
        assert hasattr(L, s), s


def test_library_built_from_these_sources(tmp_path):
    """provenance: the loaded library embeds the digest of exactly the sources beside it, and the
    loader refuses a library whose embedded digest differs"""
    info = _lib.lib().ppr_build_info().decode()
    assert f"ppr_src_sha256={_lib.source_digest()}" in info and "arch=gfx950" in info
    assert _lib.embedded_digest(_lib.LIB_PATH) == _lib.source_digest()
    other = tmp_path / "csrc"
    other.mkdir()
    for f in _lib.CSRC_SOURCES:  # the same tree with one edited source has another digest
        txt = open(os.path.join(_lib.CSRC, f)).read()
        (other / f).write_text(txt + ("\n// edited\n" if f == "grank.hip" else ""))
    assert _lib.source_digest(str(other)) != _lib.source_digest()


def test_strerror_messages_match_reference():
    L = _lib.lib()
    # include/grank.h:51-55, header-only/grankMulti.h:304
    for code, msg in [(2, "K must be positive"), (3, "L must be positive"), (4, "K must be <= L"),
                      (5, "iterations must be positive"), (6, "damping must be [0,1]"),
                      (7, "nThreads must be positive")]:
        assert L.ppr_strerror(code).decode() == msg
        assert _lib.ERRORS[code] == msg


@pytest.mark.parametrize("args,msg", [((0, 3, 42, 0.5, 1e-4), "K must be positive"),
                                      ((2, 0, 32, 0.85, 1e-4), "L must be positive"),
                                      ((2, 1, 10, 0.5, 1e-4), "K must be <= L"),
                                      ((2, 2, 0, 0.5, 1e-4), "iterations must be positive"),
                                      ((2, 2, 10, 1.5, 1e-4), r"damping must be \[0,1\]"),
                                      ((2, 2, 10, -1.5, 1e-4), r"damping must be \[0,1\]")])
def test_bad_parameters(args, msg):
    # test/grankTest.cc:20-29 (validation happens before any device work)
    with pytest.raises(ppr.PprError, match=msg):
        ppr.grank({}, *args)
    with pytest.raises(ppr.PprError, match="nThreads must be positive"):
        ppr.grank_multi({}, 2, 2, 10, 0.5, 1e-4, 0)


def test_abi_param_validation_without_device():
    L = _lib.lib()
    c = _lib.PprCsr(0, None, None)
    out = ctypes.c_void_p()
    assert L.ppr_grank_plan_create(ctypes.byref(c), None, 0, 3, 0.85, None, ctypes.byref(out)) == 2
    assert L.ppr_grank_plan_create(ctypes.byref(c), None, 4, 3, 0.85, None, ctypes.byref(out)) == 4
    assert L.ppr_grank_csr(ctypes.byref(c), None, 2, 2, 0, 0.85, 0.0, None, None, None, None, None) == 5
    # empty graph: nothing to do, no device needed
    assert L.ppr_grank_csr(ctypes.byref(c), None, 2, 2, 3, 0.85, 0.0, None, None, None, None, None) == 0


@pytest.mark.parametrize("name", all_names())
def test_product_partitions_match_reference(name):
    f = load(name)
    assert np.array_equal(ppr.Csr(f["rp"], f["col"]).partitions(), f["part"])


def test_rmat_shape_and_determinism():
    g1 = ppr.rmat(12, seed=42)
    g2 = ppr.rmat(12, seed=42)
    assert np.array_equal(g1.row_ptr, g2.row_ptr) and np.array_equal(g1.col, g2.col)
    assert g1.n == 4096 and 0.75 * 16 * 4096 < g1.m <= 16 * 4096
    for v in range(0, g1.n, 97):  # successors ascending and unique
        s = g1.col[g1.row_ptr[v]:g1.row_ptr[v + 1]]
        assert np.all(np.diff(s) > 0)
    assert not np.array_equal(ppr.rmat(12, seed=43).col[:100], g1.col[:100])


def test_execution_order_is_permutation():
    g = ppr.rmat(11, seed=1)
    o = g.execution_order()
    assert np.array_equal(np.sort(o), np.arange(g.n))


def test_from_dict_rejects_unknown_successor():
    with pytest.raises(ppr.PprError):
        ppr.Csr.from_dict({0: [1]})


def test_import_edge_csv_semantics(tmp_path):
    # src/main.cc:78-112: targets inserted, repeated edges kept once, successor order kept, \r dropped
    p = tmp_path / "g.csv"
    p.write_bytes(b"1,2\r\n1,3\n2,1\n1,2\n4,4\n3,5\n")
    g = ppr.import_edge_csv(str(p))
    succ = {g.key(i): [g.key(int(c)) for c in g.col[g.row_ptr[i]:g.row_ptr[i + 1]]] for i in range(g.n)}
    assert succ == {1: [2, 3], 2: [1], 3: [5], 4: [4], 5: []}
    assert g.m == 5


@pytest.mark.skipif(not os.path.exists("/root/reference/example.txt"), reason="reference tree absent")
def test_import_edge_csv_reference_order_eat():
    # the reference's own iteration order of example.txt (recorded in the g4 fixture by ref_driver)
    g = ppr.import_edge_csv("/root/reference/example.txt")
    f = load("g4_eat_k50_l100")
    assert np.array_equal(np.array(g.keys), f["z"]["order"])
    assert np.array_equal(g.row_ptr, f["rp"]) and np.array_equal(g.col, f["col"])


def test_plan_rejects_candidate_count_overflow():
    """a source whose candidate count could pass 2^31 - 1 (out-degree * L + 1) is refused at plan
    creation (the device keeps per-source counts and staging offsets in 32 bits), before any
    device call"""
    L = _lib.lib()
    deg = 1 << 19                    # 2^19 * 4096 + 1 > INT32_MAX
    n = deg + 1
    rp = np.zeros(n + 1, dtype=np.int64)
    rp[1:] = deg                     # node 0 -> every other node
    col = np.arange(1, n, dtype=np.int32)
    part = np.zeros(n, dtype=np.uint8)
    part[1:] = 1
    c = _lib.csr_struct(rp, col)
    out = ctypes.c_void_p()
    assert L.ppr_grank_plan_create(ctypes.byref(c), _lib.ptr(part), 2, 4096, 0.85, None, ctypes.byref(out)) == 11
    assert L.ppr_mccp2_plan_create(ctypes.byref(c), 2, 4096, 0.85, None, ctypes.byref(out)) == 11


def test_bench_parses_timing_lines():
    """bench.py's end_to_end leg reads the PPR_TIMING split off the drop-in program's stderr"""
    import importlib
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    bench = importlib.import_module("bench")
    txt = ("noise\nppr_timing plan_create partitions_s 0.786 colx_s 0.050 alloc_upload_s 0.142 work_s 0.051\n"
           "ppr_timing flatten_s 1.17 csr_call_s 4.82 device_s 3.56 materialize_s 2.81\n")
    d = bench.parse_ppr_timing(txt)
    assert d["partitions_s"] == 0.786 and d["work_s"] == 0.051
    assert d["flatten_s"] == 1.17 and d["csr_call_s"] == 4.82 and d["materialize_s"] == 2.81
    assert bench.parse_ppr_timing("") == {}


def test_bench_traffic_summary_names_its_build():
    """roofline.traffic comes from a committed PMC summary stamped with the source digest of the
    library it profiled (tools/stamp_build.py), which the bench line sets beside its own build"""
    import importlib
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    traffic, src, build = bench.pmc_traffic("grank_rmat22_k64_l128", "exact")
    assert traffic and traffic > 0 and src.startswith("profiles/")
    assert build and len(build) == 64 and all(c in "0123456789abcdef" for c in build)


def _path_csr(n, reverse=False):
    """a directed path 0 -> 1 -> ... -> n-1 (or n-1 -> ... -> 0), one successor per node"""
    rp = np.zeros(n + 1, dtype=np.int64)
    if reverse:
        rp[2:] = np.arange(1, n)
        col = np.arange(0, n - 1, dtype=np.int32)
    else:
        rp[1:n] = np.arange(1, n)
        rp[n] = n - 1
        col = np.arange(1, n, dtype=np.int32)
    return ppr.Csr(rp, col)


@pytest.mark.parametrize("reverse", [False, True])
def test_partitions_long_path_linear_time(reverse):
    """the out-edge BFS scanned every unvisited node at every level, O(depth x n)
    -- a 200 K-node path took minutes. Past 2 (n + m) of scanning it now switches to predecessor
    lists. Partitions = the reference BFS's (oracle restatement of pprInternal.h:29-99): alternate
    along the path from node 0, whichever way the edges point."""
    import time
    import oracle
    n = 200_000
    g = _path_csr(n, reverse)
    t0 = time.time()
    part = g.partitions()
    assert time.time() - t0 < 10.0
    assert np.array_equal(part, (np.arange(n) & 1).astype(np.uint8))
    small = _path_csr(5000, reverse)
    assert np.array_equal(small.partitions(), oracle.find_partitions(small.row_ptr, small.col))


@pytest.mark.parametrize("name", ["g3_rmat12_k16_l32", "g3_rmat14_k32_l64", "g4_eat_k50_l100"])
def test_partitions_transposed_mode_match_reference(name, monkeypatch):
    """the predecessor-list levels (forced from level 0) give the reference's partitions too"""
    monkeypatch.setenv("PPR_BFS_TRANSPOSE", "1")
    f = load(name)
    assert np.array_equal(ppr.Csr(f["rp"], f["col"]).partitions(), f["part"])


def test_basket_width_limit_refused_without_device():
    """L above MAX_L = 4096 (csrc/ppr_common.h) is refused with PPR_ERR_RANGE
    (11) before any device work, by GRank and by MCCompletePathV2 (the reference merges any L,
    include/grank.h:42-48; INTEGRATION.md "Limits"); L = 4096 passes the checks (run on the GPU:
    tests/test_gpu_parity.py::test_gpu_widest_basket_limit)"""
    L = _lib.lib()
    rp = np.array([0, 1], dtype=np.int64)
    col = np.array([0], dtype=np.int32)
    c = _lib.csr_struct(rp, col)
    out = ctypes.c_void_p()
    assert L.ppr_grank_plan_create(ctypes.byref(c), None, 1, 4097, 0.85, None, ctypes.byref(out)) == 11
    assert L.ppr_mccp2_plan_create(ctypes.byref(c), 1, 4097, 0.85, None, ctypes.byref(out)) == 11
    assert L.ppr_grank_csr(ctypes.byref(c), None, 1, 4097, 2, 0.85, -1.0, None, None, None, None, None) == 11
    assert "outside the supported range" in _lib.lib().ppr_strerror(11).decode()
