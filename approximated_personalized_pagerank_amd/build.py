"""In-tree build of libppr_hip.so for gfx950 (hipcc, no JIT cache, no torch extension)."""
from __future__ import annotations

import os
import re
import subprocess
import sys

from ._lib import CSRC, CSRC_HEADERS as HEADERS, CSRC_SOURCES as SOURCES, LIB_PATH, PKG_DIR, embedded_digest, \
    source_digest

ARCH = os.environ.get("PPR_OFFLOAD_ARCH", "gfx950")


def _stale() -> bool:
    # by content, not mtime: the library must embed the digest of exactly these sources
    return embedded_digest(LIB_PATH) != source_digest()


def build(force: bool = False, verbose: bool = False, out: str | None = None, defines=(),
          csrc: str | None = None) -> str:
    """Compile the library (only when a source is newer than it, unless `force`). `out`,
    `defines` (-D flags) and `csrc` (another source tree) build an experiment variant beside it
    (tools/build_variant.py)."""
    out = out or LIB_PATH
    src_dir = csrc or CSRC
    # a variant loaded for an A/B (PPR_LIB_VARIANT: LIB_PATH is the variant) is prebuilt by
    # tools/build_variant.py with its own defines or sources: never rebuild it from these sources
    # without them (that silently turned variant A/Bs into product-vs-product runs)
    if out == LIB_PATH and os.environ.get("PPR_LIB_VARIANT") and not force:
        return LIB_PATH
    if out == LIB_PATH and not force and not _stale():
        return LIB_PATH
    hipcc = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
    digest = source_digest(src_dir)
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-Wno-unused-value", f'-DPPR_SRC_SHA256="{digest}"',
           f'-DPPR_OFFLOAD_ARCH="{ARCH}"'] + [f"-D{d}" for d in defines] + [
           "-I", os.path.join(PKG_DIR, "..", "include"),
           "-o", out + ".tmp"] + [os.path.join(src_dir, s) for s in SOURCES
                                  # an older revision (tools/build_variant.py --rev) may predate a source
                                  if csrc is None or os.path.exists(os.path.join(src_dir, s))] + ["-lrccl", "-lpthread"]
    cmd.append("-Rpass-analysis=kernel-resource-usage")
    if verbose:
        print(" ".join(cmd))
    r = subprocess.run(cmd, stderr=subprocess.PIPE, text=True)
    if r.returncode != 0:
        print(r.stderr, file=sys.stderr)
        raise subprocess.CalledProcessError(r.returncode, cmd)
    if not any(str(d).startswith("PPR_PHASE_TIMING") for d in defines):  # (diagnostic variants keep counters in scratch)
        try:
            check_resources(r.stderr)
        except RuntimeError:
            os.remove(out + ".tmp")  # (the library in place stays the last accepted build)
            raise
    os.replace(out + ".tmp", out)
    return out


def check_resources(remarks: str) -> None:
    """every kernel of the library keeps its state in registers and LDS: private (scratch) memory
    per lane or register spills would turn into HBM traffic on every wave (an indexable per-lane
    array cost 3 TB of scratch writes per RMAT-22 job once) -- refuse such a build"""
    bad, fn = [], None
    for ln in remarks.splitlines():
        if "remark:" not in ln:
            continue
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            fn = m.group(1)
            continue
        if "/rocprim/" in ln or "/hipcub/" in ln:
            continue
        m = re.search(r"(ScratchSize \[bytes/lane\]|VGPRs Spill): (\d+)", ln)  # (SGPR spills go to VGPR lanes)
        if m and int(m.group(2)) > 0:
            bad.append(f"{fn}: {m.group(1)} {m.group(2)}")
    if bad:
        raise RuntimeError("kernels with scratch memory or register spills:\n  " + "\n  ".join(bad))


DROPIN_SRC = os.path.join(PKG_DIR, "..", "tests", "cpp", "dropin_test.cc")
DROPIN_BIN = os.path.join(PKG_DIR, "..", "tests", "cpp", "_dropin_test")


def build_dropin(force: bool = False) -> str:
    """g++ the reference-API program tests/cpp/dropin_test.cc (include/ppr/*.h over libppr_hip.so):
    the C++ drop-in tests and bench.py's end_to_end leg run it."""
    lib = build()
    inc = os.path.join(PKG_DIR, "..", "include")
    deps = [DROPIN_SRC, lib] + [os.path.join(inc, "ppr", f) for f in os.listdir(os.path.join(inc, "ppr"))]
    if (not force and os.path.exists(DROPIN_BIN)
            and os.path.getmtime(DROPIN_BIN) > max(os.path.getmtime(d) for d in deps)):
        return DROPIN_BIN
    subprocess.run(["g++", "-std=c++11", "-O2", "-I", inc, DROPIN_SRC, "-o", DROPIN_BIN + ".tmp", "-pthread",
                    "-L", PKG_DIR, "-lppr_hip", f"-Wl,-rpath,{PKG_DIR}"], check=True)
    os.replace(DROPIN_BIN + ".tmp", DROPIN_BIN)
    return DROPIN_BIN


HOST_ASAN_SRC = os.path.join(PKG_DIR, "..", "tests", "cpp", "host_asan_test.cc")
HOST_ASAN_BIN = os.path.join(PKG_DIR, "..", "tests", "cpp", "_host_asan_test")


def build_host_asan(force: bool = False) -> str:
    """The engine's host code (csrc/host_graph.cpp and include/ppr/grank.h's flatten / KeyIndex /
    materialisation) under g++ -fsanitize=address,undefined, driven by tests/cpp/host_asan_test.cc
    (SURVEY.md s5). The sanitized host_graph.cpp symbols interpose over the library's copies;
    libppr_hip.so supplies only ppr_strerror. No device code is involved."""
    lib = build()
    inc = os.path.join(PKG_DIR, "..", "include")
    hg = os.path.join(CSRC, "host_graph.cpp")
    deps = [HOST_ASAN_SRC, hg, lib, os.path.join(inc, "ppr", "grank.h"), os.path.join(CSRC, "host_par.h")]
    if (not force and os.path.exists(HOST_ASAN_BIN)
            and os.path.getmtime(HOST_ASAN_BIN) > max(os.path.getmtime(d) for d in deps)):
        return HOST_ASAN_BIN
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                    "-fno-sanitize-recover=undefined", "-I", inc, HOST_ASAN_SRC, hg, "-o", HOST_ASAN_BIN + ".tmp",
                    "-pthread", "-L", PKG_DIR, "-lppr_hip", f"-Wl,-rpath,{PKG_DIR}"], check=True)
    os.replace(HOST_ASAN_BIN + ".tmp", HOST_ASAN_BIN)
    return HOST_ASAN_BIN
