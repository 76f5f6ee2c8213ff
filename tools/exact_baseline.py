"""f3 baseline: the reference's exact single-source PPR (pprSingleSource(g, 100, .85, 1e-4),
include/internal/pprSingleSource.h:28-75, compiled from /root/reference into oracle/_ref/ref_driver;
single-threaded by design) for a few sources of RMAT-<scale>, next to the engine's batched exact PPR
(ExactPPR) for --sources sources on one MI355X.

    python tools/exact_baseline.py [--scale 22] [--ref-sources 4] [--sources 200]
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import approximated_personalized_pagerank_amd as ppr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--ref-sources", type=int, default=4)
    ap.add_argument("--sources", type=int, default=200)
    a = ap.parse_args()
    g = ppr.rmat(a.scale, seed=42)
    deg = g.degrees()
    rng = np.random.default_rng(7)
    src = np.sort(rng.choice(np.nonzero(deg > 0)[0], a.sources, replace=False)).astype(np.int32)
    t = time.perf_counter()
    ex = ppr.ExactPPR(g, src, 0.85, device=0)
    its = ex.run(100, 1e-4)
    ex.topk(64)
    ex.close()
    gpu_s = time.perf_counter() - t
    out = {"graph": f"RMAT-{a.scale}: {g.n} nodes, {g.m} edges",
           "engine": {"sources": a.sources, "wall_s": gpu_s, "per_source_ms": 1e3 * gpu_s / a.sources,
                      "iterations_mean": float(its.mean()), "includes": "transposed CSR upload, run, top-64"}}
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    if os.path.exists(drv):
        with tempfile.TemporaryDirectory() as td:
            gp = os.path.join(td, "g.bin")
            with open(gp, "wb") as f:
                np.array([g.n, g.m], dtype=np.int64).tofile(f)
                np.arange(g.n, dtype=np.int32).tofile(f)
                g.row_ptr.astype(np.int64).tofile(f)
                g.col.astype(np.int32).tofile(f)
            lp = os.path.join(td, "l.bin")
            # dense indices of the reference's own iteration order: any non-dangling-heavy sample
            np.arange(0, a.ref_sources * 997, 997, dtype=np.int32).tofile(lp)
            p = subprocess.run([drv, "pprss_list", gp, os.path.join(td, "o.bin"), "1", "1", "100", "0.85", "0.0001",
                                "1", lp], capture_output=True, text=True, check=True)
            ms = float(re.search(r"([0-9.]+) ms", p.stderr.strip().splitlines()[-1]).group(1))
        out["reference"] = {"sources": a.ref_sources, "ms": ms, "per_source_ms": ms / a.ref_sources, "threads": 1,
                            "note": "pprSingleSource only (graph loading excluded); sources spread over the "
                                    "reference's iteration order"}
        out["speedup_per_source"] = out["reference"]["per_source_ms"] / out["engine"]["per_source_ms"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
