"""Exact-sum path debugging: one config under several planning variants, mismatch counts vs the oracle."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

VARIANTS = [
    {}, {"PPR_XR_DSCALE": "1000"}, {"PPR_XR_RMAX": "64"}, {"PPR_XR_RMAX": "64", "PPR_XR_DSCALE": "1000"},
    {"PPR_XR_RMAX": "1", "PPR_XR_DSCALE": "1000"}, {"PPR_HUB_STREAMS": "1"}, {"PPR_TIER_MASK": "0x0"},
    {"PPR_XR_DSCALE": "1000", "PPR_TIER_MASK": "0x0"},
]


def one(scale, K, L, it, seed):
    import approximated_personalized_pagerank_amd as ppr
    import oracle
    g = ppr.rmat(scale, seed=seed)
    part = g.partitions()
    r = ppr.grank_csr(g, K, L, it, 0.85, -1.0, part=part, device=0)
    o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0)
    bad = np.nonzero((r.ids != o["ids"]).any(1) | (r.scores != o["scores"]).any(1) | (r.lens != o["lens"]))[0]
    md = np.array_equal(r.max_diff, o["max_diff"])
    deg = np.diff(g.row_ptr)
    info = [(int(v), int(deg[v]), int(r.lens[v]), int(o["lens"][v]),
             int((r.ids[v] != o["ids"][v]).sum()), float(np.abs(r.scores[v] - o["scores"][v]).max())) for v in bad[:6]]
    print(f"  maxdiff_equal {md} bad_rows {len(bad)} sample (v, deg, len_gpu, len_or, ids_diff, max|ds|) {info}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1:
        one(*[int(x) for x in sys.argv[1:]])
        sys.exit(0)
    for cfg in [(13, 32, 128, 4, 104), (13, 32, 128, 1, 104), (13, 32, 128, 2, 104)]:
        for v in VARIANTS:
            env = dict(os.environ, PPR_TIMING="1", **v)
            print(cfg, v, flush=True)
            p = subprocess.run([sys.executable, __file__] + [str(x) for x in cfg], env=env, capture_output=True,
                               text=True, timeout=300)
            print(p.stdout.strip())
            print("  " + " | ".join(l for l in p.stderr.splitlines() if "redo" in l or "Error" in l or "error" in l))
