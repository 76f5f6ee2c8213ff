"""Golden digests for the full-size GPU checks (tests/test_gpu_scale.py), computed here by the
CPU oracle (oracle/grank_oracle.c): C2 = RMAT-18 K32/L64/20 iterations (BASELINE.json configs[1]).
The whole result is too large to commit; its SHA-256 digests are bit-exact targets.

    python tools/make_scale_digests.py [exact|chain]
        -> tests/golden/c2_rmat18_k32_l64_i20.json (chain), c2_rmat18_k32_l64_i20_exact.json (exact)
"""
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import approximated_personalized_pagerank_amd as ppr  # noqa: E402
import oracle  # noqa: E402


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "chain"
    oracle.set_sum(mode)
    scale, K, L, it, d, tol, seed = 18, 32, 64, 20, 0.85, -1.0, 42
    g = ppr.rmat(scale, seed=seed)
    part = g.partitions()
    t = time.time()
    o = oracle.grank(g.row_ptr, g.col, part, K, L, it, d, tol)
    out = {"config": f"RMAT-{scale} seed {seed} K={K} L={L} iterations={it} damping={d} tol={tol}",
           "scale": scale, "seed": seed, "K": K, "L": L, "iters": it, "damping": d, "tol": tol,
           "n": int(g.n), "m": int(g.m), "graph_sha256": digest(g.col),
           "iterations_run": int(o["iterations_run"]),
           "max_diff": [float(x).hex() for x in o["max_diff"]],
           "ids_sha256": digest(o["ids"]), "scores_sha256": digest(o["scores"]), "lens_sha256": digest(o["lens"]),
           "oracle_seconds": round(time.time() - t, 1), "sum": mode}
    path = os.path.join(ROOT, "tests", "golden", "c2_rmat18_k32_l64_i20" + ("_exact" if mode == "exact" else "") + ".json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(path, out["oracle_seconds"], "s")


if __name__ == "__main__":
    main()
