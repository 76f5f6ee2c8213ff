"""Quality of the engine vs exact PPR at benchmark scale: GRank (or
MCCompletePathV2, --algo mc) on RMAT-<scale> on the GPU, then the reference harness's measure
(benchmarkAlgorithm: top-K Jaccard and Kendall against pprSingleSource(g, 100, .85, 1e-4) of sampled
non-dangling sources) with the exact PPR batched on the GPU.

    python tools/quality_rmat.py [--algo grank|mc] [--scale 22] [--K 64] [--L 128] [--iters 30] [--sources 200]
      (mc: --iters = random walks per node R; C5 = --algo mc --K 50 --L 200 --iters 1000)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import approximated_personalized_pagerank_amd as ppr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--sources", type=int, default=200)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--algo", choices=["grank", "mc"], default="grank")
    a = ap.parse_args()
    t0 = time.time()
    g = ppr.rmat(a.scale, seed=a.seed)
    if a.algo == "mc":
        r = ppr.mccp2_csr(g, a.K, a.L, a.iters, 0.85, seed=20261016, device=0)
    else:
        r = ppr.grank_csr(g, a.K, a.L, a.iters, 0.85, -1.0, part=g.partitions(), device=0)
    t1 = time.time()
    deg = g.degrees()
    rng = np.random.default_rng(2026)
    src = np.sort(rng.choice(np.nonzero(deg > 0)[0], a.sources, replace=False)).astype(np.int32)
    ex = ppr.ExactPPR(g, src, 0.85, device=0)
    its = ex.run(100, 1e-4)
    t2 = time.time()
    eids, esc, eln = ex.topk(a.K)
    qk = np.full((len(src), a.K), -1, dtype=np.int32)
    for i, v in enumerate(src):
        qk[i, :r.lens[v]] = r.ids[v, :r.lens[v]]
    at = ex.gather(qk)
    ex.close()
    js, ks = [], []
    for i, v in enumerate(src):
        m = int(r.lens[v])
        js.append(ppr.jaccard(r.ids[v, :m].tolist(), eids[i, :min(m, eln[i])].tolist()))
        ks.append(ppr.kendall_correlation(r.scores[v, :m], at[i, :m]))
    what = f"mccompletepathv2 RMAT-{a.scale} K={a.K} L={a.L} R={a.iters}" if a.algo == "mc" else \
        f"grank RMAT-{a.scale} K={a.K} L={a.L} iters={a.iters}"
    out = {"config": what, "sources": len(src),
           "jaccard_average": float(np.mean(js)), "jaccard_min": float(np.min(js)),
           "kendall_average": float(np.mean(ks)), "kendall_min": float(np.min(ks)),
           "exact_ppr_iterations_mean": float(its.mean()), "engine_s": round(t1 - t0, 1),
           "exact_ppr_s": round(t2 - t1, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
