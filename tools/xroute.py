#!/usr/bin/env python3
"""Exchange volume of the source-sharded GRank loop with consumer routing vs the all-to-all
broadcast (a model; host only).

Each rank merges fixed work-balanced ranges of the two partitions' active lists (the bounds of
ppr_grank_plan_shard_bounds: work = 1 + sum over successors of min(L, deg(u) + 1)). Rank q only ever
reads the rows of its own sources' successors C_q, so a row u written by rank r must reach rank q
only if u is in C_q. Rows are priced at their full compact size (8 + 12 L bytes; active rows are
nearly all full at L = 128, profiles/r02_exchange_bytes_rmat22_k64_l128.json).

    python tools/xroute.py [--scale 22] [--L 128] [--iters 30] [--worlds 2 4 8]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def shard_bounds(w, world):
    tot = w.sum()
    cw = np.cumsum(w)
    b = [0]
    for r in range(1, world):
        # largest i with cw[i-1] <= target (the native loop's greedy walk)
        b.append(int(np.searchsorted(cw, tot * r / world, side="right")))
    b.append(len(w))
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--worlds", type=int, nargs="+", default=[2, 4, 8])
    args = ap.parse_args()
    import approximated_personalized_pagerank_amd as ppr
    g = ppr.rmat(args.scale, seed=42)
    part = g.partitions()
    rp, col = g.row_ptr, g.col.astype(np.int64)
    deg = np.diff(rp)
    n = g.n
    L = args.L
    src_of_edge = np.repeat(np.arange(n, dtype=np.int64), deg)
    lim = np.minimum(L, deg + 1).astype(np.float64)
    work = 1.0 + np.bincount(src_of_edge, weights=lim[col], minlength=n)
    act = [np.nonzero((part == q) & (deg > 0))[0] for q in (0, 1)]
    row_bytes = 8 + 12 * L
    out = {"workload": f"grank RMAT-{args.scale} L={L} iters={args.iters}", "row_bytes": row_bytes, "worlds": {}}
    its = {0: (args.iters + 1) // 2, 1: args.iters // 2}
    for world in args.worlds:
        owner = [np.full(n, -1, dtype=np.int64) for _ in (0, 1)]
        for q in (0, 1):
            b = shard_bounds(work[act[q]], world)
            for r in range(world):
                owner[q][act[q][b[r]:b[r + 1]]] = r
        # consumer mask: bit q of node u = some source of rank q (either partition) reads u
        mask = np.zeros(n, dtype=np.int64)
        for q in (0, 1):
            o = owner[q][src_of_edge]
            ok = o >= 0
            np.bitwise_or.at(mask, col[ok], (1 << o[ok]))
        recv_b = np.zeros(world)
        recv_r = np.zeros(world)
        for q in (0, 1):
            for r in range(world):
                mine = act[q][owner[q][act[q]] == r]
                m = mask[mine]
                for d in range(world):
                    if d == r:
                        continue
                    k = int(((m >> d) & 1).sum())
                    recv_r[d] += k * its[q]
                    recv_b[d] += len(mine) * its[q]
        out["worlds"][world] = {
            "broadcast_bytes_per_rank_max": float(recv_b.max() * row_bytes),
            "routed_bytes_per_rank_max": float(recv_r.max() * row_bytes),
            "routed_bytes_per_rank": [float(x * row_bytes) for x in recv_r],
            "cut": float(recv_b.max() / max(recv_r.max(), 1)),
        }
        print(f"world {world}: max received per job broadcast {recv_b.max() * row_bytes / 1e9:.1f} GB, "
              f"routed {recv_r.max() * row_bytes / 1e9:.1f} GB ({recv_b.max() / max(recv_r.max(), 1):.2f}x less)",
              file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
