"""Exchange volume of source sharding at a workload: per iteration, the compact block bytes of the
whole active list (what the ranks of an N-GPU run receive in total, summed over senders, before the
(N-1)/N share) against the fixed-size row format of round 1 (8 + 4 Le + 8 L + 8 + 128 bytes a row).

    python tools/xbytes.py [--scale 22] [--K 64] [--L 128] [--iters 30] > profiles/<round>_exchange_bytes.json
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--seed", type=int, default=42)
    args = ap.parse_args()
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import GpuEngine
    g = ppr.rmat(args.scale, seed=args.seed)
    plan = ppr.GrankPlan(g, args.K, args.L, 0.85, part=g.partitions(), device=0)
    eng = GpuEngine(plan)
    Le = (args.L + 1) & ~1
    fixed_row = 8 + 4 * Le + 8 * args.L + 8 + 128
    plan.init()
    rows = []
    t0 = time.time()
    for it in range(args.iters):
        n = plan.active_count(it)
        plan.iterate(it, 0, n)
        blk = len(eng.pack(it, 0, n))
        rows.append({"iteration": it, "active_rows": n, "compact_bytes": blk, "fixed_bytes": n * fixed_row})
        print(f"it {it}: {n} rows, compact {blk / 1e9:.3f} GB, fixed {n * fixed_row / 1e9:.3f} GB "
              f"({time.time() - t0:.0f}s)", file=sys.stderr, flush=True)
    plan.close()
    tc = sum(r["compact_bytes"] for r in rows)
    tf = sum(r["fixed_bytes"] for r in rows)
    print(json.dumps({"workload": f"grank RMAT-{args.scale} K={args.K} L={args.L} iters={args.iters}",
                      "fixed_row_bytes": fixed_row, "compact_bytes_per_job": tc, "fixed_bytes_per_job": tf,
                      "ratio": tc / tf, "mean_compact_row_bytes": tc / max(1, sum(r["active_rows"] for r in rows)),
                      "per_iteration": rows}, indent=1))


if __name__ == "__main__":
    main()
