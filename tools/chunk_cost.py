"""Cost of splitting an iteration's merge into sub-ranges (the sharded loop's chunked, overlapped
exchange merges each rank's range in C chunks): one RMAT-22 job with every iteration merged as S
consecutive sub-ranges, for several S. At N ranks with C chunks a rank merges S = N * C pieces'
worth of ranges per iteration.

    python tools/chunk_cost.py [--splits 1 8 16 32]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--splits", type=int, nargs="+", default=[1, 8, 16, 32])
    args = ap.parse_args()
    import approximated_personalized_pagerank_amd as ppr
    g = ppr.rmat(args.scale, seed=42)
    plan = ppr.GrankPlan(g, 64, 128, 0.85, part=g.partitions(), device=0)
    w = [None, None]
    for S in [args.splits[0]] + args.splits:  # first entry twice: warm-up
        t = time.perf_counter()
        plan.init()
        for it in range(30):
            n = plan.active_count(it)
            for k in range(S):
                plan.iterate(it, n * k // S, n * (k + 1) // S)
        plan.read_maxdiff(29)
        plan.finish(30)
        print(f"splits {S}: {time.perf_counter() - t:.3f} s per job", flush=True)
    plan.close()


if __name__ == "__main__":
    main()
