"""Per-iteration wall time of one GRank job on the bench workload (diagnostics).

    python tools/iter_profile.py [--scale 22] [--K 64] [--L 128] [--iters 30] [--jobs 2]

Runs `jobs` whole jobs through the step-level API (init, iterate, read_maxdiff per iteration) and
prints the last job's per-iteration milliseconds (host-timed around a synchronising maxDiff read)
and the merge-phase total; tuning variables (PPR_*) come from the environment.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import approximated_personalized_pagerank_amd as ppr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--jobs", type=int, default=2)
    ap.add_argument("--seed", type=int, default=42)
    args = ap.parse_args()
    g = ppr.rmat(args.scale, seed=args.seed)
    plan = ppr.GrankPlan(g, args.K, args.L, 0.85, device=0, stats=True)
    for j in range(args.jobs):
        t0 = time.perf_counter()
        plan.init()
        plan.read_maxdiff(0)
        ti = time.perf_counter()
        per = []
        for it in range(args.iters):
            a = time.perf_counter()
            plan.iterate(it, 0, plan.active_count(it))
            plan.read_maxdiff(it)
            per.append((time.perf_counter() - a) * 1e3)
        plan.finish(args.iters)
        plan.fetch()
        tot = time.perf_counter() - t0
        print(f"job {j}: {tot * 1e3:.0f} ms (init {1e3 * (ti - t0):.0f}) iterations: "
              + " ".join(f"{x:.0f}" for x in per), flush=True)


if __name__ == "__main__":
    main()
