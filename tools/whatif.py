"""Same-process A/B of plan environment variants on one RMAT graph (GRank, device phase only).

    python tools/whatif.py [--scale 22] [--reps 2] "A=1 B=2" "A=3" ...

The graph and its partitions are built once; each variant sets its environment (read by
ppr_grank_plan_create), creates a plan, runs one untimed job and `reps` timed jobs, and prints
ms per job (and the merge-phase ms). An empty string is the default configuration. PPR_WHATIF
variants (plan.h) give wrong results on purpose: they time what a pipeline stage costs.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import approximated_personalized_pagerank_amd as ppr  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    t0 = time.time()
    g = ppr.rmat(a.scale, seed=42)
    part = g.partitions()
    print(f"RMAT-{a.scale} ready in {time.time() - t0:.1f} s", flush=True)
    rows = []
    for var in (a.variants or [""]):
        kv = dict(x.split("=", 1) for x in var.split())
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        try:
            plan = ppr.GrankPlan(g, a.K, a.L, 0.85, part=part, device=0, stats=True)
            plan.run(a.iters, -1.0)
            ms, mg = [], []
            for _ in range(a.reps):
                t = time.perf_counter()
                st = plan.run(a.iters, -1.0)
                ms.append((time.perf_counter() - t) * 1e3)
                mg.append(st.merge_ms)
            plan.close()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        r = {"variant": var or "default", "ms_per_job": min(ms), "merge_ms": min(mg), "all_ms": ms}
        rows.append(r)
        print(json.dumps(r), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
