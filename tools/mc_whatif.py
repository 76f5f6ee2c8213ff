"""Same-process A/B of plan environment variants for MCCompletePathV2 (walks + combine) on RMAT.

    python tools/mc_whatif.py [--scale 22] [--reps 2] "A=1 B=2" "A=3" ...

The graph is built once; each variant sets its environment (read at plan creation), creates an
MccpPlan, runs one untimed job and `reps` timed jobs, and prints walk / combine ms per job.
An empty string is the default configuration.
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
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--L", type=int, default=200)
    ap.add_argument("--walks", type=int, default=1000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("variants", nargs="*")
    a = ap.parse_args()
    t0 = time.time()
    g = ppr.rmat(a.scale, seed=42)
    print(f"RMAT-{a.scale} ready in {time.time() - t0:.1f} s", flush=True)
    for var in (a.variants or [""]):
        kv = dict(x.split("=", 1) for x in var.split())
        old = {k: os.environ.get(k) for k in kv}
        os.environ.update(kv)
        try:
            plan = ppr.MccpPlan(g, a.K, a.L, 0.85, device=0)
            plan.run(a.walks, 1)
            walk, comb, tot = [], [], []
            for r in range(a.reps):
                t = time.perf_counter()
                st = plan.run(a.walks, 2 + r)
                tot.append((time.perf_counter() - t) * 1e3)
                walk.append(st.walk_ms)
                comb.append(st.combine_ms)
            plan.close()
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        print(json.dumps({"variant": var or "default", "ms_per_job": min(tot), "walk_ms": min(walk),
                          "combine_ms": min(comb), "all_combine_ms": comb}), flush=True)


if __name__ == "__main__":
    main()
