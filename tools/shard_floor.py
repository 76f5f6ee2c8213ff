"""Strong-scaling compute floor of the source-sharded GRank loop, measured on ONE GPU.

    python tools/shard_floor.py [--scale 22] [--worlds 1 2 4 8] [--out profiles/r03_shard_floor.json]

For every world size w, one full job (init + 30 iterations, K64/L128) runs on one plan, but each
iteration's active list is merged as the w work-balanced ranges ppr_grank_plan_shard_bounds hands
the ranks of a w-GPU run (header-only/grankMulti.h:376-396 splits the sources the same way), one
range after another, each timed alone (host wall clock around ppr_grank_plan_iterate + a stream
sync). The rows are those of the real job, so per iteration max over ranges = what the slowest
rank of a w-GPU run merges; the sum over iterations of that maximum is the job's compute floor on
w GPUs (the exchange and the collectives come on top, and are reported separately as the block
bytes every rank receives per iteration). No multi-GPU run is made: this is a model input.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import approximated_personalized_pagerank_amd as ppr  # noqa: E402
from approximated_personalized_pagerank_amd import _lib  # noqa: E402


def bounds(plan, it, w):
    b = np.zeros(w + 1, dtype=np.int64)
    _lib.check(_lib.lib().ppr_grank_plan_shard_bounds(plan._p, it, w, b.ctypes.data), "shard_bounds")
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--worlds", type=int, nargs="*", default=[1, 2, 4, 8])
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    g = ppr.rmat(a.scale, seed=42)
    part = g.partitions()
    plan = ppr.GrankPlan(g, a.K, a.L, 0.85, part=part, device=0)
    rb = ctypes.c_int64()
    _lib.check(_lib.lib().ppr_grank_plan_row_bytes(plan._p, ctypes.byref(rb)), "row_bytes")
    plan.run(a.iters, -1.0)  # warm-up job
    res = {"workload": f"grank RMAT-{a.scale} K={a.K} L={a.L} iters={a.iters}", "row_bytes_bound": rb.value,
           "worlds": {}}
    for w in a.worlds:
        t0 = time.perf_counter()
        plan.init()
        plan.read_maxdiff(0)  # sync
        t_init = time.perf_counter() - t0
        per_it = []
        for it in range(a.iters):
            b = bounds(plan, it, w)
            ts = []
            for r in range(w):
                t = time.perf_counter()
                plan.iterate(it, int(b[r]), int(b[r + 1]))
                plan.read_maxdiff(it)  # stream sync
                ts.append(time.perf_counter() - t)
            rows = np.diff(b)
            blocks = 8 + rows * rb.value  # each rank's block at its bound (the sharded loop's exchange)
            recv = [int(blocks.sum() - blocks[r]) for r in range(w)]
            per_it.append({"it": it, "range_s": ts, "rows": rows.tolist(), "max_recv_bytes": max(recv) if w > 1 else 0})
        plan.finish(a.iters)
        floor = sum(max(x["range_s"]) for x in per_it)
        total = sum(sum(x["range_s"]) for x in per_it)
        recv = sum(x["max_recv_bytes"] for x in per_it)
        # the sharded ends of a routed run (grank.hip init_sharded / x_gather_topk): each rank's
        # top-K of its own rows (after this job), then each rank's init of its own sources
        ms = ctypes.c_double()
        topk_ms, init_ms = [], []
        for r in range(w):
            _lib.check(_lib.lib().ppr_grank_plan_ends_time(plan._p, w, r, a.iters, 0, ctypes.byref(ms)), "ends_time")
            topk_ms.append(ms.value)
        for r in range(w):
            _lib.check(_lib.lib().ppr_grank_plan_ends_time(plan._p, w, r, a.iters, 1, ctypes.byref(ms)), "ends_time")
            init_ms.append(ms.value)
        res["worlds"][str(w)] = {"init_s": t_init, "merge_floor_s": floor, "merge_sum_s": total,
                                 "max_rank_recv_bytes_per_job": recv, "sharded_topk_ms": topk_ms,
                                 "sharded_init_ms": init_ms, "iterations": per_it}
        print(f"world {w}: init {t_init:.3f} s (sharded: slowest rank {max(init_ms):.1f} ms), slowest-rank merge "
              f"{floor:.3f} s / job (all ranges {total:.3f} s), sharded top-K slowest rank {max(topk_ms):.1f} ms, "
              f"largest per-rank receive {recv / 1e9:.1f} GB / job", flush=True)
    plan.close()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
