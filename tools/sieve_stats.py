#!/usr/bin/env python3
"""Workload study for a sketch-filtered merge of the wide GRank sources (RMAT-22 K64/L128).

For the sources the wave tier does not take (candidates + 1 > 1536), at a settled iteration:
the L-th final total theta, the bound theta_lb = the smallest new total of the source's previous
top-L keys (a rigorous lower bound of theta: L distinct keys reach it), the mass of the other keys,
and how many of those other keys a count-min sketch (r rows x w counters, no prev keys in it)
lets through at theta_lb -- the keys an exact second pass would have to accumulate.

    python tools/sieve_stats.py [--scale 22] [--iters 20] [--out gpurun_out/sieve_stats.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def mhash(k, seed):
    x = (k.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15) + np.uint64(seed)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    x ^= x >> np.uint64(29)
    x = (x * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    x ^= x >> np.uint64(32)
    return x


def analyse(g, ids, sc, lens, part_p, L, damping, rng, per_bin=12, top=24):
    rp, col = g.row_ptr, g.col
    deg = np.diff(rp)
    src_of_edge = np.repeat(np.arange(g.n, dtype=np.int64), deg)
    cand = np.bincount(src_of_edge, weights=lens[col].astype(np.float64), minlength=g.n).astype(np.int64)
    act = np.nonzero(part_p & (deg > 0))[0]
    wide = act[cand[act] + 1 > 1536]
    summary = {"active": int(len(act)), "active_cand": int(cand[act].sum()), "wide": int(len(wide)),
               "wide_cand": int(cand[wide].sum()), "wide_edges": int(deg[wide].sum())}
    lb = np.floor(np.log2(np.maximum(cand[wide], 1))).astype(int)
    hist = {int(b): [int((lb == b).sum()), int(cand[wide][lb == b].sum())] for b in np.unique(lb)}
    summary["wide_by_log2_cand"] = hist
    pick = []
    for b in np.unique(lb):
        m = wide[lb == b]
        pick.extend(rng.choice(m, min(per_bin, len(m)), replace=False).tolist())
    pick.extend(wide[np.argsort(-cand[wide])[:top]].tolist())
    pick = sorted(set(pick))
    configs = [(1, 8192), (2, 4096), (2, 8192), (3, 8192), (2, 16384)]
    rows = []
    for v in pick:
        s = col[rp[v]:rp[v + 1]]
        ln = lens[s]
        mask = np.arange(L)[None, :] < ln[:, None]
        keys = ids[s][mask].astype(np.int64)
        f = damping / len(s)
        p = sc[s][mask] * f
        tot = np.bincount(keys, weights=p, minlength=g.n)
        tot[v] += 1.0 - damping
        nzk = np.nonzero(tot)[0]
        D = len(nzk)
        tv = tot[nzk]
        theta = float(np.partition(tv, D - L)[D - L]) if D >= L else 0.0
        prev = ids[v, :lens[v]].astype(np.int64)
        full = lens[v] == L
        theta_lb = float(tot[prev].min()) if full else 0.0
        isprev = np.zeros(g.n, dtype=bool)
        isprev[prev] = True
        cm = ~isprev[keys]
        okeys, op = keys[cm], p[cm]
        tail_mass = float(op.sum()) + (0.0 if isprev[v] else 1.0 - damping)
        other = nzk[~isprev[nzk]]
        need = int((tot[other] >= theta_lb).sum())
        r = {"v": int(v), "deg": int(len(s)), "cand": int(len(keys)), "distinct": D, "theta": theta,
             "theta_lb": theta_lb, "prev_full": bool(full), "tail_mass": tail_mass,
             "other_keys_true_ge_lb": need, "prev_in_new_topL": int(np.isin(prev, nzk[tv >= theta]).sum()) if D >= L else None}
        ok = np.concatenate([okeys, [v]]) if not isprev[v] else okeys
        opp = np.concatenate([op, [1.0 - damping]]) if not isprev[v] else op
        for (nr, w) in configs:
            ub = None
            for j in range(nr):
                h = (mhash(ok, 17 + 101 * j) % np.uint64(w)).astype(np.int64)
                cnt = np.bincount(h, weights=opp, minlength=w)
                hk = (mhash(other, 17 + 101 * j) % np.uint64(w)).astype(np.int64)
                u = cnt[hk]
                ub = u if ub is None else np.minimum(ub, u)
            passing = ub >= theta_lb
            # candidates of passing keys (the second pass's exact inserts)
            pk = np.zeros(g.n, dtype=bool)
            pk[other[passing]] = True
            r[f"pass_r{nr}_w{w}"] = int(passing.sum())
            r[f"pcand_r{nr}_w{w}"] = int(pk[okeys].sum())
            r[f"mean_counter_r{nr}_w{w}"] = float(opp.sum() / w)
        rows.append(r)
    return summary, rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--iters", type=int, nargs="+", default=[2, 20, 21])
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "sieve_stats.json"))
    args = ap.parse_args()
    import approximated_personalized_pagerank_amd as ppr
    t = time.time()
    g = ppr.rmat(args.scale, seed=42)
    part = g.partitions()
    L, K, d = 128, 64, 0.85
    plan = ppr.GrankPlan(g, K, L, d, part=part, device=0)
    print(f"graph + plan {time.time() - t:.1f} s", flush=True)
    out = {"scale": args.scale, "L": L, "by_iteration": {}}
    rng = np.random.default_rng(1)
    for it in args.iters:
        plan.run(it, -1.0)
        ids, sc, lens = plan.fetch_slab()
        p = it % 2  # iteration `it` updates partition it % 2
        t = time.time()
        summ, rows = analyse(g, ids, sc, lens, part == p, L, d, rng)
        print(f"iteration {it} (partition {p}): {len(rows)} sources analysed in {time.time() - t:.1f} s", flush=True)
        out["by_iteration"][str(it)] = {"partition": p, "summary": summ, "rows": rows}
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f)
        del ids, sc, lens
    plan.close()


if __name__ == "__main__":
    main()
