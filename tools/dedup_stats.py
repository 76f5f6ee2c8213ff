"""Distinct-key statistics of the hub sources' candidate streams (design input, not a test).

Runs GRank RMAT-<scale> K64/L128 for a few iterations on the GPU, fetches the slab, then (torch on
the GPU) for every source whose candidate count exceeds the wave tiers (C + 1 > 1536):
  C_v  candidates (sum of successor basket lengths), D_v distinct keys,
  the share of hub candidates in sources with D_v <= X (one workgroup LDS table could hold them),
  and the distinct-per-tile ratio sum_t D_{v,t} / C_v for tiles of tw consecutive successors
  (how much an order-free tile-level pre-aggregation would shrink the staged records).
usage: python tools/dedup_stats.py [scale] [iterations]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import approximated_personalized_pagerank_amd as ppr  # noqa: E402


def main():
    scale = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    t0 = time.time()
    g = ppr.rmat(scale, seed=42)
    part = g.partitions()
    plan = ppr.GrankPlan(g, 64, 128, 0.85, part=part, device=0)
    plan.run(iters, -1.0)
    ids_h, _, lens_h = plan.fetch_slab()
    plan.close()
    print(f"run + fetch {time.time() - t0:.1f} s", flush=True)
    stats(g, ids_h, lens_h, torch.device("cuda:0"), scale, iters)


def stats(g, ids_h, lens_h, dev, scale, iters):
    rp = torch.from_numpy(g.row_ptr.astype(np.int64)).to(dev)
    col = torch.from_numpy(g.col.astype(np.int64)).to(dev)
    ids = torch.from_numpy(ids_h).to(dev)
    lens = torch.from_numpy(lens_h.astype(np.int64)).to(dev)
    n = g.n
    L = ids.shape[1]
    deg = rp[1:] - rp[:-1]
    src_of_edge = torch.repeat_interleave(torch.arange(n, device=dev), deg)
    C = torch.zeros(n, dtype=torch.int64, device=dev).index_add_(0, src_of_edge, lens[col])
    hub = (C + 1 > 1536).nonzero().flatten()
    Ch = C[hub]
    print(f"n {n}, hub sources {hub.numel()}, hub candidates {int(Ch.sum())} of {int(C.sum())}", flush=True)
    tws = [4, 8, 16, 32, 64, 256]
    D_all = torch.zeros(hub.numel(), dtype=torch.int64, device=dev)
    tile_d = {tw: torch.zeros(hub.numel(), dtype=torch.int64, device=dev) for tw in tws}
    budget = 3 * 10 ** 8
    cs = torch.cumsum(Ch, 0).cpu().numpy()
    i0 = 0
    H = hub.numel()
    while i0 < H:
        base = cs[i0 - 1] if i0 else 0
        i1 = int(np.searchsorted(cs, base + budget, side="right"))
        i1 = max(i1, i0 + 1)
        srcs = hub[i0:i1]
        d = deg[srcs]
        e_loc = torch.repeat_interleave(torch.arange(srcs.numel(), device=dev), d)
        starts = rp[srcs]
        e_first = torch.repeat_interleave(torch.cumsum(d, 0) - d, d)
        e_pos = torch.arange(e_loc.numel(), device=dev) - e_first
        e_u = col[starts[e_loc] + e_pos]
        rows = ids[e_u]                                    # [E, L]
        mask = torch.arange(L, device=dev)[None, :] < lens[e_u][:, None]
        keys = rows.to(torch.int64)[mask]                  # hot-tag free: plain runs (PPR_HOT_N off)
        eloc_c = e_loc[:, None].expand(-1, L)[mask]
        epos_c = e_pos[:, None].expand(-1, L)[mask]
        del rows, mask
        u = torch.unique(eloc_c * (1 << 23) + keys)
        D_all[i0:i1] += torch.bincount(u >> 23, minlength=srcs.numel())
        del u
        for tw in tws:
            u = torch.unique((eloc_c * (1 << 18) + epos_c // tw) * (1 << 23) + keys)
            tile_d[tw][i0:i1] += torch.bincount(u >> 41, minlength=srcs.numel())
            del u
        del keys, eloc_c, epos_c
        torch.cuda.empty_cache()
        i0 = i1
    Cn = Ch.double()
    tot = Cn.sum().item()
    out = {"scale": scale, "iterations": iters, "hub_sources": H, "hub_candidates": tot,
           "distinct_total": int(D_all.sum()), "distinct_over_candidates": D_all.sum().item() / tot}
    thr = {}
    for X in [1024, 2048, 4096, 6144, 8192, 12288, 16384, 32768, 65536]:
        m = D_all <= X
        thr[str(X)] = {"sources": int(m.sum()), "cand_share": Cn[m].sum().item() / tot}
    out["cand_share_by_distinct_cap"] = thr
    out["tile_distinct_ratio"] = {str(tw): tile_d[tw].sum().item() / tot for tw in tws}
    big = D_all > 8192
    out["tile_distinct_ratio_D_gt_8192"] = {str(tw): tile_d[tw][big].sum().item() / max(1.0, Cn[big].sum().item())
                                            for tw in tws}
    order = torch.argsort(Ch, descending=True)[:15]
    out["largest"] = [{"v": int(hub[i]), "deg": int(deg[hub[i]]), "C": int(Ch[i]), "D": int(D_all[i]),
                       "tile64_ratio": tile_d[64][i].item() / Ch[i].item()} for i in order.tolist()]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
