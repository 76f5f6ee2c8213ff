"""Sieve on vs off on the device (PPR_SV=1 vs PPR_SV=0: the range / partition engines, bit-exact vs
the oracle) -- iteration by iteration maxDiff, and at the first difference the rows that differ.

    python tools/sv_check.py SCALE K L ITERS [VAR=X ...]    # VARs apply to the sieve plan only
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import approximated_personalized_pagerank_amd as ppr  # noqa: E402

scale, K, L, iters = (int(x) for x in sys.argv[1:5])
extra = dict(a.split("=", 1) for a in sys.argv[5:])
t0 = time.time()
g = ppr.rmat(scale, seed=42)
part = g.partitions()
print(f"graph n={g.n} m={g.m} {time.time() - t0:.1f} s", flush=True)
os.environ.update(extra)
os.environ["PPR_SV"] = "1"
a = ppr.GrankPlan(g, K, L, 0.85, part=part, device=0)
for k in extra:
    del os.environ[k]
os.environ["PPR_SV"] = "0"
b = ppr.GrankPlan(g, K, L, 0.85, part=part, device=0)
del os.environ["PPR_SV"]
a.init()
b.init()
deg = np.diff(g.row_ptr)
for it in range(iters):
    a.iterate(it, 0, a.active_count(it))
    b.iterate(it, 0, b.active_count(it))
    ma, mb = a.read_maxdiff(it), b.read_maxdiff(it)
    print(f"it {it}: maxdiff {ma.hex()} {mb.hex()} {'same' if ma == mb else 'DIFF'}", flush=True)
    if ma != mb:
        ia, sa, la = a.fetch_slab(it + 1)
        ib, sb, lb = b.fetch_slab(it + 1)
        bad = np.nonzero((la != lb) | np.any(ia != ib, axis=1) | np.any(sa.view(np.int64) != sb.view(np.int64), axis=1))[0]
        print(f"rows differing: {len(bad)}")
        for v in bad[:12]:
            n1, n2 = la[v], lb[v]
            ka = dict(zip(ia[v, :n1].tolist(), sa[v, :n1].tolist()))
            kb = dict(zip(ib[v, :n2].tolist(), sb[v, :n2].tolist()))
            dup = n1 - len(ka)
            only_a = sorted(set(ka) - set(kb))[:4]
            only_b = sorted(set(kb) - set(ka))[:4]
            vd = [(k, ka[k], kb[k]) for k in set(ka) & set(kb) if ka[k] != kb[k]][:4]
            print(f" v={v} deg={deg[v]} part={part[v]} len {n1}/{n2} dup_in_sieve_row={dup} only_sv={only_a} "
                  f"only_ref={only_b} value_diffs={len([1 for k in set(ka) & set(kb) if ka[k] != kb[k]])} {vd}")
        break
a.close()
b.close()
