"""Diagnostic: compare GPU slab vs oracle slab after init and after each iteration."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import approximated_personalized_pagerank_amd as ppr
import oracle

def compare(tag, a, b):
    ids, sc, ln = a
    bad = np.nonzero((ln != b["slab_lens"]) | (ids != b["slab_ids"]).any(1) | (sc != b["slab_scores"]).any(1))[0]
    print(f"{tag}: {len(bad)} differing rows of {len(ln)}")
    for v in bad[:3]:
        print("  v", v, "gpu len", ln[v], "ora len", b["slab_lens"][v])
        d = np.nonzero((ids[v] != b["slab_ids"][v]) | (sc[v] != b["slab_scores"][v]))[0]
        print("   first diff at", d[:5], "deg", g.row_ptr[v+1]-g.row_ptr[v], "part", part[v])
        for i in d[:3]:
            print("   gpu", ids[v, i], repr(sc[v, i]), " ora", b["slab_ids"][v, i], repr(b["slab_scores"][v, i]))
    return len(bad)

scale, K, L = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
g = ppr.rmat(scale, seed=int(sys.argv[5]) if len(sys.argv) > 5 else 7)
part = g.partitions()
deg = g.degrees()
print("n", g.n, "m", g.m, "maxdeg", deg.max())
for it in range(0, int(sys.argv[4]) if len(sys.argv) > 4 else 4):
    plan = ppr.GrankPlan(g, K, L, 0.85, part=part, device=0)
    plan.init()
    for i in range(it):
        plan.iterate(i, 0, plan.active_count(i))
    plan.finish(it)
    gs = plan.fetch_slab(it)
    plan.close()
    if it == 0:
        # oracle with 0 iterations is not allowed; emulate: 1 iteration then compare only inactive? use iterations=1 tol huge
        o = oracle.grank(g.row_ptr, g.col, part, K, L, 0, 0.85, -1.0, want_slab=True)
    else:
        o = oracle.grank(g.row_ptr, g.col, part, K, L, it, 0.85, -1.0, want_slab=True)
    compare(f"after {it} iterations", gs, o)
