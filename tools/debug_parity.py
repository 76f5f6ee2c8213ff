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
        print("   gpu", list(zip(ids[v, :8].tolist(), sc[v, :8].round(6).tolist())))
        print("   ora", list(zip(b["slab_ids"][v, :8].tolist(), b["slab_scores"][v, :8].round(6).tolist())))
    return len(bad)

scale, K, L = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
g = ppr.rmat(scale, seed=7)
part = g.partitions()
deg = g.degrees()
print("n", g.n, "m", g.m, "maxdeg", deg.max())
for it in range(0, 4):
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
