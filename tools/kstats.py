"""Per-kernel totals of a rocprofv3 trace database (diagnostics): total / max duration, count,
and for one kernel name (second argument, substring) its longest dispatches with grid and
register counts.

    python tools/kstats.py gpurun_out/prof/run_results.db [k_hub_hot]
"""
import sqlite3
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
rows = list(con.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count, "
                        "scratch_size from kernels"))
tot, cnt, mx = defaultdict(float), defaultdict(int), defaultdict(float)
for n, s, e, *_ in rows:
    k = n.split("(")[0].replace("void ", "")[-44:]
    tot[k] += (e - s) / 1e6
    cnt[k] += 1
    mx[k] = max(mx[k], (e - s) / 1e6)
print(f"{'kernel':44s} {'total ms':>10s} {'max ms':>8s} {'calls':>6s}")
for k, v in sorted(tot.items(), key=lambda x: -x[1])[:18]:
    print(f"{k:44s} {v:10.1f} {mx[k]:8.2f} {cnt[k]:6d}")
if len(sys.argv) > 2:
    sel = sorted(((e - s) / 1e6, gx // max(wx, 1), lds, vg, sg, scr) for n, s, e, gx, wx, lds, vg, sg, scr in rows
                 if sys.argv[2] in n)
    sel.reverse()
    print(f"{sys.argv[2]}: {len(sel)} dispatches; longest (ms, blocks, lds, vgpr, sgpr, scratch):")
    for r in sel[:12]:
        print("  ", r)
