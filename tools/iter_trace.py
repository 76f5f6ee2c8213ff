#!/usr/bin/env python3
"""Per-iteration view of a rocprofv3 kernel trace of one GRank job (the last job in the trace):
iteration span, and per kernel group the summed kernel time and its first start / last end
relative to the iteration start -- where an iteration's critical path and tail are.

    python tools/iter_trace.py gpurun_out/<tag>/prof/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")
       .replace("pprk::", ""), int(r["Queue_Id"]), int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"])))
      for r in rows]
ks.sort()
# iterations start at k_classify; jobs at k_probe / the init (unit) classify: take the last 30 iterations' classify calls
cls = [i for i, k in enumerate(ks) if k[2] == "k_classify"]
starts = cls[-31:]  # init + 30 iterations of the last job
print(f"{'it':>3} {'span ms':>8}  " + "  ".join(f"{n}" for n in ["groups (sum ms | first..last ms)"]))
for it in range(len(starts) - 1):
    a, b = starts[it], starts[it + 1]
    t0 = ks[a][0]
    t1 = ks[b][0]
    grp = defaultdict(lambda: [0.0, 1e18, 0.0, 0])
    for s, e, n, q, nb in ks[a:b]:
        g = grp[n]
        g[0] += (e - s) / 1e6
        g[1] = min(g[1], (s - t0) / 1e6)
        g[2] = max(g[2], (e - t0) / 1e6)
        g[3] += nb
    top = sorted(grp.items(), key=lambda kv: -kv[1][0])[:7]
    print(f"{it:3d} {(t1 - t0) / 1e6:8.2f}  " + "  ".join(f"{n}:{v[0]:.1f}|{v[1]:.1f}..{v[2]:.1f}[{v[3]}]" for n, v in top))
