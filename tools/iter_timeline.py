"""Per-iteration view of a rocprofv3 run (rocpd database): each iteration (from one k_classify to the
next) with its span, GPU-busy time and the first-start / last-end of the main kernel families.

    python tools/iter_timeline.py gpurun_out/TAG/prof/run_results.db > profiles/<round>_grank_iteration_timeline.txt
"""
import sqlite3, sys
from collections import defaultdict
con = sqlite3.connect(sys.argv[1])
rows = sorted(con.execute("select name, start, end, queue_id from kernels"), key=lambda r: r[1])
t0, t1 = rows[0][1], max(r[2] for r in rows)
mid = t0 + (t1 - t0) // 2
rows = [r for r in rows if r[1] >= mid]
# iteration starts: k_classify( launches (not _big)
starts = [r[1] for r in rows if r[0].startswith("pprk::k_classify(")]
starts.append(max(r[2] for r in rows))
def fam(n):
    n = n.split("(")[0]
    for k in ["k_sv1_redo", "k_sv1", "k_svA", "k_svB", "k_svF", "k_svfin", "k_xm", "k_xr", "k_merge_lds_x", "k_xb", "k_xfin1", "k_classify"]:
        if k in n: return k
    return "other"
for it in range(len(starts) - 1):
    a, b = starts[it], starts[it + 1]
    rs = [r for r in rows if a <= r[1] < b]
    last = defaultdict(int); first = {}
    busy = 0; ev = sorted([(r[1], 1) for r in rs] + [(r[2], -1) for r in rs]); act = 0; lt = a
    for t, k in ev:
        if act > 0: busy += t - lt
        act += k; lt = t
    for r in rs:
        f = fam(r[0]); last[f] = max(last[f], r[2] - a); first.setdefault(f, r[1] - a)
    s = " ".join(f"{f}:{first[f]/1e6:.1f}-{last[f]/1e6:.1f}" for f in ["k_merge_lds_x", "k_sv1", "k_xr", "k_xm", "k_xb"] if f in last)
    print(f"it {it:2d} span {(b-a)/1e6:6.2f} busy {busy/1e6:6.2f}  {s}")
