"""Timeline view of a rocprofv3 run (rocpd database): GPU busy union vs idle over the second half
of the trace (the timed steps), and per kernel the time it ran alone ("exclusive") vs overlapped
with another stream's kernel.

    python tools/timeline.py gpurun_out/prof7/run_results.db
"""
import sqlite3
import sys
from collections import defaultdict

con = sqlite3.connect(sys.argv[1])
rows = sorted(con.execute("select name, start, end, queue_id from kernels"), key=lambda r: r[1])
t0, t1 = rows[0][1], max(r[2] for r in rows)
mid = t0 + (t1 - t0) // 2
rows = [r for r in rows if r[1] >= mid]
ev = []
for i, (n, s, e, q) in enumerate(rows):
    ev.append((s, 1, i))
    ev.append((e, -1, i))
ev.sort()
active = set()
last = ev[0][0]
busy = idle = 0
excl = defaultdict(int)
shared = defaultdict(int)
for t, kind, i in ev:
    dt = t - last
    if active:
        busy += dt
        if len(active) == 1:
            excl[next(iter(active))] += dt
        else:
            for j in active:
                shared[j] += dt / len(active)
    else:
        idle += dt
    last = t
    if kind == 1:
        active.add(i)
    else:
        active.discard(i)
byname = defaultdict(lambda: [0, 0, 0])
for i, (n, s, e, q) in enumerate(rows):
    k = n.split("(")[0].replace("void ", "")[-40:]
    byname[k][0] += e - s
    byname[k][1] += excl[i]
    byname[k][2] += shared[i]
span = ev[-1][0] - ev[0][0]
print(f"span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f}  idle {idle / 1e6:.1f}  queues {sorted(set(r[3] for r in rows))}")
print(f"{'kernel':40s} {'dur ms':>9s} {'alone ms':>9s} {'shared ms':>9s}")
for k, (d, x, sh) in sorted(byname.items(), key=lambda kv: -kv[1][0])[:14]:
    print(f"{k:40s} {d / 1e6:9.1f} {x / 1e6:9.1f} {sh / 1e6:9.1f}")
