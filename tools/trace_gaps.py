"""Kernel-time and idle-gap breakdown of a rocprofv3 --kernel-trace CSV (second half of the
trace = the timed step when the bench ran one warmup and one timed step).

    python tools/trace_gaps.py gpurun_out/prof/run_kernel_trace.csv
"""
import collections
import csv
import sys


def main(path, frac=0.5):
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                 r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pprk::", "")[:24]) for r in rows)
    ev = ev[int(len(ev) * frac):]
    span = ev[-1][1] - ev[0][0]
    agg = collections.defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        agg[n][0] += 1
        agg[n][1] += e - s
    gaps = collections.defaultdict(lambda: [0, 0])
    for (s0, e0, n0), (s1, e1, n1) in zip(ev, ev[1:]):
        if s1 > e0:
            gaps[(n0, n1)][0] += 1
            gaps[(n0, n1)][1] += s1 - e0
    print(f"span {span / 1e9:.3f} s, kernels {len(ev)}, idle {sum(g for _, g in gaps.values()) / 1e9:.3f} s")
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:14]:
        print(f"  {n:26s} {c:7d} {d / 1e6:9.1f} ms")
    print("largest gaps (after -> before):")
    for k, (c, g) in sorted(gaps.items(), key=lambda x: -x[1][1])[:8]:
        print(f"  {k[0]:24s} -> {k[1]:24s} {c:6d} {g / 1e6:8.1f} ms {g / c / 1e3:8.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
