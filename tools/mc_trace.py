"""Per-level critical-path breakdown of the MC combine from a rocprofv3 --kernel-trace CSV
(tools/mc_trace_run.sh): levels start at k_classify; per level the span, the GPU-busy union of
kernel intervals, and per kernel name its mean duration and the mean idle gap before it.

    python tools/mc_trace.py gpurun_out/mctrace/trace/run_kernel_trace.csv
"""
import collections
import csv
import sys


def short(n):
    n = n.split("(")[0].replace("void ", "").replace("pprk::", "")
    return n[:28]


def main(path):
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
                for r in csv.DictReader(open(path)))
    starts = [i for i, e in enumerate(ev) if e[2].startswith("k_classify") and not e[2].startswith("k_classify_big")]
    levels = [ev[a:b] for a, b in zip(starts, starts[1:])]
    span = busy = 0
    dur = collections.defaultdict(lambda: [0, 0])
    gap = collections.defaultdict(lambda: [0, 0])
    nk = 0
    for lv in levels:
        s0, e_end = lv[0][0], max(e for _, e, _ in lv)
        span += e_end - s0
        cur_s, cur_e = lv[0][0], lv[0][1]
        for s, e, n in lv[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        prev_end = None
        for s, e, n in lv:
            dur[n][0] += 1
            dur[n][1] += e - s
            if prev_end is not None:
                gap[n][0] += 1
                gap[n][1] += max(0, s - prev_end)
            prev_end = e if prev_end is None else max(prev_end, e)
            nk += 1
    L = len(levels)
    print(f"levels {L}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  kernels/level {nk / L:.1f}")
    print(f"  per level: span {span / L / 1e3:.1f} us  busy {busy / L / 1e3:.1f} us")
    print(f"  {'kernel':28s} {'count':>7s} {'mean us':>8s} {'total ms':>9s} {'gap before us':>14s} {'gap ms':>8s}")
    for n, (c, d) in sorted(dur.items(), key=lambda x: -x[1][1]):
        gc, gs = gap.get(n, [0, 0])
        print(f"  {n:28s} {c:7d} {d / c / 1e3:8.1f} {d / 1e6:9.1f} {gs / gc / 1e3 if gc else 0:14.1f} {gs / 1e6:8.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
