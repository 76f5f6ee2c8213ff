"""Per-kernel sums of SQ counters from rocprofv3 --pmc csv outputs (one or more passes):

    python tools/sq_summary.py gpurun_out/sq/a/run_counter_collection.csv [more.csv ...]

Prints, for the hub and merge kernels, each counter's total and per-wave-cycle ratios."""
import collections
import csv
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("pprk::", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", kv[1].get("SQ_LDS_IDX_ACTIVE", 0))):
    if not any(x in k for x in ("hub", "merge", "classify", "k_x", "k_sv")):
        continue
    print(k)
    wc = c.get("SQ_WAVE_CYCLES", 0)
    for n, v in sorted(c.items()):
        extra = f"  ({v / wc:.3f} of wave cycles)" if wc and n.startswith("SQ_WAIT") or n.startswith("SQ_ACTIVE") else ""
        print(f"   {n:28s} {v:16.4g}{extra}")
