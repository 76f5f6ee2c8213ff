"""Per-kernel roofline table of one GRank job from a round's profile set (tools/profile_round.sh):

    python tools/kernel_roofline.py STATS.csv FETCH.csv WRITE.csv TRACE_STEPS PMC_STEPS [SQ_SUMMARY.txt] [BENCH.json]

STATS.csv  rocprofv3 --kernel-trace --stats summary (TotalDurationNs per kernel)
FETCH.csv  rocprofv3 --pmc FETCH_SIZE counter collection (KiB; x2 on gfx950, MI355X_MICROARCH.md "HBM")
WRITE.csv  rocprofv3 --pmc WRITE_SIZE counter collection (KiB)
TRACE_STEPS / PMC_STEPS  jobs in the traced run and in each PMC run
SQ_SUMMARY tools/sq_summary.py output: the wave-cycle fractions waiting / issuing (optional; "-": none)
BENCH.json the bench line of the traced build (optional): its roofline.kernels give each kernel
           group's algorithmic bytes per job (counted on the device per tier), which
           are joined with the group's kernels' traced time and PMC traffic ("groups" below)

Per kernel, per job: summed launch durations, HBM bytes (2 x FETCH + WRITE), their rate and the
fraction of the 8 TB/s peak, and a bound label: "hbm" when the rate is >= 60 % of the measured
6.3 TB/s streaming ceiling, otherwise "latency" (waves parked on s_waitcnt for most of their
cycles: SQ_WAIT_ANY) or "issue" (SQ_ACTIVE_INST_ANY high). Kernels of the merge phase run on four
streams at once, so their durations overlap: the sum exceeds the job's merge span, and a kernel's
rate is its own bytes over its own duration.
"""
import collections
import csv
import json
import re
import sys

PEAK = 8000e9
STREAM_CEIL = 6300e9  # measured float4 copy (MI355X_MICROARCH.md chip table)


def kname(s):
    s = s.split("(")[0].replace("void ", "").replace("pprk::", "")
    return re.sub(r"<.*", "", s) if "rocprim" not in s else "rocprim scan"


def durations(path):
    d = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = kname(r["Name"])
        d[k] += float(r["TotalDurationNs"]) * 1e-9
        calls[k] += int(r["Calls"])
    return d, calls


def pmc(path):
    acc = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        acc[kname(r["Kernel_Name"])] += float(r["Counter_Value"]) * 1024.0
    return acc


def sq(path):
    out, cur = {}, None
    for ln in open(path):
        if not ln.startswith(" "):
            cur = re.sub(r"<.*", "", ln.strip())
            out[cur] = {}
            continue
        m = re.match(r"\s+(SQ_\w+)\s+([\d.e+]+)(?:\s+\(([\d.]+) of wave cycles\))?", ln)
        if m and m.group(3):
            out[cur][m.group(1)] = float(m.group(3))
    return out


def main():
    stats, fetch, write = sys.argv[1], sys.argv[2], sys.argv[3]
    steps, psteps = int(sys.argv[4]), int(sys.argv[5])
    d, calls = durations(stats)
    f, w = pmc(fetch), pmc(write)
    q = sq(sys.argv[6]) if len(sys.argv) > 6 and sys.argv[6] != "-" else {}
    bench = json.load(open(sys.argv[7])) if len(sys.argv) > 7 else None
    rows = []
    for k in sorted(d, key=lambda k: -d[k]):
        t = d[k] / steps
        if t < 1e-3:
            continue
        b = (2 * f.get(k, 0.0) + w.get(k, 0.0)) / psteps
        rate = b / t if t else 0.0
        sqk = q.get(k, {})
        wait, act = sqk.get("SQ_WAIT_ANY"), sqk.get("SQ_ACTIVE_INST_ANY")
        bound = "hbm" if rate >= 0.6 * STREAM_CEIL else ("latency" if (wait or 0) >= 0.5 else "issue")
        rows.append({"kernel": k, "calls_per_job": calls[k] / steps, "time_s_per_job": round(t, 4),
                     "hbm_bytes_per_job": b, "read_bytes": 2 * f.get(k, 0.0) / psteps, "write_bytes": w.get(k, 0.0) / psteps,
                     "gbps": round(rate / 1e9, 1), "frac_of_peak": round(rate / PEAK, 4),
                     "sq_wait_frac": wait, "sq_active_frac": act, "bound": bound})
    out = {"note": __doc__.split("\n\n")[2].replace("\n", " "), "trace_steps": steps, "pmc_steps": psteps,
           "kernels": rows}
    if bench:
        # kernel groups of the bench line (bench.py KERNEL_GROUPS): their kernels by name
        members = {"wave tier": ["k_merge_lds_x"], "sieve one-slice": ["k_sv1", "k_sv1_redo", "k_sv1_list", "k_svfin"],
                   "sieve multi-slice": ["k_svA", "k_svB", "k_svF"]}
        kb = bench["roofline"].get("kernels", {})
        algo = {"wave tier": sum(v["algo_bytes_per_step"] for k, v in kb.items() if k.startswith("wave tier")),
                "sieve one-slice": sum(v["algo_bytes_per_step"] for k, v in kb.items() if k.startswith("sieve")
                                       and "multi" not in k),
                "sieve multi-slice": sum(v["algo_bytes_per_step"] for k, v in kb.items() if "multi" in k)}
        groups = {}
        for gname, ks in members.items():
            t = sum(d.get(k, 0.0) for k in ks) / steps
            hb = sum(2 * f.get(k, 0.0) + w.get(k, 0.0) for k in ks) / psteps
            a = algo[gname]
            groups[gname] = {"kernels": ks, "algo_bytes_per_job": a, "kernel_time_s_per_job": round(t, 4),
                             "hbm_bytes_per_job": hb, "traffic_over_algo": round(hb / a, 3) if a else None,
                             "algo_gbps": round(a / t / 1e9, 1) if t else None,
                             "algo_frac_of_peak": round(a / t / PEAK, 4) if t else None}
        rest = [r for r in rows if not any(r["kernel"] in ks for ks in members.values())]
        groups["range / partition engines and the rest"] = {
            "kernels": [r["kernel"] for r in rest], "algo_bytes_per_job": bench["roofline"]["algo_bytes_per_step"] - sum(algo.values()),
            "hbm_bytes_per_job": sum(r["hbm_bytes_per_job"] for r in rest)}
        out["groups"] = groups
        out["merge_phase"] = {"algo_bytes_per_job": bench["roofline"]["algo_bytes_per_step"],
                              "merge_s_per_job": bench["roofline"]["merge_ms_per_step"] / 1e3,
                              "frac": bench["roofline"]["frac"]}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
