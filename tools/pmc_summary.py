"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (one counter per run, as the
MI355X guide prescribes) into per-kernel HBM traffic.

    python tools/pmc_summary.py FETCH.csv WRITE.csv steps > profiles/<round>_<workload>_pmc.json

FETCH_SIZE / WRITE_SIZE are reported in KiB. gfx950 correction (MI355X_MICROARCH.md "HBM"):
FETCH_SIZE counts 128-B requests at 64 B, so fetched bytes = 2 x FETCH_SIZE; WRITE_SIZE is used
as is. Both factors are calibrated for this engine's own access patterns by tools/pmc_calib.hip
(profiles/r02_pmc_calibration.json): 4-B and 8-B per-lane basket-row gathers and 12-B staging
record streams read 2.00x FETCH_SIZE, 12-B record stores write 1.00x WRITE_SIZE; the stable
partition's short runs (48 B per bucket per tile) really do cost 3.4x their bytes in HBM writes.
Totals are per step (one whole job) over the kernels of the merge phase.
"""
from __future__ import annotations

import collections
import csv
import json
import sys

MERGE_KERNELS = ("k_classify", "k_merge_lds", "k_merge_wg", "k_merge_glb", "k_hub_", "rocprim", "k_stat", "k_xr", "k_xb",
                 "k_xfin", "k_gather", "k_sv", "k_xg_", "k_wfin", "k_xm")


def per_kernel(path):
    acc = collections.defaultdict(float)
    calls = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        acc[k] += float(r["Counter_Value"]) * 1024.0
        calls[k] += 1
    return acc, calls


def main(fetch_csv, write_csv, steps, mode="chain"):
    f, calls = per_kernel(fetch_csv)
    w, _ = per_kernel(write_csv)
    kernels = {}
    for k in sorted(set(f) | set(w), key=lambda k: -(2 * f.get(k, 0) + w.get(k, 0))):
        kernels[k] = {"calls": calls.get(k, 0), "fetch_bytes": 2 * f.get(k, 0.0) / steps,
                      "write_bytes": w.get(k, 0.0) / steps}
    merge = [k for k in kernels if any(t in k for t in MERGE_KERNELS)]
    out = {
        "note": ("bytes per step; fetch = 2 x FETCH_SIZE, write = WRITE_SIZE (gfx950; factors calibrated on "
                 "this engine's access patterns, profiles/r02_pmc_calibration.json); KiB -> bytes"),
        "merge_phase_traffic_bytes": sum(kernels[k]["fetch_bytes"] + kernels[k]["write_bytes"] for k in merge),
        "merge_kernels": merge,
        "sum": mode,
        "kernels": kernels,
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    # (4th argument: the GRank summation mode the profiled run used, exact | chain)
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1, sys.argv[4] if len(sys.argv) > 4 else "chain")
