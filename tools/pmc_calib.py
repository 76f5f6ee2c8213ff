"""Turn the calibration runs of tools/pmc_calib.hip into FETCH_SIZE / WRITE_SIZE correction factors.

    rocprofv3 --pmc FETCH_SIZE -d D/fetch -o run --output-format csv -- tools/_build/pmc_calib > D/known.json
    rocprofv3 --pmc WRITE_SIZE -d D/write -o run --output-format csv -- tools/_build/pmc_calib
    python tools/pmc_calib.py D > profiles/r02_pmc_calibration.json

factor = known bytes / reported bytes (counters in KiB); tools/pmc_summary.py applies them per
kernel by its access pattern.
"""
import csv
import glob
import json
import os
import sys


def counter(d, sub):
    vals = {}
    for path in glob.glob(os.path.join(d, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"]) * 1024.0
    return vals


def main(d):
    known = json.load(open(os.path.join(d, "known.json")))
    fetch, write = counter(d, "fetch"), counter(d, "write")
    out = {"note": "factor = known bytes / counter bytes (FETCH_SIZE, WRITE_SIZE in KiB); "
                   "tools/pmc_calib.hip kernels on buffers beyond the 256 MiB Infinity Cache",
           "kernels": {}}
    for k, kb in known.items():
        ent = {}
        if "fetch" in kb:
            ent.update(known_fetch=kb["fetch"], fetch_size_bytes=fetch.get(k), fetch_factor=kb["fetch"] / fetch[k])
        if "write" in kb:
            ent.update(known_write=kb["write"], write_size_bytes=write.get(k), write_factor=kb["write"] / write[k])
        out["kernels"][k] = ent
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
