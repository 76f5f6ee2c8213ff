"""Stamp a profile summary (JSON) with the source digest of the library it profiled, so a bench
line can tell whether its roofline.traffic came from the same kernels (bench.py traffic_same_build):

    python tools/stamp_build.py profiles/<round>_<workload>_pmc.json

Loads the in-tree library with ctypes only (no GPU call).
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from approximated_personalized_pagerank_amd import _lib  # noqa: E402

path = sys.argv[1]
info = _lib.lib().ppr_build_info().decode()
with open(path) as f:
    d = json.load(f)
d["build"] = info.split("ppr_src_sha256=")[1].split()[0]
with open(path, "w") as f:
    json.dump(d, f, indent=1)
    f.write("\n")
print(path, "build", d["build"])
