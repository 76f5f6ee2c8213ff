"""Build an experiment variant of the library beside the product one, for same-box A/B runs:

    python tools/build_variant.py NAME [--rev GITREV] [DEFINE ...]   # -> libpprab_NAME.so (delete it after the A/B session)
    PPR_LIB_VARIANT=NAME python bench.py ...                          # loads the variant

--rev builds the sources of a git revision (exported to /tmp) instead of the working tree.
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from approximated_personalized_pagerank_amd import build as b  # noqa: E402
from approximated_personalized_pagerank_amd._lib import PKG_DIR  # noqa: E402

args = sys.argv[1:]
name = args.pop(0)
# the walk clears its flag bytes a dword per lane (merge_wave.h hub_window_walk_part): a batch that is
# not a multiple of 4 groups leaves stale flags and faults the GPU (round 6: PPR_TW_BATCH=6 did)
for d in args:
    if d.startswith("PPR_TW_BATCH=") and (int(d.split("=")[1]) % 4 or int(d.split("=")[1]) < 4):
        sys.exit("PPR_TW_BATCH must be a multiple of 4")
csrc = None
if args and args[0] == "--rev":
    rev = args[1]
    args = args[2:]
    tmp = f"/tmp/ppr_variant_{name}"
    subprocess.run(["rm", "-rf", tmp], check=True)
    os.makedirs(tmp)
    arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "include",
                           "approximated_personalized_pagerank_amd/csrc"], check=True, capture_output=True).stdout
    subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
    csrc = os.path.join(tmp, "approximated_personalized_pagerank_amd", "csrc")
print(b.build(out=os.path.join(PKG_DIR, f"libpprab_{name}.so"), defines=args, csrc=csrc, verbose=False))
