"""Build an experiment variant of the library beside the product one, for same-box A/B runs:

    python tools/build_variant.py NAME DEFINE [DEFINE ...]   # -> libppr_hip_NAME.so
    PPR_LIB_VARIANT=NAME python bench.py ...                  # loads the variant
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from approximated_personalized_pagerank_amd import build as b  # noqa: E402
from approximated_personalized_pagerank_amd._lib import PKG_DIR  # noqa: E402

name, defines = sys.argv[1], sys.argv[2:]
print(b.build(out=os.path.join(PKG_DIR, f"libppr_hip_{name}.so"), defines=defines, verbose=True))
