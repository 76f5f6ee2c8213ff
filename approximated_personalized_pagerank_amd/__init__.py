"""MI355X-native all-sources approximate Personalized PageRank (GRank / MCCompletePathV2).

Drop-in surface of fruttasecca/approximated_personalized_pagerank:
  * C++: include/ppr/grank.h, include/ppr/grankMulti.h (same templates, same signatures)
  * C ABI: include/ppr_hip.h (libppr_hip.so, built in-tree for gfx950)
  * Python: grank / grank_multi / GrankPlan below.
"""
from ._lib import PprError
from .graph import Csr, read_edge_csv, rmat
from .grank import GrankPlan, GrankResult, grank, grank_csr, grank_multi

__all__ = [
    "PprError", "Csr", "rmat", "read_edge_csv", "GrankPlan", "GrankResult", "grank", "grank_csr",
    "grank_multi",
]
