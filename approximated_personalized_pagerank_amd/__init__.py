"""MI355X-native all-sources approximate Personalized PageRank (GRank / MCCompletePathV2).

Drop-in surface of fruttasecca/approximated_personalized_pagerank:
  * C++: include/ppr/grank.h, include/ppr/grankMulti.h (same templates, same signatures)
  * C ABI: include/ppr_hip.h (libppr_hip.so, built in-tree for gfx950)
  * Python: grank / grank_multi / GrankPlan / mccompletepathv2 / MccpPlan below, and the
    reference's quality harness (exact PPR, batched on the GPU; benchmark_algorithm).
"""
from ._lib import PprError
from .graph import Csr, import_edge_csv, read_edge_csv, rmat
from .grank import GrankPlan, GrankResult, grank, grank_csr, grank_multi
from .mccp2 import MccpPlan, McStats, mccompletepathv2, mccp2_csr
from .exact import ExactPPR, benchmark_algorithm, jaccard, kendall_correlation

__all__ = [
    "PprError", "Csr", "rmat", "read_edge_csv", "import_edge_csv", "GrankPlan", "GrankResult", "grank", "grank_csr",
    "grank_multi", "MccpPlan", "McStats", "mccompletepathv2", "mccp2_csr", "ExactPPR", "benchmark_algorithm",
    "jaccard", "kendall_correlation",
]
