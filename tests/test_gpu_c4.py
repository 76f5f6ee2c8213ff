"""C4 (BASELINE.json configs[3]) at full size on one GPU: RMAT-22 K64/L128/30 iterations through
the source-sharded native loop (ppr_grank_plan_run_sharded) with 8 ranks -- 8 plans of this
process, one thread each (LocalGroup: device copies stand in for RCCL, which refuses two ranks on
one GPU). This exercises what only full size shows: the RMAT-22 shard bounds
(header-only/grankMulti.h:376-396 splits sources the same way), compact blocks of 340 MB per rank
and 2.4 GB receive buffers per A-iteration, and the unpack of 7/8 of every iteration's rows.
Every rank must end with the CPU oracle's whole-run result bit for bit (digests from
tools/make_c3_digest.py, the same the one-GPU C3 test checks).

Memory: a plan holds the two-slot slab (12.9 GB), the range index (1.1 GB), the exchange buffers
(about 2.8 GB) and the hub scratch regions of its merge calls -- up to ~7.5 GB each at the default
2^28-candidate batches, two of them for a 1/8 range. Eight such ranks would need ~280 GB of the
288 GB, so this test halves the batch budget (PPR_HUB_BUDGET = 2^27: batching never changes a
result, tests/test_gpu_parity.py): ~22 GB per rank, ~180 GB for 8.
"""
import json
import os
import sys
import time

import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr
from helpers import GOLDEN

pytestmark = pytest.mark.gpu

# the default summation mode's whole-run digest (the exact sum; the chain-order digest is checked
# on one GPU by tests/test_gpu_scale.py -- the sharded loop does not depend on the mode)
C3_DIGESTS = [f for f in ("c3_rmat22_k64_l128_i30_exact.json",) if os.path.exists(os.path.join(GOLDEN, f))]


def progress(msg):
    print(f"[c4] {msg}", file=sys.__stderr__, flush=True)


def _dig(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


@pytest.mark.parametrize("digest", C3_DIGESTS)
def test_gpu_c4_rmat22_eight_ranks_equal_oracle(digest, monkeypatch):
    from approximated_personalized_pagerank_amd.shard import run_local_group
    monkeypatch.setenv("PPR_HUB_BUDGET", str(1 << 27))
    with open(os.path.join(GOLDEN, digest)) as f:
        ref = json.load(f)
    world = 8
    t0 = time.time()
    g = ppr.rmat(ref["scale"], seed=ref["seed"])
    part = g.partitions()
    assert (g.n, g.m, _dig(g.col)) == (ref["n"], ref["m"], ref["graph_sha256"])
    K, L, d = ref["K"], ref["L"], ref["damping"]
    plans = [ppr.GrankPlan(g, K, L, d, part=part, device=0, stats=True, sum_mode=ref.get("sum", "chain"))
             for _ in range(world)]
    progress(f"graph + {world} plans {time.time() - t0:.1f} s")
    t1 = time.time()
    st = run_local_group(plans, ref["iters"], ref["tol"])
    progress(f"{world}-rank sharded job (one GPU) {time.time() - t1:.1f} s")
    for rank, (pl, s) in enumerate(zip(plans, st)):
        assert int(s.iterations_run) == ref["iterations_run"], rank
        assert [float(x).hex() for x in s.max_diff[: ref["iterations_run"]]] == ref["max_diff"], rank
        r = pl.fetch()
        assert _dig(r.lens) == ref["lens_sha256"], rank
        assert _dig(r.ids) == ref["ids_sha256"], rank
        assert _dig(r.scores) == ref["scores_sha256"], rank
        pl.close()
    progress(f"every rank == oracle ({time.time() - t0:.1f} s)")
