"""C5 (BASELINE.json configs[4]) as a whole multi-rank job: MCCompletePathV2 on RMAT-22 through
ppr_mccp2_plan_run_sharded with 8 ranks -- 8 MC plans of this process, one thread each (LocalGroup:
device copies stand in for RCCL, which refuses two ranks on one GPU). Each rank walks 1/8 of the
walk set, the walk baskets are all-gathered as compact blocks, every rank runs the combine and
the top-K. Every rank must equal the one-GPU job bit for bit (the walks are keyed by seed, step,
walk and source, not by the rank that runs them).

Memory: an MC plan holds the two-slot slab (n * L * 24 B: 6.4 GB at L = 64, 20 GB at L = 200), the
range index (1.1 GB), the walk-basket exchange buffers (7/8 of the walk rows) and its hub scratch.
Eight ranks run at L = 64 (~12 GB each); the configs[4] row width L = 200 runs with 2 ranks.
"""
import sys
import time

import numpy as np
import pytest

import approximated_personalized_pagerank_amd as ppr

pytestmark = pytest.mark.gpu


def progress(msg):
    print(f"[c5x] {msg}", file=sys.__stderr__, flush=True)


@pytest.mark.parametrize("world,K,L", [(8, 50, 64), (2, 50, 200)])
def test_gpu_c5_rmat22_sharded_mc_job_equals_one_gpu(world, K, L, monkeypatch):
    from approximated_personalized_pagerank_amd.shard import exchange_bytes, run_local_group_mc
    monkeypatch.setenv("PPR_HUB_BUDGET", str(1 << 26))  # (batching never changes a result)
    R, d, seed = 1000, 0.85, 11
    t0 = time.time()
    g = ppr.rmat(22, seed=1)
    one = ppr.MccpPlan(g, K, L, d, device=0)
    st1 = one.run(R, seed)
    r1 = one.fetch()
    one.close()
    progress(f"one GPU: {st1.device_ms:.0f} ms (walks {st1.walk_ms:.0f}, combine {st1.combine_ms:.0f}) "
             f"[{time.time() - t0:.1f} s]")
    plans = [ppr.MccpPlan(g, K, L, d, device=0) for _ in range(world)]
    t1 = time.time()
    st = run_local_group_mc(plans, R, seed)
    progress(f"{world} ranks on one GPU: {time.time() - t1:.1f} s")
    wb = st1.walk_nodes
    rows = 0
    for rank, pl in enumerate(plans):
        r = pl.fetch()
        assert np.array_equal(r.lens, r1.lens), rank
        assert np.array_equal(r.ids, r1.ids), rank
        assert np.array_equal(r.scores.view(np.int64), r1.scores.view(np.int64)), rank
        recv, sent = exchange_bytes(pl)
        rows += sent
        progress(f"rank {rank}: walked {st[rank].walks} walks, sent {sent} walk rows, received {recv / 1e9:.3f} GB")
        pl.close()
    assert rows == wb
    assert sum(s.walks for s in st) == st1.walks
