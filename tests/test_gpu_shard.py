"""Sharded GRank on the GPU: two ranks (gloo, sharing cuda:0 on a one-GPU box; RCCL on a node)
must reproduce the single-GPU result bit for bit."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PPR_DIST_BACKEND="gloo")
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import ShardedGrank
    import torch.distributed as dist
    g = ppr.rmat(12, seed=21)
    job = ShardedGrank(g, g.partitions(), 32, 64, 0.85, rank)  # gloo mode: ranks share cuda:0
    its = job.run(8, 1e-4)
    r = job.fetch()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), ids=r.ids, sc=r.scores, lens=r.lens, its=its)
    job.close()
    dist.destroy_process_group()


def test_gpu_sharded_equals_single(tmp_path):
    import approximated_personalized_pagerank_amd as ppr
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    g = ppr.rmat(12, seed=21)
    ref = ppr.grank_csr(g, 32, 64, 8, 0.85, 1e-4, device=0)
    for r in range(2):
        z = np.load(tmp_path / f"r{r}.npz")
        assert int(z["its"]) == ref.iterations_run
        assert np.array_equal(z["lens"], ref.lens)
        assert np.array_equal(z["ids"], ref.ids)
        assert np.array_equal(z["sc"], ref.scores)


def _worker_native(rank, world, port, outdir):
    # world 1 through the native (RCCL-mode) loop: ppr_grank_plan_run_sharded without a peer
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PPR_DIST_BACKEND="nccl")
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import ShardedGrank
    import torch.distributed as dist
    g = ppr.rmat(12, seed=21)
    job = ShardedGrank(g, g.partitions(), 32, 64, 0.85, rank)
    its = job.run(8, 1e-4)
    r = job.fetch()
    np.savez(os.path.join(outdir, f"n{rank}.npz"), ids=r.ids, sc=r.scores, lens=r.lens, its=its)
    job.close()
    dist.destroy_process_group()


def test_gpu_native_sharded_loop_single_rank(tmp_path):
    import approximated_personalized_pagerank_amd as ppr
    mp.spawn(_worker_native, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    g = ppr.rmat(12, seed=21)
    ref = ppr.grank_csr(g, 32, 64, 8, 0.85, 1e-4, device=0)
    z = np.load(tmp_path / "n0.npz")
    assert int(z["its"]) == ref.iterations_run
    assert np.array_equal(z["ids"], ref.ids) and np.array_equal(z["sc"], ref.scores)


@pytest.mark.parametrize("hot", [False, True])
def test_gpu_compact_block_round_trip(hot, monkeypatch):
    """Device pack -> host -> device unpack of compact blocks is lossless: plan B skips iteration
    0's merge and installs plan A's block instead; from there on both runs stay bit-identical
    (the unpack rebuilds each row's minimum and hash-range index the later merges use). The block
    decodes on the host (shard.unpack_block) to the rows fetch_slab reports."""
    if hot:  # stored ids carry the hot-key encoding from iteration 1 on
        monkeypatch.setenv("PPR_HOT_N", "64")
        monkeypatch.setenv("PPR_HOT_AT", "1")
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import GpuEngine, unpack_block
    g = ppr.rmat(13, seed=5)
    part = g.partitions()
    K, L, iters = 16, 32, 6
    a = ppr.GrankPlan(g, K, L, 0.85, part=part, device=0)
    b = ppr.GrankPlan(g, K, L, 0.85, part=part, device=0)
    ea, eb = GpuEngine(a), GpuEngine(b)
    a.init()
    b.init()
    for it in range(iters):
        n = a.active_count(it)
        a.iterate(it, 0, n)
        if it in (0, 3):  # B merges only the first half; the rest arrives as A's block
            h = n // 2
            b.iterate(it, 0, h)
            blk = ea.pack(it, h, n)
            assert len(blk) % 8 == 0 and len(blk) <= 8 + (n - h) * ea.row_bytes
            eb.unpack(it, h, n, blk)
            rows = unpack_block(blk, n - h)
            assert len(blk) == 8 * (n - h + 1) + sum(12 * len(i) + 4 * (len(i) & 1) for i, _ in rows)
        else:
            b.iterate(it, 0, n)
    a.finish(iters)
    b.finish(iters)
    ra, rb = a.fetch(), b.fetch()
    assert np.array_equal(ra.lens, rb.lens) and np.array_equal(ra.ids, rb.ids)
    assert np.array_equal(ra.scores.view(np.uint64), rb.scores.view(np.uint64))
    ref = ppr.grank_csr(g, K, L, iters, 0.85, -1.0, part=part, device=0)
    assert np.array_equal(ra.ids, ref.ids) and np.array_equal(ra.scores, ref.scores)
    a.close()
    b.close()


@pytest.mark.parametrize("world,tol", [(2, 1e-4), (3, -1.0), (4, 1e-3)])
def test_gpu_native_loop_multi_rank_local_group(world, tol):
    """ppr_grank_plan_run_sharded with world > 1 -- work-balanced ranges, compact blocks, size
    all-gather, block exchange, unpack, maxDiff all-reduce and the stop rule -- with `world` plans
    of this process as the ranks (device copies stand in for RCCL): every rank ends with the
    single-GPU result bit for bit"""
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import run_local_group
    g = ppr.rmat(13, seed=31)
    part = g.partitions()
    K, L, iters = 32, 64, 12
    ref = ppr.grank_csr(g, K, L, iters, 0.85, tol, part=part, device=0)
    plans = [ppr.GrankPlan(g, K, L, 0.85, part=part, device=0, stats=True) for _ in range(world)]
    st = run_local_group(plans, iters, tol)
    for pl, s in zip(plans, st):
        assert int(s.iterations_run) == ref.iterations_run
        r = pl.fetch()
        assert np.array_equal(r.lens, ref.lens) and np.array_equal(r.ids, ref.ids)
        assert np.array_equal(r.scores.view(np.uint64), ref.scores.view(np.uint64))
        pl.close()


@pytest.mark.parametrize("hot", [False, True])
def test_gpu_local_group_more_ranks_than_sources_past_256_iterations(hot, monkeypatch):
    """a rank with an empty source range must still reset the shared maxDiff slot of
    iterations >= 256 (PPR_MAX_ITER_STATS) and build the run's hot set. A 10-node ring at damping
    0.99 converges slowly enough that maxDiff stays > 0 past iteration 300; tol is set to the
    single-GPU maxDiff of iteration 300, so the stop falls beyond 256; 8 ranks share 5 active
    sources per iteration, so at least 3 ranks merge nothing. Every rank must stop at the same
    iteration as the single GPU and hold its result bit for bit."""
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import run_local_group
    if hot:
        monkeypatch.setenv("PPR_HOT_N", "4")
        monkeypatch.setenv("PPR_HOT_AT", "1")
    n = 10
    g = ppr.Csr(np.arange(n + 1, dtype=np.int64), np.array([(i + 1) % n for i in range(n)], dtype=np.int32))
    part = g.partitions()
    K, L, d, iters = 4, 8, 0.99, 420
    probe = ppr.GrankPlan(g, K, L, d, part=part, device=0)
    probe.init()
    md = []
    for it in range(320):
        probe.iterate(it, 0, probe.active_count(it))
        md.append(probe.read_maxdiff(it))
    probe.close()
    tol = md[300]
    assert tol > 0 and md[299] > tol
    ref = ppr.grank_csr(g, K, L, iters, d, tol, part=part, device=0)
    assert 256 < ref.iterations_run < iters
    plans = [ppr.GrankPlan(g, K, L, d, part=part, device=0) for _ in range(8)]
    st = run_local_group(plans, iters, tol)
    for pl, s in zip(plans, st):
        assert int(s.iterations_run) == ref.iterations_run
        r = pl.fetch()
        assert np.array_equal(r.lens, ref.lens) and np.array_equal(r.ids, ref.ids)
        assert np.array_equal(r.scores.view(np.uint64), ref.scores.view(np.uint64))
        pl.close()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_gpu_routed_exchange_bit_exact_and_smaller(world, monkeypatch):
    """consumer routing (a row goes only to the ranks whose sources read it; exact block sizes; the
    final rows broadcast once) ends every rank with the single-GPU result bit for bit, tolerance
    stop included, and moves fewer bytes than the broadcast exchange (PPR_XROUTE=0)"""
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import exchange_bytes, run_local_group
    g = ppr.rmat(14, seed=17)
    part = g.partitions()
    K, L, iters, tol = 32, 64, 9, 1e-5
    ref = ppr.grank_csr(g, K, L, iters, 0.85, tol, part=part, device=0)
    got = {}
    for route in ("1", "0"):
        monkeypatch.setenv("PPR_XROUTE", route)
        plans = [ppr.GrankPlan(g, K, L, 0.85, part=part, device=0) for _ in range(world)]
        st = run_local_group(plans, iters, tol)
        got[route] = max(exchange_bytes(pl)[0] for pl in plans)
        for pl, s in zip(plans, st):
            assert int(s.iterations_run) == ref.iterations_run
            r = pl.fetch()
            assert np.array_equal(r.lens, ref.lens) and np.array_equal(r.ids, ref.ids)
            assert np.array_equal(r.scores.view(np.uint64), ref.scores.view(np.uint64))
            pl.close()
    assert got["1"] < got["0"], got


@pytest.mark.parametrize("bad", [0, 3])
def test_gpu_routed_exchange_size_mismatch_fails_every_rank(bad, monkeypatch):
    """a block size that does not fit its receive slot must fail the run on EVERY rank
    (PPR_ERR_RANGE), not leave peers blocked in a half-posted exchange. Every rank checks the sizes
    it is about to receive and the ranks agree on the outcome before any block moves (an
    all-reduce MIN over RCCL; the host rendezvous here). PPR_XTEST_BADSIZE=r makes rank r advertise
    sizes 2^40 too large."""
    import time
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import run_local_group
    g = ppr.rmat(12, seed=5)
    part = g.partitions()
    monkeypatch.setenv("PPR_XROUTE", "1")
    monkeypatch.setenv("PPR_XTEST_BADSIZE", str(bad))
    plans = [ppr.GrankPlan(g, 16, 32, 0.85, part=part, device=0) for _ in range(4)]
    t0 = time.time()
    with pytest.raises(ppr.PprError) as e:
        run_local_group(plans, 4, -1.0)
    assert e.value.code == 11  # PPR_ERR_RANGE, not a barrier time-out
    assert time.time() - t0 < 60.0
    for pl in plans:
        pl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("rank,it", [(1, 0), (2, 5), (0, 11)])
def test_gpu_failing_rank_releases_every_rank(rank, it, monkeypatch):
    """a rank that fails inside the sharded loop (PPR_XTEST_FAIL="rank,it": that
    rank returns an error right after its merge of iteration it, before the exchange) must not
    strand its peers: every rank returns, promptly and with an error. Over RCCL the failing rank
    aborts its communicator and the peers' polling waits end (x_sync); in the in-process group the
    failure releases the barriers. Then the same plans run a clean job again, bit-exact."""
    import time
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import run_local_group
    g = ppr.rmat(12, seed=5)
    part = g.partitions()
    monkeypatch.setenv("PPR_XTEST_FAIL", f"{rank},{it}")
    plans = [ppr.GrankPlan(g, 16, 32, 0.85, part=part, device=0) for _ in range(3)]
    t0 = time.time()
    with pytest.raises(ppr.PprError):
        run_local_group(plans, 16, -1.0)
    assert time.time() - t0 < 60.0
    for pl in plans:
        pl.close()
    monkeypatch.delenv("PPR_XTEST_FAIL")
    ref = ppr.GrankPlan(g, 16, 32, 0.85, part=part, device=0)
    ref.run(16, -1.0)
    one = ref.fetch()
    ref.close()
    plans = [ppr.GrankPlan(g, 16, 32, 0.85, part=part, device=0) for _ in range(3)]
    run_local_group(plans, 16, -1.0)
    for pl in plans:
        r = pl.fetch()
        assert np.array_equal(r.ids, one.ids) and np.array_equal(r.scores.view(np.int64), one.scores.view(np.int64))
        pl.close()


@pytest.mark.gpu
def test_gpu_failing_rank_releases_every_rank_mc(monkeypatch):
    """The MC job's sharded loop likewise: rank 1 fails after its walks, before the walk-basket
    all-gather; every rank returns with an error instead of waiting for it."""
    import time
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import run_local_group_mc
    g = ppr.rmat(10, seed=2)
    monkeypatch.setenv("PPR_XTEST_FAIL", "1,0")
    plans = [ppr.MccpPlan(g, 8, 32, 0.85, device=0) for _ in range(3)]
    t0 = time.time()
    with pytest.raises(ppr.PprError):
        run_local_group_mc(plans, 100, 5)
    assert time.time() - t0 < 60.0
    for pl in plans:
        pl.close()


@pytest.mark.gpu
@pytest.mark.parametrize("var", ["PPR_XSHARD_ENDS", "PPR_XH_FIRST"])
def test_gpu_local_group_knobs_off_bit_exact(var, monkeypatch):
    """the non-sharded ends (x_exchange_bulk + a full top-K on every rank) and the
    sieve-first ordering are read per plan now, so a process can switch them: each off, LocalGroup
    world 3 equals the one-GPU run bit for bit."""
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd.shard import run_local_group
    g = ppr.rmat(13, seed=7)
    part = g.partitions()
    ref = ppr.GrankPlan(g, 32, 64, 0.85, part=part, device=0)
    ref.run(12, -1.0)
    one = ref.fetch()
    ref.close()
    monkeypatch.setenv(var, "0")
    plans = [ppr.GrankPlan(g, 32, 64, 0.85, part=part, device=0) for _ in range(3)]
    run_local_group(plans, 12, -1.0)
    for pl in plans:
        r = pl.fetch()
        assert np.array_equal(r.lens, one.lens)
        assert np.array_equal(r.ids, one.ids) and np.array_equal(r.scores.view(np.int64), one.scores.view(np.int64))
        pl.close()
