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
