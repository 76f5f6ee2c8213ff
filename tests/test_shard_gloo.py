"""Source-sharded driver (approximated_personalized_pagerank_amd/shard.py) on CPU: world_size 2
gloo, the oracle as the per-rank engine. The sharded result must equal the single-process oracle
run bit for bit (Jacobi within a partition makes the sharding invisible)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import approximated_personalized_pagerank_amd as ppr
from approximated_personalized_pagerank_amd import shard
import oracle


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, scale, K, L, iters, tol, outdir):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    g = ppr.rmat(scale, seed=11)
    part = g.partitions()
    eng = oracle.OracleEngine(g.row_ptr, g.col, part, K, L, 0.85)
    comm = shard.TorchComm(torch.device("cpu"))
    w = shard.work_estimate(g.row_ptr, g.col, L)
    weights = [w[eng.active_list(p)] for p in (0, 1)]
    its = shard.run_sharded(eng, comm, iters, tol, weights)
    ids, sc, lens = eng.fetch()
    np.savez(os.path.join(outdir, f"r{rank}.npz"), ids=ids, sc=sc, lens=lens, its=its,
             md=np.array([eng.md[i] for i in range(its)]))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,scale,K,L,iters,tol", [(2, 9, 8, 16, 6, -1.0), (2, 10, 16, 32, 20, 1e-3),
                                                       (3, 9, 4, 8, 5, -1.0)])
def test_sharded_equals_single(tmp_path, world, scale, K, L, iters, tol):
    port = _free_port()
    mp.spawn(_worker, args=(world, port, scale, K, L, iters, tol, str(tmp_path)), nprocs=world, join=True)
    g = ppr.rmat(scale, seed=11)
    part = g.partitions()
    ref = oracle.grank(g.row_ptr, g.col, part, K, L, iters, 0.85, tol)
    for r in range(world):
        z = np.load(tmp_path / f"r{r}.npz")
        assert int(z["its"]) == ref["iterations_run"]
        assert np.array_equal(z["md"], ref["max_diff"])
        assert np.array_equal(z["lens"], ref["lens"])
        assert np.array_equal(z["ids"], ref["ids"])
        assert np.array_equal(z["sc"], ref["scores"])


def test_balanced_bounds():
    w = np.array([1, 1, 1, 100, 1, 1, 1, 1], dtype=float)
    b = shard.balanced_bounds(w, 2)
    assert b[0] == 0 and b[-1] == len(w) and b[1] in (4, 5)
    assert shard.balanced_bounds(np.zeros(0), 3) == [0, 0, 0, 0]
    b = shard.balanced_bounds(np.ones(10), 4)
    assert b == sorted(b) and b[-1] == 10


def test_compact_block_round_trip():
    """pack_block / unpack_block: empty rows, odd and even lengths, sizes 8 + 12 len (+4 if odd)"""
    rng = np.random.default_rng(3)
    rows = []
    for n in [0, 1, 2, 3, 7, 64, 0, 5]:
        rows.append((rng.integers(0, 1 << 30, n).astype(np.int32), rng.random(n)))
    blk = shard.pack_block(rows)
    assert len(blk) == 8 * (len(rows) + 1) + sum(12 * len(i) + 4 * (len(i) & 1) for i, _ in rows)
    assert len(blk) % 8 == 0
    back = shard.unpack_block(blk, len(rows))
    for (i0, s0), (i1, s1) in zip(rows, back):
        assert np.array_equal(i0, i1) and np.array_equal(s0.view(np.uint64), s1.view(np.uint64))
    assert shard.unpack_block(shard.pack_block([]), 0) == []
    assert len(shard.pack_block([])) == 8
