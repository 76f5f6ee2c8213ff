"""Source-sharded GRank over several GPUs (one process per GPU, torch.distributed over RCCL).

The reference parallelises the per-source merge with std::thread over static chunks of the active
partition (header-only/grankMulti.h:379-396) and joins every iteration. Here every rank holds the
whole graph and a replica of the basket slab, merges a contiguous, work-balanced range of the
iteration's active sources, and the rows it wrote are all-gathered so every replica enters the
next iteration with the complete state (Jacobi within a partition: an iteration only reads the
previous state, include/grank.h:96-126). maxDiff is all-reduced with MAX so the reference's
stopping rule (include/grank.h:90-94,140) is evaluated identically on every rank. The result is
bit-identical to the single-GPU run (the per-source maths does not depend on the sharding).

The driver is generic over an *engine* (GpuEngine below wraps GrankPlan; the CPU tests use the
oracle-backed oracle.OracleEngine) and a *comm* (all-gather of variable-size byte blocks,
all_reduce max). Rows travel as compact blocks (include/ppr_hip.h, ppr_grank_plan_pack): an int64
offset per row, then each row's ids and scores -- only the entries, 8 + 12 len bytes per row;
pack_block / unpack_block below are the format's host-side statement.
"""
from __future__ import annotations

import time
from typing import List, Sequence

import numpy as np


def work_estimate(row_ptr: np.ndarray, col: np.ndarray, L: int) -> np.ndarray:
    """Per-source merge work estimate: sum over successors of their initial basket size bound
    min(L, deg(u) + 1) (a dangling successor contributes 1)."""
    deg = np.diff(row_ptr)
    per_succ = np.minimum(L, deg + 1).astype(np.float64)
    src = np.repeat(np.arange(len(deg), dtype=np.int64), deg)
    w = np.bincount(src, weights=per_succ[col], minlength=len(deg))
    return w + 1.0


def balanced_bounds(weights: np.ndarray, world: int) -> List[int]:
    """Split a list into `world` contiguous ranges of roughly equal total weight."""
    n = len(weights)
    if n == 0:
        return [0] * (world + 1)
    cw = np.cumsum(weights)
    targets = cw[-1] * np.arange(1, world) / world
    cuts = np.searchsorted(cw, targets, side="left") + 1
    b = [0] + [int(min(max(c, 0), n)) for c in cuts] + [n]
    for i in range(1, len(b)):  # monotone
        b[i] = max(b[i], b[i - 1])
    return b


def pack_block(rows) -> np.ndarray:
    """Compact exchange block of a list of rows [(ids int32[len], scores f64[len]), ...] in stored
    order: int64 off[cnt + 1], then per row int32 ids padded to an even count and f64 scores."""
    sizes = np.array([12 * len(i) + 4 * (len(i) & 1) for i, _ in rows], dtype=np.int64)
    off = np.zeros(len(rows) + 1, dtype=np.int64)
    np.cumsum(sizes, out=off[1:])
    hdr = 8 * (len(rows) + 1)
    out = np.zeros(hdr + int(off[-1]), dtype=np.uint8)
    out[:hdr] = off.view(np.uint8)
    for r, (ids, sc) in enumerate(rows):
        n = len(ids)
        o = hdr + int(off[r])
        out[o:o + 4 * n] = np.ascontiguousarray(ids, dtype=np.int32).view(np.uint8)
        o += 4 * (n + (n & 1))
        out[o:o + 8 * n] = np.ascontiguousarray(sc, dtype=np.float64).view(np.uint8)
    return out


def unpack_block(block: np.ndarray, cnt: int):
    """Rows of a compact block of cnt rows (inverse of pack_block)."""
    block = np.asarray(block, dtype=np.uint8)
    hdr = 8 * (cnt + 1)
    off = block[:hdr].view(np.int64)
    rows = []
    for r in range(cnt):
        n = int((off[r + 1] - off[r]) // 12)
        o = hdr + int(off[r])
        ids = block[o:o + 4 * n].view(np.int32).copy()
        o += 4 * (n + (n & 1))
        rows.append((ids, block[o:o + 8 * n].view(np.float64).copy()))
    return rows


class TorchComm:  # collectives on torch tensors (tests; the GPU path never touches torch's HIP)
    """all-gather of variable-size blocks / all_reduce over torch.distributed (gloo on CPU)."""

    def __init__(self, device=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        self.device = device if device is not None else torch.device("cpu")
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def all_gather_blocks(self, block: np.ndarray) -> List[np.ndarray]:
        """Every rank's block (sizes all-gathered first, then the blocks padded to the largest)."""
        torch = self.torch
        sz = torch.tensor([len(block)], dtype=torch.int64, device=self.device)
        sizes = torch.empty(self.world, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(sizes, sz)
        sizes = [int(x) for x in sizes.cpu()]
        mx = max(sizes)
        if mx == 0:
            return [np.zeros(0, dtype=np.uint8) for _ in sizes]
        send = torch.zeros(mx, dtype=torch.uint8, device=self.device)
        send[:len(block)] = torch.from_numpy(np.ascontiguousarray(block)).to(self.device)
        out = torch.empty(self.world * mx, dtype=torch.uint8, device=self.device)
        self.dist.all_gather_into_tensor(out, send)
        out = out.cpu().numpy()
        return [out[r * mx:r * mx + sizes[r]] for r in range(self.world)]

    def all_reduce_max(self, x: float) -> float:
        torch = self.torch
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        self.dist.barrier()


def run_sharded(engine, comm, iterations: int, tolerance: float, weights, bounds=None) -> int:
    """GRank with the active sources of every iteration split over comm.world ranks.
    weights[p]: work estimate of partition p's active list (engine.active_list order), or
    bounds[p]: explicit range boundaries per partition. engine.pack(it, b, e) -> compact block
    (np.uint8) of the rows the rank wrote; engine.unpack(it, b, e, block) installs another rank's.
    Returns the number of iterations run."""
    rank, world = comm.rank, comm.world
    if bounds is None:
        bounds = [balanced_bounds(weights[p], world) for p in (0, 1)]
    engine.init()
    md = [tolerance, tolerance]
    it = 0
    while it < iterations and max(md) >= tolerance:
        bd = bounds[it & 1]
        b, e = bd[rank], bd[rank + 1]
        engine.iterate(it, b, e)
        if bd[world] > bd[0]:
            blocks = comm.all_gather_blocks(engine.pack(it, b, e))
            for r in range(world):
                if r != rank and bd[r + 1] > bd[r]:
                    engine.unpack(it, bd[r], bd[r + 1], blocks[r])
        engine.commit(it)
        d = comm.all_reduce_max(engine.read_maxdiff(it))
        engine.fold_maxdiff(it, d)
        md[0] = d
        md[0], md[1] = md[1], md[0]
        it += 1
    engine.finish(it)
    return it


class GpuEngine:
    """GrankPlan's step-level ABI with host-staged row exchange (single-GPU rehearsal over gloo;
    the production path is the native RCCL loop, ppr_grank_plan_run_sharded)."""

    def __init__(self, plan):
        from . import _lib
        import ctypes
        self.plan, self._lib, self._ct = plan, _lib, ctypes
        rb = ctypes.c_int64()
        _lib.check(_lib.lib().ppr_grank_plan_row_bytes(plan._p, ctypes.byref(rb)), "row_bytes")
        self.row_bytes = int(rb.value)

    def init(self):
        self.plan.init()

    def active_count(self, it):
        return self.plan.active_count(it)

    def active_list(self, it):
        n = self.plan.active_count(it)
        out = np.zeros(n, dtype=np.int32)
        self._lib.check(self._lib.lib().ppr_grank_plan_active_list(self.plan._p, it, self._lib.ptr(out)), "active_list")
        return out

    def iterate(self, it, b, e):
        self.plan.iterate(it, b, e)

    def pack(self, it, b, e):
        cap = 8 + max(0, e - b) * self.row_bytes
        out = np.empty(cap, dtype=np.uint8)
        nb = self._ct.c_int64(0)
        self._lib.check(self._lib.lib().ppr_grank_plan_pack_host(self.plan._p, it, b, e, self._lib.ptr(out), cap,
                                                                 self._ct.byref(nb)), "pack")
        return out[:nb.value]

    def unpack(self, it, b, e, block):
        block = np.ascontiguousarray(block, dtype=np.uint8)
        self._lib.check(self._lib.lib().ppr_grank_plan_unpack_host(self.plan._p, it, b, e, self._lib.ptr(block),
                                                                   len(block)), "unpack")

    def commit(self, it):
        pass  # the slot flip is implicit on the device

    def read_maxdiff(self, it):
        return self.plan.read_maxdiff(it)

    def fold_maxdiff(self, it, d):
        self._lib.check(self._lib.lib().ppr_grank_plan_fold_maxdiff(self.plan._p, it, d), "fold_maxdiff")

    def finish(self, iterations_run):
        self.plan.finish(iterations_run)


class CpuComm(TorchComm):
    """gloo collectives on host tensors (bootstrap and rehearsal)."""


def run_local_group(plans, iterations: int, tolerance: float):
    """The native sharded loop (ppr_grank_plan_run_sharded) with these GrankPlans of one process as
    its ranks, one thread each, blocks exchanged by device copies (tests: RCCL refuses two ranks
    on one GPU). Returns the per-rank PprStats."""
    import ctypes
    from . import _lib
    n = len(plans)
    arr = (ctypes.c_void_p * n)(*[pl._p for pl in plans])
    st = (_lib.PprStats * n)()
    _lib.check(_lib.lib().ppr_grank_plan_run_local_group(arr, n, iterations, tolerance, st), "run_local_group")
    for pl, s in zip(plans, st):
        pl.iterations_run = int(s.iterations_run)
    return list(st)


def run_local_group_mc(plans, walks: int, seed: int):
    """The sharded MC job (ppr_mccp2_plan_run_sharded) with these MccpPlans of one process as its
    ranks, one thread each (tests). Returns the per-rank McStats."""
    import ctypes
    from . import _lib
    from .mccp2 import McStats
    n = len(plans)
    arr = (ctypes.c_void_p * n)(*[pl._p for pl in plans])
    st = (_lib.PprMcStats * n)()
    _lib.check(_lib.lib().ppr_mccp2_plan_run_local_group(arr, n, walks, seed & 0xFFFFFFFFFFFFFFFF, st),
               "mccp2_run_local_group")
    return [McStats.of(s) for s in st]


def exchange_bytes(plan):
    """(block bytes this rank received, rows it sent) in the plan's last sharded run"""
    import ctypes
    from . import _lib
    rb, rs = ctypes.c_int64(), ctypes.c_int64()
    _lib.check(_lib.lib().ppr_grank_plan_exchange_bytes(plan._p, ctypes.byref(rb), ctypes.byref(rs)), "exchange_bytes")
    return int(rb.value), int(rs.value)


def device_count() -> int:
    import ctypes
    from . import _lib
    c = ctypes.c_int32(0)
    _lib.lib().ppr_device_count(ctypes.byref(c))
    return int(c.value)


class ShardedGrank:
    """Source-sharded GRank job of this rank. torch.distributed (gloo, host tensors only) is used
    to bootstrap: torch's own HIP runtime is never initialised in this process, all device work
    and the RCCL collectives run inside libppr_hip.so on the plan's stream.

    PPR_DIST_BACKEND=nccl (default): native loop, RCCL all-gather of rows over xGMI.
    PPR_DIST_BACKEND=gloo: Python loop, host-staged rows over gloo (lets several ranks share one
    GPU, which RCCL refuses)."""

    def __init__(self, g, part, K, L, damping, local):
        import os
        import ctypes
        import torch
        import torch.distributed as dist
        from . import _lib
        from .grank import GrankPlan
        self._lib, self._ct, self.torch, self.dist = _lib, ctypes, torch, dist
        if not dist.is_initialized():
            dist.init_process_group("gloo")
        self.comm = CpuComm()
        self.device = local % max(1, device_count())
        self.mode = os.environ.get("PPR_DIST_BACKEND", "nccl")
        self.plan = GrankPlan(g, K, L, damping, part=part, device=self.device, stats=True)
        if self.mode == "nccl" and self.comm.world > 1:
            uid = torch.zeros(128, dtype=torch.uint8)
            if self.comm.rank == 0:
                _lib.check(_lib.lib().ppr_comm_unique_id(uid.data_ptr()), "comm_unique_id")
            dist.broadcast(uid, 0)
            _lib.check(_lib.lib().ppr_grank_plan_comm_init(self.plan._p, uid.data_ptr(), self.comm.world,
                                                           self.comm.rank), "comm_init")
        self.eng = GpuEngine(self.plan)
        self.last_stats = None

    def run(self, iterations, tolerance):
        if self.mode == "nccl" or self.comm.world == 1:
            st = self._lib.PprStats()
            self._lib.check(self._lib.lib().ppr_grank_plan_run_sharded(self.plan._p, iterations, tolerance,
                                                                       self._ct.byref(st)), "run_sharded")
            self.plan.iterations_run = int(st.iterations_run)
            self.last_stats = st
            return int(st.iterations_run)
        weights = []
        for p in (0, 1):
            b = np.zeros(self.comm.world + 1, dtype=np.int64)
            self._lib.check(self._lib.lib().ppr_grank_plan_shard_bounds(self.plan._p, p, self.comm.world,
                                                                        self._lib.ptr(b)), "bounds")
            weights.append([int(x) for x in b])  # python ints: ctypes rejects numpy scalars
        its = run_sharded(self.eng, self.comm, iterations, tolerance, None, bounds=weights)
        self.plan.iterations_run = its
        return its

    def fetch(self):
        return self.plan.fetch()

    def close(self):
        self.plan.close()


class ShardedMccp:
    """The whole MCCompletePathV2 job of this rank (one process per GPU): walks of its walk-set range,
    walk baskets all-gathered over RCCL, the combine and top-K on every rank
    (ppr_mccp2_plan_run_sharded). torch.distributed (gloo) only carries the RCCL unique id."""

    def __init__(self, g, K, L, damping, local):
        import torch
        import torch.distributed as dist
        from . import _lib
        from .mccp2 import MccpPlan
        self._lib, self.torch, self.dist = _lib, torch, dist
        if not dist.is_initialized():
            dist.init_process_group("gloo")
        self.comm = CpuComm()
        self.device = local % max(1, device_count())
        self.plan = MccpPlan(g, K, L, damping, device=self.device)
        if self.comm.world > 1:
            uid = torch.zeros(128, dtype=torch.uint8)
            if self.comm.rank == 0:
                _lib.check(_lib.lib().ppr_comm_unique_id(uid.data_ptr()), "comm_unique_id")
            dist.broadcast(uid, 0)
            _lib.check(_lib.lib().ppr_grank_plan_comm_init(self.plan._p, uid.data_ptr(), self.comm.world,
                                                           self.comm.rank), "comm_init")

    def run(self, walks, seed):
        return self.plan.run_sharded(walks, seed)

    def fetch(self):
        return self.plan.fetch()

    def close(self):
        self.plan.close()


def run_distributed_bench(g, part, args, rank, world, local):
    """bench.py N>1 path: one source-sharded GRank job per step; (max elapsed, stats) on rank 0.
    The graph is generated identically on every rank (same seed)."""
    job = ShardedGrank(g, part, args.K, args.L, args.damping, local)
    for _ in range(args.warmup):
        job.run(args.iters, args.tol)
    job.comm.barrier()
    t0 = time.perf_counter()
    its = 0
    merge_ms = algo = 0.0
    for _ in range(args.steps):
        its = job.run(args.iters, args.tol)
        if job.last_stats is not None:
            merge_ms += job.last_stats.merge_ms
            algo += job.last_stats.algo_bytes
    el = time.perf_counter() - t0
    job.comm.barrier()
    elapsed = job.comm.all_reduce_max(el)
    # algorithmic bytes are per rank: the job's total is their sum; merge time is the max
    t = job.torch.tensor([algo], dtype=job.torch.float64)
    job.dist.all_reduce(t)
    algo_tot = float(t.item())
    merge_max = job.comm.all_reduce_max(merge_ms)
    job.close()
    job.dist.destroy_process_group()
    if rank != 0:
        return None
    return elapsed, dict(merge_ms=merge_max, algo_bytes=algo_tot, device_ms=elapsed * 1e3, iterations=its,
                         launches=0)
