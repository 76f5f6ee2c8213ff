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
oracle-backed oracle.OracleEngine) and a *comm* (all_gather of byte rows, all_reduce max).
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


class TorchComm:
    """all_gather / all_reduce over torch.distributed (RCCL on GPUs, gloo on CPU)."""

    def __init__(self, device):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.device = torch, dist, device
        self.rank, self.world = dist.get_rank(), dist.get_world_size()

    def all_gather_rows(self, send, nbytes_max: int):
        torch = self.torch
        out = torch.empty(self.world * nbytes_max, dtype=torch.uint8, device=self.device)
        self.dist.all_gather_into_tensor(out, send)
        return out

    def all_reduce_max(self, x: float) -> float:
        torch = self.torch
        t = torch.tensor([x], dtype=torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def barrier(self):
        self.dist.barrier()


def run_sharded(engine, comm, iterations: int, tolerance: float, weights: Sequence[np.ndarray],
                alloc_send, to_engine_buf) -> int:
    """GRank with the active sources of every iteration split over comm.world ranks.
    weights[p]: work estimate of partition p's active list (engine.active_list order).
    alloc_send(nbytes) -> a send buffer the engine can pack into; to_engine_buf(t) -> what
    engine.unpack accepts. Returns the number of iterations run."""
    rank, world = comm.rank, comm.world
    bounds = [balanced_bounds(weights[p], world) for p in (0, 1)]
    rb = engine.row_bytes
    engine.init()
    md = [tolerance, tolerance]
    it = 0
    while it < iterations and max(md) >= tolerance:
        bd = bounds[it & 1]
        b, e = bd[rank], bd[rank + 1]
        engine.iterate(it, b, e)
        rows_max = max(bd[r + 1] - bd[r] for r in range(world))
        if rows_max > 0:
            send = alloc_send(rows_max * rb)
            engine.pack_into(it, b, e, send)
            recv = comm.all_gather_rows(send, rows_max * rb)
            for r in range(world):
                if r != rank and bd[r + 1] > bd[r]:
                    engine.unpack(it, bd[r], bd[r + 1], to_engine_buf(recv, r * rows_max * rb))
        engine.commit(it)
        d = comm.all_reduce_max(engine.read_maxdiff(it))
        engine.fold_maxdiff(it, d)
        md[0] = d
        md[0], md[1] = md[1], md[0]
        it += 1
    engine.finish(it)
    return it


class GpuEngine:
    """GrankPlan's step-level ABI with device row buffers from torch (plumbing only)."""

    def __init__(self, plan, torch, device):
        self.plan, self.torch, self.device = plan, torch, device
        from . import _lib
        import ctypes
        rb = ctypes.c_int64()
        _lib.check(_lib.lib().ppr_grank_plan_row_bytes(plan._p, ctypes.byref(rb)), "row_bytes")
        self.row_bytes = int(rb.value)
        self._lib, self._ct = _lib, ctypes

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

    def pack_into(self, it, b, e, send):
        self._lib.check(self._lib.lib().ppr_grank_plan_pack(self.plan._p, it, b, e, send.data_ptr()), "pack")

    def unpack(self, it, b, e, ptr):
        self._lib.check(self._lib.lib().ppr_grank_plan_unpack(self.plan._p, it, b, e, ptr), "unpack")

    def commit(self, it):
        pass  # the slot flip is implicit on the device

    def read_maxdiff(self, it):
        return self.plan.read_maxdiff(it)

    def fold_maxdiff(self, it, d):
        self._lib.check(self._lib.lib().ppr_grank_plan_fold_maxdiff(self.plan._p, it, d), "fold_maxdiff")

    def finish(self, iterations_run):
        self.plan.finish(iterations_run)


def _setup(local):
    """device for this rank (ranks beyond the visible GPUs share them: rehearsal on one GPU) and
    the process group (PPR_DIST_BACKEND, default nccl = RCCL on ROCm)."""
    import os
    import torch
    import torch.distributed as dist
    ndev = max(1, torch.cuda.device_count())
    dev = torch.device("cuda", local % ndev)
    torch.cuda.set_device(dev)
    if not dist.is_initialized():
        backend = os.environ.get("PPR_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    return dev


class ShardedGrank:
    """Sharded GRank job on this rank's GPU (torch.distributed must be launched)."""

    def __init__(self, g, part, K, L, damping, local):
        import torch
        from .grank import GrankPlan
        self.torch = torch
        self.dev = _setup(local)
        self.comm = TorchComm(self.dev)
        # one dedicated stream for the library's kernels and torch's collectives, so packing, the
        # all-gather and unpacking are ordered (the legacy default stream would be handle 0, which
        # the ABI reads as "library-owned stream")
        self.stream = torch.cuda.Stream(device=self.dev)
        self.plan = GrankPlan(g, K, L, damping, part=part, device=self.dev.index,
                              stream=self.stream.cuda_stream)
        self.eng = GpuEngine(self.plan, torch, self.dev)
        w = work_estimate(g.row_ptr, g.col, L)
        self.weights = [w[self.eng.active_list(p)] for p in (0, 1)]
        self._bufs = {}
        self.gloo = self.comm.dist.get_backend() == "gloo"

    def _alloc(self, nbytes):
        t = self._bufs.get(nbytes)
        if t is None:
            t = self._bufs[nbytes] = self.torch.empty(nbytes, dtype=self.torch.uint8, device=self.dev)
        return t

    def run(self, iterations, tolerance):
        torch = self.torch

        def to_buf(recv, off):
            return recv.data_ptr() + off

        comm = self.comm
        if self.gloo:  # gloo: host staging of the row buffers
            class HostComm:
                rank, world = comm.rank, comm.world

                def all_gather_rows(_, send, nb):
                    torch.cuda.synchronize(self.dev)
                    host = send.cpu()
                    out = torch.empty(comm.world * nb, dtype=torch.uint8)
                    comm.dist.all_gather_into_tensor(out, host)
                    return out.to(self.dev)

                def all_reduce_max(_, x):
                    t = torch.tensor([x], dtype=torch.float64)
                    comm.dist.all_reduce(t, op=comm.dist.ReduceOp.MAX)
                    return float(t.item())

                def barrier(_):
                    comm.dist.barrier()
            use = HostComm()
        else:
            use = comm
        with torch.cuda.stream(self.stream):
            its = run_sharded(self.eng, use, iterations, tolerance, self.weights, self._alloc, to_buf)
        torch.cuda.synchronize(self.dev)
        return its

    def fetch(self):
        return self.plan.fetch()

    def close(self):
        self.plan.close()


def run_distributed_bench(g, part, args, rank, world, local):
    """bench.py N>1 path: source-sharded GRank job per step; returns (max elapsed, stats) on
    rank 0. The graph is generated identically on every rank (same seed)."""
    import torch
    import torch.distributed as dist
    job = ShardedGrank(g, part, args.K, args.L, args.damping, local)
    dev = job.dev
    for _ in range(args.warmup):
        job.run(args.iters, args.tol)
    torch.cuda.synchronize(dev)
    job.comm.barrier()
    t0 = time.perf_counter()
    its = 0
    for _ in range(args.steps):
        its = job.run(args.iters, args.tol)
    torch.cuda.synchronize(dev)
    job.comm.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if job.gloo:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    else:
        el = el.to(dev)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    job.close()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return elapsed, dict(merge_ms=0.0, algo_bytes=0, device_ms=elapsed * 1e3, iterations=its, launches=0)
