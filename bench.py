#!/usr/bin/env python3
"""bench.py -- GRank all-sources approximate PPR on synthetic RMAT (BASELINE.json metric).

Metric: source-nodes/sec of ppr::grank K=64 L=128 30 iterations on RMAT-22 (configs[2]),
whole-job throughput with the graph already resident in HBM: one "step" = one complete GRank
job on the device (init baskets + 30 iterations of the basket merge + final top-K).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scale 22] [--K 64] [--L 128] [--iters 30]

N > 1 (torch.distributed.run, one rank per GPU over RCCL): every rank holds the graph and a
slab replica, merges a contiguous shard of each iteration's active sources, and the updated
basket rows are all-gathered (approximated_personalized_pagerank_amd/shard.py).
value = |V| * steps / max-over-ranks time; scaling "strong" (the job is fixed, sources split).

Extra objects on the JSON line (DESIGN.md "measurement"):
  roofline      merge phase: SURVEY s8d algorithmic bytes / merge-phase time (hipEvents on the
                plan's stream), against 8 TB/s HBM
  end_to_end    the reference's API end to end (tests/cpp/dropin_test.cc: unordered_map graph in,
                unordered_map result out) with its flatten / plan / device / materialise split
  cpu_baseline  the reference's own combineMaps (oracle/_ref/ref_driver, compiled from
                /root/reference) timed on a stratified sample of the end-state workload on this
                host, extrapolated to the whole job
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
PROFILES = os.path.join(ROOT, "profiles")


def sum_mode():
    """the GRank summation mode the plans of this process use (include/ppr_hip.h PPR_FLAG_CHAIN_SUM;
    PPR_SUM overrides the default, the exact sum)"""
    return "chain" if os.environ.get("PPR_SUM") == "chain" else "exact"


def pmc_traffic(tag, mode):
    """HBM bytes per step of the merge phase from the newest committed rocprofv3 PMC summary of this
    workload in this summation mode (tools/pmc_summary.py: 2 x FETCH_SIZE + WRITE_SIZE, separate
    passes; a summary without a "sum" field predates the exact sum: chain), its path and the source
    digest of the library it profiled (tools/gpu_run.sh pmc stamps it), or None."""
    import glob
    for path in sorted(glob.glob(os.path.join(PROFILES, f"*_{tag}_pmc.json")), reverse=True):
        with open(path) as f:
            d = json.load(f)
        if d.get("sum", "chain") == mode:
            return d.get("merge_phase_traffic_bytes"), os.path.relpath(path, ROOT), d.get("build")
    return None, None, None


def kernel_groups(kst, merge_ms, steps):
    """Per kernel group of the merge phase: algorithmic bytes and time per step, and the roofline
    fraction on that time.

    The library times each group with HIP events around its launches on its own stream
    (ppr_grank_plan_kernel_stats). The groups run concurrently on four streams, so those spans
    overlap: they summed to about twice the phase. Each group's `ms_per_step` is therefore its share
    of the phase: its span times phase / (sum of the spans), i.e. concurrent groups split the time
    they share in proportion to how long each was resident. The shares sum to the phase, never past
    the summed kernel time, and `span_ms_per_step` keeps the raw span. The three one-slice sieve
    classes are one group here ("sieve one-slice k_sv1+k_svfin"): they are the same kernel,
    k_sv1, at three launch geometries, so the dominant group matches rocprof's top kernel; the
    classes stay listed under `classes`."""
    groups = {}
    for k, v in kst.items():
        name = "sieve one-slice k_sv1+k_svfin" if k.startswith("sieve") and "k_sv1" in k else k
        g = groups.setdefault(name, {"algo_bytes": 0.0, "ms": 0.0, "launches": 0, "classes": {}})
        g["algo_bytes"] += v["algo_bytes"]
        g["ms"] += v["ms"]
        g["launches"] += v["launches"]
        if name != k:
            g["classes"][k] = {"algo_bytes_per_step": v["algo_bytes"] / steps, "span_ms_per_step": v["ms"] / steps}
    span_sum = sum(g["ms"] for g in groups.values())
    scale = merge_ms / span_sum if span_sum > 0 else 0.0
    out = {}
    for k, g in groups.items():
        if g["ms"] <= 0:
            continue
        share = g["ms"] * scale
        gbs = g["algo_bytes"] / 1e9 / (share / 1e3) if share > 0 else 0.0
        out[k] = {"algo_bytes_per_step": g["algo_bytes"] / steps, "ms_per_step": share / steps,
                  "span_ms_per_step": g["ms"] / steps, "launches_per_step": g["launches"] / steps,
                  "achieved": gbs, "frac": gbs / HBM_PEAK_GBS}
        if g["classes"]:
            out[k]["classes"] = g["classes"]
    return out


def lib_build():
    """source digest of the loaded HIP library (ppr_build_info: ppr_src_sha256=...)"""
    from approximated_personalized_pagerank_amd import _lib
    info = _lib.lib().ppr_build_info().decode()
    return info.split("ppr_src_sha256=")[1].split()[0] if "ppr_src_sha256=" in info else None


def mc_cpu_baseline(scale, K, L, walks, damping, seed):
    """The reference's own mccompletepathv2 (single-threaded by design, include/mccompletepathv2.h)
    compiled from /root/reference (oracle/_ref/ref_driver), timed on a bounded RMAT sample."""
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    if not os.path.exists(drv):
        return None
    import approximated_personalized_pagerank_amd as ppr
    g = ppr.rmat(scale, seed=seed)
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "g.bin")
        with open(path, "wb") as f:
            np.array([g.n, g.m], dtype=np.int64).tofile(f)
            np.arange(g.n, dtype=np.int32).tofile(f)
            g.row_ptr.astype(np.int64).tofile(f)
            g.col.astype(np.int32).tofile(f)
        t0 = time.time()
        subprocess.run([drv, "mc", path, os.path.join(td, "o.bin"), str(K), str(L), str(walks), repr(damping),
                        "-1", "1"], check=True, capture_output=True)
        wall = time.time() - t0
    return {"value": g.n / wall, "unit": "source-nodes/s", "cores": 1, "kind": "reference",
            "sample": (f"reference ppr::mccompletepathv2 (include/mccompletepathv2.h, -O3 -march=x86-64-v3, "
                       f"sequential by design) whole job on RMAT-{scale} ({g.n} nodes, {g.m} edges, same K/L/R/d), "
                       f"{wall:.1f} s incl. graph load; its per-node cost grows with scale (1.5x per 2 scales "
                       f"measured at RMAT-14..18), so this overstates the RMAT-22 rate")}


def parse_ppr_timing(text):
    """key -> seconds from the library's PPR_TIMING lines ("ppr_timing [section] key value ...")"""
    split = {}
    for ln in text.splitlines():
        if not ln.startswith("ppr_timing"):
            continue
        f = ln.split()[1:]
        i = 0
        while i + 1 < len(f):
            try:
                split[f[i]] = float(f[i + 1])
                i += 2
            except ValueError:
                i += 1
    return split


def end_to_end(scale, iters, K, L):
    """f1: the reference's own API end to end -- tests/cpp/dropin_test.cc calls
    ppr::grank(unordered_map graph, K=64, L=128, iters) through include/ppr/grank.h, so the timing
    covers flattening the map graph, plan creation + upload, the device job and materialising the
    unordered_map<int, unordered_map<int, double>> result (PPR_TIMING=1 split)."""
    if (K, L) != (64, 128):
        return None
    from approximated_personalized_pagerank_amd import build as _build
    binary = _build.build_dropin()
    # PPR_HEAP_PAD: the result maps' malloc heaps grow 64 MB at a time (include/ppr/grank.h HeapGrowth,
    # opt-in because mallopt is process-wide; this program sets nothing else)
    env = dict(os.environ, PPR_TIMING="1", PPR_HEAP_PAD=os.environ.get("PPR_HEAP_PAD", "64"))
    p = subprocess.run([binary, "e2e", str(scale), str(iters)], capture_output=True, text=True, env=env,
                       check=True, timeout=900)
    d = json.loads(p.stdout.strip().splitlines()[-1])
    split = parse_ppr_timing(p.stderr)
    out = {"total_s": d["total_s"], "graph": "RMAT-%d as unordered_map<int, vector<int>> (%d nodes, %d edges)"
           % (scale, d["nodes"], d["edges"]), "result_entries": d["entries"],
           "call": f"ppr::grank(graph, K={K}, L={L}, {iters}, 0.85, -1) via include/ppr/grank.h",
           "env": {"PPR_HEAP_PAD": env["PPR_HEAP_PAD"]}}
    if split:
        out.update(flatten_s=split.get("flatten_s"), device_s=split.get("device_s"),
                   plan_and_upload_s=split["csr_call_s"] - split["device_s"] if "csr_call_s" in split else None,
                   materialize_s=split.get("materialize_s"),
                   plan_create={k: split[k] for k in ("partitions_s", "colx_s", "alloc_upload_s", "work_s")
                                if k in split})
    return out


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def host_cpus():
    """Host threads this process may run on: the CPU affinity set, capped by a cgroup v2 CPU
    quota when one is set (a GPU box shares its host between GPUs), and the CPU model name."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = max(1, min(n, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return n, model


# ------------------------------------------------------------------------------------------
# CPU baseline: reference combineMaps on a stratified sample (rank 0, N=1 only)
def cpu_baseline(g, part, slab, L, damping, iters, threads, budget, seed=0):
    drv = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
    if not os.path.exists(drv):
        return None
    ids, sc, lens = slab
    rp, col = g.row_ptr, g.col
    deg = np.diff(rp)
    src_of_edge = np.repeat(np.arange(g.n, dtype=np.int64), deg)
    cand = np.bincount(src_of_edge, weights=lens[col].astype(np.float64), minlength=g.n)
    work = cand + deg
    rng = np.random.default_rng(seed)
    strata = []  # (partition, population count, sample array)
    n_strata = 4
    for p in (0, 1):
        act = np.nonzero((part == p) & (deg > 0))[0]
        if len(act) == 0:
            continue
        order = act[np.argsort(-work[act], kind="stable")]
        cw = np.cumsum(work[order])
        cuts = np.searchsorted(cw, cw[-1] * np.arange(1, n_strata) / n_strata)
        bounds = [0] + sorted(set(int(c) + 1 for c in cuts)) + [len(order)]
        bounds = sorted(set(min(b, len(order)) for b in bounds))
        for h in range(len(bounds) - 1):
            pop = order[bounds[h]:bounds[h + 1]]
            if len(pop) == 0:
                continue
            mean_w = work[pop].mean()
            k = int(min(len(pop), max(2, np.ceil(budget / (2 * n_strata) / max(mean_w, 1.0)))))
            smp = pop if k == len(pop) else rng.choice(pop, k, replace=False)
            strata.append((p, len(pop), np.sort(smp)))
    src = np.concatenate([s for _, _, s in strata]).astype(np.int32)
    off = np.cumsum([0] + [len(s) for _, _, s in strata]).astype(np.int64)
    srp = np.zeros(len(src) + 1, dtype=np.int64)
    srp[1:] = np.cumsum(deg[src])
    succ = np.concatenate([col[rp[v]:rp[v + 1]] for v in src]).astype(np.int32)
    need = np.unique(np.concatenate([src, succ]))
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sample.bin")
        with open(path, "wb") as f:
            np.array([L], dtype=np.int32).tofile(f)
            np.array([len(src)], dtype=np.int64).tofile(f)
            src.tofile(f)
            srp.tofile(f)
            succ.tofile(f)
            np.array([len(need)], dtype=np.int64).tofile(f)
            for v in need:
                ln = int(lens[v])
                np.array([v, ln], dtype=np.int32).tofile(f)
                ids[v, :ln].tofile(f)
                sc[v, :ln].tofile(f)
            np.array([len(strata)], dtype=np.int64).tofile(f)
            off.tofile(f)
        t0 = time.time()
        out = subprocess.run([drv, "bench_combine", path, str(threads), repr(damping)], check=True,
                             capture_output=True, text=True).stdout
        wall = time.time() - t0
    rows = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    per_part = {0: 0.0, 1: 0.0}
    sampled_ms = 0.0
    for (p, pop, smp), r in zip(strata, rows):
        per_part[p] += pop / len(smp) * r["ms"]
        sampled_ms += r["ms"]
    iters_p = {0: (iters + 1) // 2, 1: iters // 2}
    job_ms = sum(iters_p[p] * per_part[p] for p in (0, 1))
    n_act = int(((deg > 0)).sum())
    return {
        "value": g.n / (job_ms / 1e3),
        "unit": "source-nodes/s",
        "cores": threads,
        "cpu_model": host_cpus()[1],
        "kind": "reference",
        "sample": (f"reference grankMultiInternal::combineMaps (header-only/grankMulti.h:230-268, "
                   f"-O3 -march=x86-64-v3) on {len(src)} of {n_act} active sources: {len(strata)} work "
                   f"strata (4 per partition), end-state L={L} baskets; {sampled_ms / 1e3:.1f} s timed of "
                   f"{wall:.1f} s wall; whole job extrapolated as {iters_p[0]} A + {iters_p[1]} B "
                   f"iterations = {job_ms / 1e3:.0f} s (init, partitions and the final top-K excluded)"),
    }


def main_mc(args):
    """MCCompletePathV2 on RMAT (configs[4]): one step = walks of the whole walk set + the
    level-synchronous combine + top-K, graph and plan resident. N > 1: the whole job on every rank
    (ppr_mccp2_plan_run_sharded): each rank walks a contiguous range of the walk set, the walk
    baskets are all-gathered over RCCL, and every rank runs the level-sequential combine."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    K = args.K if args.K != 64 else 50
    L = args.L if args.L != 128 else 200
    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd import build as _build
    if rank == 0:
        _build.build()
    t = time.time()
    g = ppr.rmat(args.scale, seed=args.seed)
    plan = ppr.MccpPlan(g, K, L, args.damping, device=local)
    log(f"[rank {rank}] RMAT-{args.scale}: n={g.n} m={g.m} walk set={plan.walk_nodes} levels={plan.levels} "
        f"dangling={plan.dangling} prep {time.time() - t:.1f}s")
    if world > 1:
        # the whole job on every step: walks of this rank's walk-set range, walk baskets all-gathered
        # over RCCL, the combine and top-K on every rank (ppr_mccp2_plan_run_sharded)
        from approximated_personalized_pagerank_amd.shard import ShardedMccp, exchange_bytes
        plan.close()
        job = ShardedMccp(g, K, L, args.damping, local)
        for _ in range(args.warmup):
            job.run(args.walks, 1)
        job.comm.barrier()
        t0 = time.perf_counter()
        walk_ms = comb_ms = 0.0
        for s in range(args.steps):
            st = job.run(args.walks, 1 + s)
            walk_ms += st.walk_ms
            comb_ms += st.combine_ms
        el = time.perf_counter() - t0
        job.comm.barrier()
        elapsed = job.comm.all_reduce_max(el)
        walk_max = job.comm.all_reduce_max(walk_ms)
        comb_max = job.comm.all_reduce_max(comb_ms)
        xb = job.comm.all_reduce_max(float(exchange_bytes(job.plan)[0]))
        job.close()
        job.dist.destroy_process_group()
        if rank != 0:
            return
        line = {
            "metric": "source-nodes/sec mccompletepathv2 K=50 L=200 R=1000 on RMAT-22",
            "value": g.n * args.steps / elapsed, "unit": "source-nodes/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic RMAT (Graph500 a=.57 b=.19 c=.19, edge factor 16, seed %d, dedup)" % args.seed,
            "config": {"workload": f"mccompletepathv2 RMAT-{args.scale} K={K} L={L} R={args.walks} d={args.damping}",
                       "nodes": g.n, "edges": g.m, "walk_nodes": st.walk_nodes, "levels": st.levels,
                       "parallelism": f"walk-shard x{world} + walk-basket all-gather + replicated combine"},
            "phases": {"walk_ms_per_step": walk_max / args.steps, "combine_ms_per_step": comb_max / args.steps,
                       "walk_basket_bytes_received_per_rank": xb},
        }
        print(json.dumps(line), flush=True)
        return
    for _ in range(args.warmup):
        plan.run(args.walks, 1)
    walk_ms = comb_ms = 0.0
    t0 = time.perf_counter()
    for s in range(args.steps):
        st = plan.run(args.walks, 1 + s)
        walk_ms += st.walk_ms
        comb_ms += st.combine_ms
    elapsed = time.perf_counter() - t0
    steps = args.steps
    cpu = None
    if not args.no_cpu_baseline:
        try:
            plan.close()
            cpu = mc_cpu_baseline(max(8, args.scale - 6), K, L, args.walks, args.damping, args.seed)
        except Exception as exc:  # reported, never fatal
            log(f"mc cpu_baseline failed: {exc!r}")
    line = {
        "metric": "source-nodes/sec mccompletepathv2 K=50 L=200 R=1000 on RMAT-22",
        "value": g.n * steps / elapsed, "unit": "source-nodes/s", "n_gpus": 1, "steps": steps,
        "warmup": args.warmup, "ms_per_step": elapsed * 1e3 / steps, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic RMAT (Graph500 a=.57 b=.19 c=.19, edge factor 16, seed %d, dedup)" % args.seed,
        "config": {"workload": f"mccompletepathv2 RMAT-{args.scale} K={K} L={L} R={args.walks} d={args.damping}",
                   "nodes": g.n, "edges": g.m, "walk_nodes": st.walk_nodes, "walks_per_step": st.walks,
                   "levels": st.levels, "parallelism": "1 GPU"},
        "phases": {"walk_ms_per_step": walk_ms / steps, "combine_ms_per_step": comb_ms / steps,
                   "walks_per_sec": st.walks * steps / (walk_ms / 1e3) if walk_ms > 0 else 0.0,
                   "merge_launches_per_step": st.merge_launches},
        "cpu_baseline": cpu,
    }
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--damping", type=float, default=0.85)
    ap.add_argument("--tol", type=float, default=-1.0)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="cpu_baseline threads (0 = every host CPU this process may use, cgroup quota included)")
    ap.add_argument("--cpu-budget", type=float, default=1.5e9, help="sampled candidates for cpu_baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end_to_end leg (reference-API call)")
    ap.add_argument("--workload", choices=["grank", "mc"], default="grank",
                    help="mc: MCCompletePathV2 (configs[4]) with --K 50 --L 200 --walks 1000 defaults")
    ap.add_argument("--walks", type=int, default=1000, help="mc: random walks per node (R)")
    args = ap.parse_args()
    if args.workload == "mc":
        return main_mc(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import approximated_personalized_pagerank_amd as ppr
    from approximated_personalized_pagerank_amd import build as _build
    if rank == 0:
        _build.build()

    t = time.time()
    g = ppr.rmat(args.scale, seed=args.seed)
    part = g.partitions()
    deg = g.degrees()
    log(f"[rank {rank}] RMAT-{args.scale}: n={g.n} m={g.m} dangling={(deg == 0).sum()} "
        f"|A|={(part == 0).sum()} |B|={(part == 1).sum()} prep {time.time() - t:.1f}s")

    if world > 1:
        from approximated_personalized_pagerank_amd.shard import run_distributed_bench
        res = run_distributed_bench(g, part, args, rank, world, local)
        if rank != 0:
            return
        elapsed, stats = res
        cpu = e2e = None
    else:
        plan = ppr.GrankPlan(g, args.K, args.L, args.damping, part=part, device=local, stats=True)
        for _ in range(args.warmup):
            plan.run(args.iters, args.tol)
        merge_ms = algo = dev_ms = 0.0
        launches = 0
        kst = {}
        t0 = time.perf_counter()
        for _ in range(args.steps):
            st = plan.run(args.iters, args.tol)  # synchronous: ends with an event sync
            merge_ms += st.merge_ms
            algo += st.algo_bytes
            dev_ms += st.device_ms
            launches += st.merge_launches
            for k, v in plan.kernel_stats().items():  # (host reads of counters the run already holds)
                d = kst.setdefault(k, {"algo_bytes": 0.0, "ms": 0.0, "launches": 0})
                for f in d:
                    d[f] += v[f]
        elapsed = time.perf_counter() - t0
        stats = dict(merge_ms=merge_ms, algo_bytes=algo, device_ms=dev_ms, iterations=st.iterations_run,
                     launches=launches, kernels=kst)
        cpu = e2e = None
        if not args.no_cpu_baseline:
            try:
                slab = plan.fetch_slab()
                plan.close()
                threads = args.cpu_threads if args.cpu_threads > 0 else host_cpus()[0]
                cpu = cpu_baseline(g, part, slab, args.L, args.damping, args.iters, threads, args.cpu_budget)
            except Exception as exc:  # reported, never fatal
                log(f"cpu_baseline failed: {exc!r}")
                cpu = None
        plan.close()
        if not args.no_e2e:
            try:
                e2e = end_to_end(args.scale, args.iters, args.K, args.L)
            except Exception as exc:  # reported, never fatal
                log(f"end_to_end failed: {exc!r}")

    steps = args.steps
    value = g.n * steps / elapsed
    achieved = stats["algo_bytes"] / 1e9 / (stats["merge_ms"] / 1e3) if stats["merge_ms"] > 0 else 0.0
    kernels = kernel_groups(stats.get("kernels", {}), stats["merge_ms"], steps)
    dominant = max(kernels, key=lambda k: kernels[k]["ms_per_step"]) if kernels else None
    traffic, traffic_src, traffic_build = (None, None, None)
    if (args.scale, args.K, args.L, args.iters) == (22, 64, 128, 30):
        traffic, traffic_src, traffic_build = pmc_traffic("grank_rmat22_k64_l128", sum_mode())
    build = lib_build()
    line = {
        "metric": f"source-nodes/sec grank K={args.K} L={args.L} on RMAT-{args.scale}; 1/2/4/8 MI355X + HBM GB/s",
        "value": value,
        "unit": "source-nodes/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic RMAT (Graph500 a=.57 b=.19 c=.19, edge factor 16, seed %d, dedup)" % args.seed,
        "config": {"workload": f"grank RMAT-{args.scale} K={args.K} L={args.L} iters={args.iters} "
                               f"damping={args.damping} tol={args.tol}",
                   "nodes": g.n, "edges": g.m, "iterations_run": stats["iterations"],
                   "parallelism": f"source-shard x{world}" if world > 1 else "1 GPU",
                   "sum": sum_mode(),
                   "step": "cold call: every run resets its per-job planning state (distinct-key estimates, "
                           "hot set) in ppr_grank_plan_init; graph and slab resident"},
        "roofline": {"bound": "hbm",
                     "kernel": ("basket-merge phase, exact sum: k_classify + k_merge_lds_x (wave tier) + sieve "
                                "(k_sv1 + k_svfin in three size classes, k_svA + k_svB + k_svF for multi-slice "
                                "sources; range / partition engines for the sources it hands back)"
                                if sum_mode() == "exact" else
                                "basket-merge phase, chain sum: k_classify + k_merge_lds (wave tiers) + hub pipeline "
                                "(k_hub_count, device scan, k_hub_scatter, k_hub_bucket_w, k_hub_final)"),
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "algo_bytes_per_step": stats["algo_bytes"] / steps,
                     "merge_ms_per_step": stats["merge_ms"] / steps,
                     "merge_launches_per_step": stats["launches"] / steps,
                     "traffic": traffic, "traffic_source": traffic_src,
                     # the PMC summary's library against this run's: equal = the same kernels profiled
                     "traffic_build": traffic_build, "traffic_same_build": traffic_build == build if traffic_build else None,
                     "dominant_kernel": dominant,
                     "kernels": kernels},
        "cpu_baseline": cpu,
        "end_to_end": e2e,
        "build": build,
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
