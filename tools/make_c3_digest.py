"""Golden digests of the WHOLE C3 job (BASELINE.json configs[2]: RMAT-22 K64/L128/30 iterations),
computed here by the CPU oracle (oracle/grank_oracle.c, pinned to the compiled reference) on all
host threads: every iteration's source list is split into chunks stepped in parallel
(oracle.step_rows_parallel: the same Jacobi step as oracle.grank, verified equal to it), the
iteration's maxDiff comes from oracle.norm1_max (the engine's summation pattern), and the final
keepTop(K) from oracle.topk_rows. The result (2 x 268 M entries) is too large to commit: its
SHA-256 digests -- final rows, the full L-slab after every iteration, the maxDiff history -- are
the bit-exact targets of tests/test_gpu_scale.py (C3, one GPU) and tests/test_gpu_c4.py (C4, the
source-sharded loop with 8 ranks).

    python tools/make_c3_digest.py [--threads 8] [--sum exact|chain]
        -> tests/golden/c3_rmat22_k64_l128_i30.json (chain), c3_rmat22_k64_l128_i30_exact.json (exact)
"""
import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import approximated_personalized_pagerank_amd as ppr  # noqa: E402
import oracle  # noqa: E402


def digest(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def slab_digest(ids, sc, ln, L):
    """rows as ppr_grank_plan_fetch_slab hands them out: first len entries by (score desc, id asc)
    -- the oracle's storage order -- then -1 / 0.0 padding"""
    pad = np.arange(L)[None, :] >= ln[:, None]
    return digest(np.where(pad, -1, ids).astype(np.int32), np.where(pad, 0.0, sc), ln)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=int, default=22)
    ap.add_argument("--K", type=int, default=64)
    ap.add_argument("--L", type=int, default=128)
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    ap.add_argument("--sum", choices=["exact", "chain"], default="chain", help="GRank summation mode (oracle.set_sum)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    oracle.set_sum(a.sum)
    if a.out is None:
        a.out = os.path.join(ROOT, "tests", "golden",
                             "c3_rmat22_k64_l128_i30" + ("_exact" if a.sum == "exact" else "") + ".json")
    d, seed, tol = 0.85, 42, -1.0
    t0 = time.time()
    g = ppr.rmat(a.scale, seed=seed)
    part = g.partitions()
    assert np.array_equal(part, oracle.find_partitions(g.row_ptr, g.col))
    n, L, K = g.n, a.L, a.K
    ids = np.full((n, L), -1, dtype=np.int32)
    sc = np.zeros((n, L), dtype=np.float64)
    ln = np.zeros(n, dtype=np.int32)
    assert oracle.lib().oracle_init_state(n, g.row_ptr.ctypes.data, g.col.ctypes.data, L, d, ids.ctypes.data,
                                          sc.ctypes.data, ln.ctypes.data) == 0
    nids, nsc, nln = ids.copy(), sc.copy(), ln.copy()
    deg = np.diff(g.row_ptr)
    md, slabs = [], []
    print(f"graph + partitions + init {time.time() - t0:.0f} s", flush=True)
    for it in range(a.iters):
        act = np.nonzero((part == (it & 1)) & (deg > 0))[0].astype(np.int32)
        oracle.step_rows_parallel(g.row_ptr, g.col, L, d, (ids, sc, ln), (nids, nsc, nln), act, a.threads)
        md.append(oracle.norm1_max(L, act, (ids, sc, ln), (nids, nsc, nln)))
        ids[act], sc[act], ln[act] = nids[act], nsc[act], nln[act]
        slabs.append(slab_digest(ids, sc, ln, L))
        print(f"iteration {it}: {len(act)} sources, maxDiff {md[-1]:.6g}, {time.time() - t0:.0f} s", flush=True)
    out = (np.full((n, K), -1, dtype=np.int32), np.zeros((n, K), dtype=np.float64), np.zeros(n, dtype=np.int32))
    oracle.topk_rows(L, K, (ids, sc, ln), np.arange(n, dtype=np.int32), out)
    res = {"config": f"RMAT-{a.scale} seed {seed} K={K} L={L} iterations={a.iters} damping={d} tol={tol}",
           "scale": a.scale, "seed": seed, "K": K, "L": L, "iters": a.iters, "damping": d, "tol": tol,
           "n": int(n), "m": int(g.m), "graph_sha256": digest(g.col), "part_sha256": digest(part),
           "iterations_run": a.iters, "max_diff": [float(x).hex() for x in md],
           "ids_sha256": digest(out[0]), "scores_sha256": digest(out[1]), "lens_sha256": digest(out[2]),
           "slab_after_iteration_sha256": slabs,
           "oracle_seconds": round(time.time() - t0, 1), "oracle_threads": a.threads, "sum": a.sum}
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    print(a.out, res["oracle_seconds"], "s")


if __name__ == "__main__":
    main()
