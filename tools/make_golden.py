#!/usr/bin/env python3
"""Generate the golden vectors under tests/golden/ by running the compiled reference.

Runs oracle/_ref/ref_driver (built by `make -C oracle ref` from the unmodified reference headers
in /root/reference) on graphs produced here, and stores inputs + reference outputs as .npz
fixtures (data only; no reference source travels). Run from the repo root:

    python tools/make_golden.py

Each fixture holds, in the REFERENCE's graph iteration order (its unordered_map order, which
defines the dense ids the engine uses): the dense CSR (rp, col), the reference's partition bits
(findPartitions), the parameters, and the reference result rows sorted by (score desc, id asc).
"""
from __future__ import annotations

import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_driver")
EAT = "/root/reference/example.txt"


def write_graph_bin(path, keys, succ_lists):
    n = len(keys)
    rp = np.zeros(n + 1, dtype=np.int64)
    flat = []
    for i, s in enumerate(succ_lists):
        flat.extend(s)
        rp[i + 1] = len(flat)
    with open(path, "wb") as f:
        np.array([n, len(flat)], dtype=np.int64).tofile(f)
        np.asarray(keys, dtype=np.int32).tofile(f)
        rp.tofile(f)
        np.asarray(flat, dtype=np.int32).tofile(f)


def read_out(path, K):
    with open(path, "rb") as f:
        buf = f.read()
    off = 0

    def take(dtype, count):
        nonlocal off
        a = np.frombuffer(buf, dtype=dtype, count=count, offset=off)
        off += a.nbytes
        return a.copy()

    n = int(take(np.int64, 1)[0])
    order = take(np.int32, n)
    m = int(take(np.int64, 1)[0])
    rp = take(np.int64, n + 1)
    col = take(np.int32, m)
    part = take(np.uint8, n)
    exec_order = take(np.int32, n)
    ms = float(take(np.float64, 1)[0])
    ids = np.full((n, K), -1, dtype=np.int32)
    sc = np.zeros((n, K), dtype=np.float64)
    cnt = np.zeros(n, dtype=np.int32)
    rec = np.dtype([("k", "<i4"), ("s", "<f8")])
    for v in range(n):
        c = int(take(np.int32, 1)[0])
        if c:
            r = np.frombuffer(buf, dtype=rec, count=c, offset=off)
            off += r.nbytes
            o = np.lexsort((r["k"], -r["s"]))  # score desc, id asc
            kk = min(c, K)
            ids[v, :kk] = r["k"][o][:kk]
            sc[v, :kk] = r["s"][o][:kk]
            cnt[v] = c
    return dict(order=order, rp=rp, col=col, part=part, exec_order=exec_order, ms=ms, ids=ids,
                scores=sc, cnt=cnt)


def run_ref(mode, graph_path, K, L, iters, d, tol, threads=1):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "out.bin")
        subprocess.run([DRIVER, mode, graph_path, out, str(K), str(L), str(iters), repr(d), repr(tol),
                        str(threads)], check=True)
        return read_out(out, K)


def save(name, res, params, sample=None, extra=None):
    d = dict(order=res["order"], rp=res["rp"], col=res["col"], part=res["part"],
             params=np.array(params, dtype=np.float64))
    if res["exec_order"].size and res["exec_order"][0] >= 0:
        d["exec_order"] = res["exec_order"]
    if sample is None:
        d.update(ids=res["ids"], scores=res["scores"], cnt=res["cnt"])
    else:
        d.update(sample=sample, ids=res["ids"][sample], scores=res["scores"][sample], cnt=res["cnt"][sample])
    if extra:
        d.update(extra)
    path = os.path.join(GOLDEN, name + ".npz")
    np.savez_compressed(path, **d)
    print(f"{name}: n={len(res['order'])} m={len(res['col'])} -> {os.path.getsize(path) / 1024:.0f} KiB")


def gen_graph(name, keys, succ, K, L, iters, d, tol, mode="grank", threads=1, sample=None, extra_modes=()):
    with tempfile.TemporaryDirectory() as td:
        gp = os.path.join(td, "g.bin")
        write_graph_bin(gp, keys, succ)
        res = run_ref(mode, gp, K, L, iters, d, tol, threads)
        extra = {}
        for em, eK, eL, eit, etol in extra_modes:
            r2 = run_ref(em, gp, eK, eL, eit, d, etol, 1)
            extra[f"{em}_ids"] = r2["ids"]
            extra[f"{em}_scores"] = r2["scores"]
            extra[f"{em}_cnt"] = r2["cnt"]
        save(name, res, [K, L, iters, d, tol], sample, extra)
        return res


def rmat_lists(scale, seed=42):
    from approximated_personalized_pagerank_amd.graph import rmat
    g = rmat(scale, seed=seed)
    keys = list(range(g.n))
    succ = [g.col[g.row_ptr[i]:g.row_ptr[i + 1]].tolist() for i in range(g.n)]
    return keys, succ


def main_mc():
    """MCCompletePathV2 fixtures (mode mc): the reference's executionOrder (exact target) and one
    sample of its random-walk result (statistical target), plus exact PPR where cheap."""
    rng = np.random.default_rng(2017)

    def mg(name, n, edges, K, L, R, pprss=False, sample=None, pprss_topk=False):
        succ = [[] for _ in range(n)]
        for a, b in edges:
            succ[a].append(b)
        extra = [("pprss", n, 0, 100, -1.0)] if pprss else ()
        res = gen_graph(name, list(range(n)), succ, K, L, R, 0.85, -1.0, mode="mc", extra_modes=extra,
                        sample=sample)
        if pprss_topk:
            # exact PPR of every source, kept to the top-K (quality reference for the MC rows)
            with tempfile.TemporaryDirectory() as td:
                gp = os.path.join(td, "g.bin")
                write_graph_bin(gp, list(range(n)), succ)
                ex = run_ref("pprss", gp, n, 0, 100, 0.85, -1.0)
            assert np.array_equal(ex["order"], res["order"])
            path = os.path.join(GOLDEN, name + ".npz")
            z = dict(np.load(path))
            z.update(pprss_ids=ex["ids"][:, :K], pprss_scores=ex["scores"][:, :K],
                     pprss_cnt=np.minimum(ex["cnt"], K))
            np.savez_compressed(path, **z)

    # test/mccompletepathv2Test.cc graphs
    mg("m1_noedges10", 10, [], 10, 30, 100)
    mg("m1_single_loop", 1, [(0, 0)], 10, 30, 1000)
    mg("m1_two_linked", 2, [(0, 1), (1, 0)], 10, 30, 1000, pprss=True)
    mg("m1_ring6", 6, [(i, (i + 1) % 6) for i in range(6)], 10, 30, 20000, pprss=True)
    mg("m1_star", 6, [(i, 0) for i in range(1, 6)], 10, 30, 100)
    mg("m1_star_loop", 6, [(i, 0) for i in range(1, 6)] + [(0, 0)], 10, 30, 1000)
    mg("m1_star_rev", 6, [(0, i) for i in range(1, 6)], 10, 30, 100)
    mg("m1_star_rev_loops", 6, [(0, i) for i in range(1, 6)] + [(i, i) for i in range(1, 6)], 10, 30, 200)
    ring100 = [(i, i + 1) for i in range(99)] + [(99, 0)]
    mg("m1_ring100_k10_l20", 100, ring100, 10, 20, 1000)
    # no truncation: statistical comparison against exact PPR
    rnd = [(int(a), int(b)) for a, b in rng.integers(0, 100, size=(400, 2))]
    mg("m2_random100_full", 100, rnd, 100, 100, 20000, pprss=True)
    # RMAT: execution order (exact) and a truncating MC run
    keys, succ = rmat_lists(10)
    edges = [(a, b) for a in range(len(succ)) for b in succ[a]]
    mg("m3_rmat10_k16_l64", len(keys), edges, 16, 64, 1000, pprss_topk=True)
    keys, succ = rmat_lists(14)
    edges = [(a, b) for a in range(len(succ)) for b in succ[a]]
    mg("m3_rmat14_order", len(keys), edges, 1, 1, 1, sample=np.arange(0, dtype=np.int64))
    # EAT, the reference CLI's call mccompletepathv2(50, 200, 1000, .85) (src/main.cc:48)
    if os.path.exists(EAT):
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "out.bin")
            subprocess.run([DRIVER, "mc", EAT, out, "50", "200", "1000", "0.85", "-1", "1"], check=True)
            res = read_out(out, 50)
        n = len(res["order"])
        sample = np.sort(rng.choice(n, 3000, replace=False)).astype(np.int64)
        save("m4_eat_k50_l200", res, [50, 200, 1000, 0.85, -1.0], sample)


def pprss_rows(name, K, keys, succ, n_src=200, tol=1e-4, seed=7):
    """exact PPR (pprSingleSource, 100 iterations, d .85, tol 1e-4: the reference's quality harness,
    include/benchmarkAlgorithm.h:91) of `n_src` sampled non-dangling sources of fixture `name`,
    kept to the top K + 32 (room for ties at the K-th score), appended to the fixture"""
    path = os.path.join(GOLDEN, name + ".npz")
    z = dict(np.load(path))
    rp, order = z["rp"], z["order"]
    deg = np.diff(rp)
    rng = np.random.default_rng(seed)
    pool = np.nonzero(deg > 0)[0]
    if "sample" in z:  # sources whose reference rows the fixture holds
        pool = np.intersect1d(pool, z["sample"])
    src = np.sort(rng.choice(pool, n_src, replace=False)).astype(np.int32)
    with tempfile.TemporaryDirectory() as td:
        gp = os.path.join(td, "g.bin")
        lp = os.path.join(td, "list.bin")
        # the graph file exactly as the fixture was made from it: the reference then iterates it
        # in the same order, so the dense ids (the fixture's) coincide
        write_graph_bin(gp, keys, succ)
        src.tofile(lp)
        out = os.path.join(td, "out.bin")
        subprocess.run([DRIVER, "pprss_list", gp, out, str(K + 32), "0", "100", "0.85", repr(tol), "1", lp],
                       check=True)
        ex = read_out(out, K + 32)
    assert np.array_equal(ex["order"], order), "dense order changed"
    z.update(pprss_src=src, pprss_ids=ex["ids"][src], pprss_scores=ex["scores"][src], pprss_cnt=ex["cnt"][src])
    np.savez_compressed(path, **z)
    print(f"{name}: exact PPR of {len(src)} sources -> {os.path.getsize(path) / 1024:.0f} KiB")


def self_ceiling(name, keys, succ, n_perm=3, seed=11):
    """the reference against itself on randomly relabelled input: mean top-K Jaccard
    and max sorted-score-profile difference over the fixture's rows, and its top-K Jaccard vs
    the fixture's exact-PPR rows -- the bar the P3/P4 checks are stated against"""
    path = os.path.join(GOLDEN, name + ".npz")
    z = dict(np.load(path))
    K, L, it, d, tol = z["params"]
    K, L, it, d, tol = int(K), int(L), int(it), float(d), float(tol)  # repr() of numpy scalars is not a number
    mode = "grankmulti" if "sample" in z else "grank"
    n = len(z["order"])
    rows = z["sample"] if "sample" in z else np.arange(n)
    dense_of_key = np.empty(n, dtype=np.int64)
    dense_of_key[z["order"]] = np.arange(n)
    rng = np.random.default_rng(seed)
    js, profs, qual = [], [], []
    for _ in range(n_perm):
        perm = rng.permutation(n)  # original key k -> new key perm[k]
        with tempfile.TemporaryDirectory() as td:
            gp = os.path.join(td, "g.bin")
            write_graph_bin(gp, [int(perm[k]) for k in keys], [[int(perm[x]) for x in s] for s in succ])
            r = run_ref(mode, gp, K, L, it, d, tol, 8)
        # r's dense id -> new key -> original key -> fixture dense id
        inv = np.argsort(perm)
        fx = dense_of_key[inv[r["order"]]]
        ids = np.full((n, K), -1, dtype=np.int64)
        cnt = np.zeros(n, dtype=np.int64)
        sc = np.zeros((n, K))
        ids[fx] = np.where(r["ids"] >= 0, fx[np.maximum(r["ids"], 0)], -1)
        cnt[fx] = np.minimum(r["cnt"], K)
        sc[fx] = r["scores"]
        zc = np.minimum(z["cnt"], K)
        zi = z["ids"] if "sample" in z else z["ids"]
        zs = z["scores"]
        j, p = [], 0.0
        for q, v in enumerate(rows):
            a, b = set(ids[v, :cnt[v]].tolist()), set(zi[q, :zc[q]].tolist())
            j.append(1.0 if not (a or b) else len(a & b) / len(a | b))
            if cnt[v] == zc[q] and cnt[v]:
                p = max(p, float(np.abs(np.sort(sc[v, :cnt[v]]) - np.sort(zs[q, :zc[q]])).max()))
        js.append(np.mean(j))
        profs.append(p)
        if "pprss_src" in z:
            kq = []
            for t, v in enumerate(z["pprss_src"]):
                a = set(ids[v, :cnt[v]].tolist())
                b = set(z["pprss_ids"][t, :min(K, z["pprss_cnt"][t])].tolist())
                kq.append(1.0 if not (a or b) else len(a & b) / len(a | b))
            qual.append(np.mean(kq))
    z.update(self_jaccard=np.array(js), self_profile=np.array(profs))
    if qual:
        z.update(self_quality=np.array(qual))
    np.savez_compressed(path, **z)
    print(f"{name}: reference vs relabelled reference: Jaccard {np.round(js, 4)} profile {np.round(profs, 6)} "
          f"quality {np.round(qual, 4)}")


def tie_replay(name, scale, L, its, d=0.85):
    """the reference's full baskets (K = L: keepTop(K) keeps the whole basket) after `it` and
    `it + 1` iterations, for the per-iteration ties-only check (tests/test_oracle_golden.py)"""
    keys, succ = rmat_lists(scale)
    out = {}
    with tempfile.TemporaryDirectory() as td:
        gp = os.path.join(td, "g.bin")
        write_graph_bin(gp, keys, succ)
        for it in its:
            for k in (it, it + 1):
                if f"ids_{k}" in out:
                    continue
                r = run_ref("grank", gp, L, L, k, d, -1.0)
                out.update({f"ids_{k}": r["ids"], f"scores_{k}": r["scores"], f"cnt_{k}": r["cnt"]})
            out.update(rp=r["rp"], col=r["col"], part=r["part"], order=r["order"])
    out["params"] = np.array([L, L, 0, d, -1.0])
    out["its"] = np.array(its, dtype=np.int32)
    path = os.path.join(GOLDEN, name + ".npz")
    np.savez_compressed(path, **out)
    print(f"{name}: -> {os.path.getsize(path) / 1024:.0f} KiB")


def main_p34():
    """P3/P4 fixtures: exact-PPR rows for sampled sources of the truncating RMAT runs,
    a K64/L128 RMAT-14 run, and reference states for the ties-only replay"""
    rng = np.random.default_rng(34)
    k14, s14 = rmat_lists(14)
    if not os.path.exists(os.path.join(GOLDEN, "g3_rmat14_k64_l128.npz")):
        sample = np.sort(rng.choice(1 << 14, 2048, replace=False)).astype(np.int64)
        gen_graph("g3_rmat14_k64_l128", k14, s14, 64, 128, 30, 0.85, -1.0, mode="grankmulti", threads=8,
                  sample=sample)
    k12, s12 = rmat_lists(12)
    if "--pprss-only" not in sys.argv:
        pprss_rows("g3_rmat12_k16_l32", 16, k12, s12)
    pprss_rows("g3_rmat14_k32_l64", 32, k14, s14)
    pprss_rows("g3_rmat14_k64_l128", 64, k14, s14)
    if "--pprss-only" not in sys.argv:
        tie_replay("r1_rmat12_l32", 12, 32, (3, 8))
    self_ceiling("g3_rmat12_k16_l32", k12, s12)
    self_ceiling("g3_rmat14_k32_l64", k14, s14)
    self_ceiling("g3_rmat14_k64_l128", k14, s14)


def main():
    if "--mc" in sys.argv:
        return main_mc()
    if "--p34" in sys.argv:
        return main_p34()
    os.makedirs(GOLDEN, exist_ok=True)
    if not os.path.exists(DRIVER):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    rng = np.random.default_rng(12345)

    # G1: README ring of 100 (README.md "GRank" example), K50 L100 30 it tol 1e-3
    ring = [[(i + 1) % 100] for i in range(100)]
    gen_graph("g1_ring100", list(range(100)), ring, 50, 100, 30, 0.85, 1e-3)
    gen_graph("g1_ring100_multi", list(range(100)), ring, 50, 100, 30, 0.85, 1e-3, mode="grankmulti", threads=4)

    # G2: no truncation (L >= |V|): bit-exact target
    keys, succ = rmat_lists(8)
    gen_graph("g2_rmat8_full", keys, succ, 256, 256, 10, 0.85, -1.0)

    # G3: truncating RMAT runs
    keys, succ = rmat_lists(12)
    gen_graph("g3_rmat12_k16_l32", keys, succ, 16, 32, 10, 0.85, -1.0)
    keys, succ = rmat_lists(14)
    sample = np.sort(rng.choice(1 << 14, 2048, replace=False)).astype(np.int64)
    gen_graph("g3_rmat14_k32_l64", keys, succ, 32, 64, 20, 0.85, -1.0, mode="grankmulti", threads=8,
              sample=sample)

    # G4: EAT (example.txt), grankMulti K50 L100 30 it 1e-4 (src/main.cc:37), 3000-source sample
    if os.path.exists(EAT):
        with tempfile.TemporaryDirectory() as td:
            out = os.path.join(td, "out.bin")
            subprocess.run([DRIVER, "grankmulti", EAT, out, "50", "100", "30", "0.85", "0.0001", "4"], check=True)
            res = read_out(out, 50)
        n = len(res["order"])
        sample = np.sort(rng.choice(n, 3000, replace=False)).astype(np.int64)
        save("g4_eat_k50_l100", res, [50, 100, 30, 0.85, 1e-4], sample)

    # G5: the reference tests' known-answer graphs (test/grankTest.cc), reference outputs + exact
    # PPR (pprSingleSource) where the test compares against it.
    def kg(name, n, edges, K, L, iters, tol, pprss=False):
        succ = [[] for _ in range(n)]
        for a, b in edges:
            succ[a].append(b)
        extra = [("pprss", n, 0, 100, -1.0)] if pprss else ()
        gen_graph(name, list(range(n)), succ, K, L, iters, 0.85, tol, extra_modes=extra)

    kg("g5_noedges10", 10, [], 10, 30, 100, 1e-4)
    kg("g5_single", 1, [], 10, 30, 100, 1e-4)
    kg("g5_single_loop", 1, [(0, 0)], 10, 30, 100, 1e-4)
    kg("g5_two_linked", 2, [(0, 1), (1, 0)], 10, 30, 100, 1e-4)
    kg("g5_ring6", 6, [(i, (i + 1) % 6) for i in range(6)], 10, 30, 100, 1e-4)
    kg("g5_ring6_k3l4", 6, [(i, (i + 1) % 6) for i in range(6)], 3, 4, 100, 1e-4)
    kg("g5_star", 6, [(i, 0) for i in range(1, 6)], 10, 30, 100, 1e-4)
    kg("g5_star_loop", 6, [(i, 0) for i in range(1, 6)] + [(0, 0)], 10, 30, 100, 1e-4)
    ring100 = [(i, i + 1) for i in range(99)] + [(99, 0)]
    kg("g5_ring100_k10_l10", 100, ring100, 10, 10, 100, 1e-4)
    kg("g5_ring100_k10_l20", 100, ring100, 10, 20, 100, 1e-4)
    kg("g5_ring100_full", 100, ring100, 100, 100, 100, -1.0, pprss=True)
    instar = [(i, 0) for i in range(99)]
    kg("g5_instar_full", 100, instar, 100, 100, 100, -1.0, pprss=True)
    kg("g5_instar_loop_full", 100, instar + [(0, 0)], 100, 100, 100, -1.0, pprss=True)
    kg("g5_instar_all_full", 100, instar + [(0, 0)] + [(0, i) for i in range(99)], 100, 100, 100, -1.0,
       pprss=True)
    rnd = [(int(a), int(b)) for a, b in rng.integers(0, 100, size=(5000, 2))]
    kg("g5_random5000_full", 100, rnd, 100, 100, 100, -1.0, pprss=True)
    kg("g5_complete_full", 100, [(i, u) for i in range(100) for u in range(100)], 100, 100, 100, -1.0,
       pprss=True)


if __name__ == "__main__":
    main()
