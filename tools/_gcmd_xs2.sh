# exact-sum path: debug variants, focused parity tests, then the bench in both summation modes (same box)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xs
timeout -k 10 300 python -u tools/debug_xs.py 13 32 128 4 104
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "exact_sum or oracle_rmat or full_slab or tier_paths" > gpurun_out/xs/pytest.txt 2>&1 || { tail -40 gpurun_out/xs/pytest.txt; exit 1; }
tail -2 gpurun_out/xs/pytest.txt
PPR_TIMING=1 timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/xs/bench_exact.json 2> gpurun_out/xs/bench_exact.err
head -c 700 gpurun_out/xs/bench_exact.json; echo
PPR_SUM=chain timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/xs/bench_chain.json 2> gpurun_out/xs/bench_chain.err
head -c 700 gpurun_out/xs/bench_chain.json; echo
