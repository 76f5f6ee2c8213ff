# exact-sum: focused parity (incl. chain hub variants: the staged record layout changed), A/B, DIAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xs
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "exact_sum or oracle_rmat or tier_paths" > gpurun_out/xs/pytest5.txt 2>&1 || { tail -40 gpurun_out/xs/pytest5.txt; exit 1; }
tail -2 gpurun_out/xs/pytest5.txt
timeout -k 10 900 python -u tools/whatif.py --reps 1 "" "PPR_SUM=chain" "PPR_DIAG=1" > gpurun_out/xs/whatif5.txt 2>&1
cat gpurun_out/xs/whatif5.txt | grep -v "^ppr_diag [ 0-9]"
