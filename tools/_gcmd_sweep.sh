# exact-sum: focused parity, then a knob sweep on RMAT-22 (one process and time limit per variant)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xs
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "exact_sum or oracle_rmat or tier_paths" > gpurun_out/xs/pytest7.txt 2>&1 || { tail -40 gpurun_out/xs/pytest7.txt; exit 1; }
tail -2 gpurun_out/xs/pytest7.txt
for v in "" "PPR_DIAG=1" ${SWEEP}; do
  echo "variant: $v"
  timeout -k 10 150 python -u tools/whatif.py --reps 1 "$v" > gpurun_out/xs/sweep_one.txt 2>&1 || { echo "variant $v failed: $?"; tail -5 gpurun_out/xs/sweep_one.txt; exit 1; }
  grep -v "^ppr_diag [ 0-9]" gpurun_out/xs/sweep_one.txt | grep -v "^RMAT" || true
done
