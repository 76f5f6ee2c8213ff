set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wi/tests.txt 2>&1
tail -2 gpurun_out/wi/tests.txt
timeout -k 10 1000 python3 tools/whatif.py --reps 2 "" "" PPR_SCAT_BATCH=0 "" PPR_SCAT_BATCH=0 PPR_WHATIF=8 PPR_WHATIF=4 > gpurun_out/wi/scat6.txt 2>&1
cat gpurun_out/wi/scat6.txt
