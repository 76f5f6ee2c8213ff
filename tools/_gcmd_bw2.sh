set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bw2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/bw2/tests.txt 2>&1
tail -2 gpurun_out/bw2/tests.txt
timeout -k 10 600 python3 tools/whatif.py "" PPR_BW2=0 "" PPR_BW2=0 > gpurun_out/bw2/ab.txt 2>&1
cat gpurun_out/bw2/ab.txt
