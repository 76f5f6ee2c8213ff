set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wi/split_tests.txt 2>&1
tail -2 gpurun_out/wi/split_tests.txt
timeout -k 10 600 python3 tools/whatif.py "" PPR_TILE_SPLIT_LOGP=12 PPR_TILE_SPLIT_LOGP=8 PPR_TILE_SPLIT_LOGP=11 "" PPR_TILE_SPLIT_LOGP=12 > gpurun_out/wi/split.txt 2>&1
cat gpurun_out/wi/split.txt
