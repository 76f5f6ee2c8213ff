set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/mc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/mc/pytest.txt 2>&1
echo tests done
tail -3 gpurun_out/mc/pytest.txt
timeout -k 10 300 python3 tools/mc_whatif.py "" "" PPR_BW2=0 "PPR_HUB_BUCKET=448 PPR_HUB_WAVE_T=512" "PPR_HUB_BUCKET=512 PPR_HUB_WAVE_T=640" "" PPR_BW2=0 > gpurun_out/mc/ab.txt 2>&1
cat gpurun_out/mc/ab.txt
timeout -k 10 500 python3 bench.py > gpurun_out/mc/bench.json 2> gpurun_out/mc/bench.err
cat gpurun_out/mc/bench.json
