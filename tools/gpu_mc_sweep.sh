# GPU tests, then an MC bucket-size sweep around the defaults
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest.txt 2>&1
tail -2 gpurun_out/chk/pytest.txt
BENCH_ARGS="--workload mc" bash tools/ab_env2.sh "" "PPR_HUB_BUCKET=576 PPR_HUB_WAVE_T=640" "PPR_HUB_BUCKET=704 PPR_HUB_WAVE_T=832" "PPR_HUB_BUCKET=640 PPR_HUB_WAVE_T=704" "PPR_HUB_BUCKET=768 PPR_HUB_WAVE_T=896" "PPR_HUB_BUCKET=448 PPR_HUB_WAVE_T=512" ""
