# round-end set: GPU tests, GRank profile set (tools/profile_round.sh), MC bench line + level trace
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest.txt 2>&1
tail -2 gpurun_out/chk/pytest.txt
bash tools/profile_round.sh r02final
bash tools/final_mc.sh
