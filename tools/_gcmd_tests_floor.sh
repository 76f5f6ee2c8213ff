set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest.txt 2>&1
echo tests done
tail -3 gpurun_out/chk/pytest.txt
timeout -k 10 300 python3 tools/shard_floor.py --out gpurun_out/chk/shard_floor.json > gpurun_out/chk/shard_floor.txt 2>&1
cat gpurun_out/chk/shard_floor.txt
