# GPU test suite + smoke, then the default bench line, under gpurun_out/chk
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest.txt 2>&1
tail -2 gpurun_out/chk/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
timeout -k 10 600 python3 bench.py > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.err
head -c 600 gpurun_out/chk/bench.json
