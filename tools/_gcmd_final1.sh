set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/chk/pytest.txt 2>&1
echo tests done
tail -3 gpurun_out/chk/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
bash tools/profile_r03.sh
