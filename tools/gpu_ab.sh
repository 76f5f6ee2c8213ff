# GPU tests, then same-box GRank A/B of the product build against the "base" variant
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest.txt 2>&1
tail -2 gpurun_out/chk/pytest.txt
bash tools/ab_variants.sh "" base "" base
