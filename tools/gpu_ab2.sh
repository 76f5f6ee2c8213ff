# GPU tests, then same-box A/B of the product build against the "base" variant: GRank and MC
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/chk gpurun_out/ab
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/chk/pytest.txt 2>&1
tail -2 gpurun_out/chk/pytest.txt
for w in mc grank; do
  for v in "" base "" base; do
    PPR_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --workload $w --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab/v.json 2>gpurun_out/ab/v.err
    python3 -c "import json; d=json.load(open('gpurun_out/ab/v.json')); print('$w variant [$v]', round(d['ms_per_step']))"
  done
done
