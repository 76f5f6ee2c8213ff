set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/c3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_c4.py tests/test_cpp_dropin.py -x -v --timeout 600 --timeout-method thread > $OUT/pytest.txt 2>&1
echo tests done
grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/pytest.txt | tail -20
timeout -k 10 300 python3 bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/mc.json 2> $OUT/mc.err
PPR_WHATIF=128 timeout -k 10 300 python3 bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/mc_cut.json 2> $OUT/mc_cut.err
python3 -c "
import json
for f in ['mc', 'mc_cut']:
    d = json.load(open('$OUT/%s.json' % f)); print(f, round(d['ms_per_step'], 1), d.get('phases', {}))"
timeout -k 10 300 python3 tools/quality_rmat.py --algo mc --K 50 --L 200 --iters 1000 > $OUT/mc_quality.json 2> $OUT/mc_quality.err
cat $OUT/mc_quality.json
