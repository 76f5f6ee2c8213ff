# GPU test suite, then (TRACE=1) the MC per-level trace, MC and GRank bench lines, under gpurun_out/chk
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/chk
mkdir -p $OUT
if [ -z "$NOTEST" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.txt 2>&1
  echo tests done
  tail -3 $OUT/pytest.txt
fi
if [ -n "$TRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python3 bench.py --workload mc --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/mctrace.json 2> $OUT/mctrace.err
  python tools/mc_trace.py $OUT/trace/run_kernel_trace.csv > $OUT/mc_levels.txt
  rm -rf $OUT/trace
  echo trace done
fi
timeout -k 10 300 python3 bench.py --workload mc --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/mc.json 2> $OUT/mc.err
echo mc done
timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/grank.json 2> $OUT/grank.err
echo grank done
python3 -c "
import json
for f in ['mc', 'grank']:
    d = json.load(open('$OUT/%s.json' % f)); print(f, round(d['ms_per_step'], 1), d.get('phases', {}).get('combine_ms_per_step'))"
