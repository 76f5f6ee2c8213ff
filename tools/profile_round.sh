# Round profile set for the headline workload: bench line, kernel trace + stats, and the two PMC
# traffic passes (FETCH_SIZE and WRITE_SIZE in runs of their own), all under gpurun_out/<$1: final>/
# (SKIP_BENCH=1: no plain bench run).
# Summaries for profiles/: tools/prof_summary.py, tools/timeline.py, tools/pmc_summary.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 500 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
  echo bench done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/trace.json 2> $OUT/trace.err
echo trace done
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/fetch.json 2> $OUT/fetch.err
echo fetch done
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/write.json 2> $OUT/write.err
echo write done
