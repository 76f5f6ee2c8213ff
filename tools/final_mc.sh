# MC bench line with cpu_baseline, and the per-level trace summary, under gpurun_out/final_mc
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/final_mc
mkdir -p $OUT
timeout -k 10 400 python3 bench.py --workload mc > $OUT/bench.json 2> $OUT/bench.err
echo bench done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --workload mc --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/trace.json 2> $OUT/trace.err
python3 tools/mc_trace.py $OUT/trace/run_kernel_trace.csv > $OUT/mc_levels.txt
cp $OUT/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
rm -rf $OUT/trace
echo trace done
