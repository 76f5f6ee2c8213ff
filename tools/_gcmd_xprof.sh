# kernel statistics of the exact-sum path (one warmup + one timed job)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/xp
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/trace.json 2> $OUT/trace.err
head -c 400 $OUT/trace.json; echo
f=$(find $OUT/trace -name "*kernel_stats.csv" | head -1)
head -30 "$f"
