# kernel trace of the exact-sum path: stats + stream timeline (busy vs idle, exclusive vs shared)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/xp2
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/trace -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/trace.json 2> $OUT/trace.err
python3 tools/timeline.py $(find $OUT/trace -name "*results.db" | head -1) > $OUT/timeline.txt || true
python3 tools/kstats.py $(find $OUT/trace -name "*kernel_stats.csv" | head -1) 2 > $OUT/kstats.txt 2>&1 || true
cat $OUT/timeline.txt | head -40
find $OUT -name "*.db" -size +60M -delete
