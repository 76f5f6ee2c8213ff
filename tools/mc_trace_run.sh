# MC combine kernel + copy trace (one timed job, no warmup) for tools/mc_trace.py
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/mctrace
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $OUT/trace -o run --output-format csv -- python3 bench.py --workload mc --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/trace.json 2> $OUT/trace.err
echo trace done
ls -R $OUT | head -20
