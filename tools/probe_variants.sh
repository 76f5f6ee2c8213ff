set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/probe
for v in ${VARIANTS:-base lin}; do
  PPR_HUB_STREAMS=1 PPR_LIB_VARIANT=$([ $v = cur ] || echo $v) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe/$v -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --iters 10 > gpurun_out/probe/$v.json 2> gpurun_out/probe/$v.err
done
