# kernel-time probe of environment settings (single hub stream, 10 iterations):
#   bash tools/probe_env.sh NAME "ENV=.. ENV=.." NAME2 "ENV=.."
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/probe
while [ $# -ge 2 ]; do
  name=$1; cfg=$2; shift 2
  env PPR_HUB_STREAMS=1 $cfg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/probe/$name -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --iters 10 > gpurun_out/probe/$name.json 2> gpurun_out/probe/$name.err
done
