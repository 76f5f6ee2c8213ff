# same-box A/B of environment settings (no cpu_baseline, no end_to_end): bash tools/ab_env2.sh "" "A=1 B=2" ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for cfg in "$@"; do
  env $cfg timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e $BENCH_ARGS > gpurun_out/ab/e.json 2>gpurun_out/ab/e.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/e.json')); print('[$cfg]', round(d['ms_per_step']))" | tee -a gpurun_out/ab/env.txt
done
