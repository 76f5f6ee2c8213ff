# same-box A/B of the MC bench under environment settings: bash tools/mc_ab_env.sh "A=1 B=2" "A=3" ...
mkdir -p gpurun_out
for e in "$@"; do
  env $e timeout -k 10 200 python3 bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mcab.json 2>gpurun_out/mcab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/mcab.json')); print('[$e]', round(d['ms_per_step']), 'combine', round(d['phases']['combine_ms_per_step']))"
done
