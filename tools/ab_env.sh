# same-box A/B of environment settings: bash tools/ab_env.sh "A=1 B=2" "A=3" ...
mkdir -p gpurun_out/ab
for cfg in "$@"; do  # (the first run of a call tends to be slower: warm the box first)
  env $cfg timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/e.json 2>gpurun_out/ab/e.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/e.json')); print('[$cfg]', round(d['ms_per_step']))"
done
