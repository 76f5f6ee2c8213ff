# same-box A/B of the split epilogue on the chain-order wave tiers (GRank chain sum, MC combine)
mkdir -p gpurun_out/abc
for v in 0 256 0 256; do
  PPR_SUM=chain PPR_WAVE_SPLIT_CHAIN=$v timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/abc/c.json 2>gpurun_out/abc/c.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abc/c.json')); print('chain split $v', round(d['ms_per_step']))"
  PPR_WAVE_SPLIT_MC=$v timeout -k 10 200 python3 bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/abc/m.json 2>gpurun_out/abc/m.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/abc/m.json')); print('mc split $v', round(d['ms_per_step']), round(d['phases']['combine_ms_per_step']))"
done
