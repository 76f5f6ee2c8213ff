for v in "" r3 pre s0 ""; do
  PPR_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/mcab.json 2>gpurun_out/mcab.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/mcab.json')); print('variant [$v]', round(d['ms_per_step']), 'combine', round(d['phases']['combine_ms_per_step']))"
done
