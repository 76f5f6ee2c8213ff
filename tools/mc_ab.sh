# same-box A/B of library variants on the MC workload: bash tools/mc_ab.sh "" base "" base  ("" = product build)
mkdir -p gpurun_out/ab
for v in "$@"; do
  PPR_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --workload mc --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/mc.json 2>gpurun_out/ab/mc.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/mc.json')); print('mc variant [$v]', round(d['ms_per_step']), 'combine', round(d['phases']['combine_ms_per_step']))"
done
