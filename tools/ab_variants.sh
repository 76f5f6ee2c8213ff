# same-box A/B of library variants: bash tools/ab_variants.sh "" base "" base  ("" = product build)
mkdir -p gpurun_out/ab
for v in "$@"; do
  PPR_LIB_VARIANT=$v timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/ab/v.json 2>gpurun_out/ab/v.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab/v.json')); print('variant [$v]', round(d['ms_per_step']))"
done
