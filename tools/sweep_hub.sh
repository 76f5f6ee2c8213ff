set -e
mkdir -p gpurun_out/sweep
for cfg in "384 512" "256 512" "512 1024" "768 1024" "320 512" "448 512"; do
  set -- $cfg
  PPR_HUB_BUCKET=$1 PPR_HUB_WAVE_T=$2 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/sweep/b_$1_$2.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/sweep/b_$1_$2.json')); print('bucket $1 T $2', round(d['ms_per_step']))"
done
