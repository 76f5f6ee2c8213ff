# MC combine: PPR_DIAG bucket histograms, then env variants of the hub tiling (combine ms each)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/mcp
mkdir -p $OUT
PPR_DIAG=1 timeout -k 10 200 python3 bench.py --workload mc --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $OUT/diag.json 2> $OUT/diag.err || exit 1
grep ppr_diag $OUT/diag.err | head -60 > $OUT/diag.txt
for v in "" "PPR_HUB_TILE_CAND=2048" "PPR_HUB_TILE_CAND=1024" "PPR_HUB_SLICE=4096" "PPR_HUB_SLICE=16384" "PPR_HUB_BUCKET=256" "PPR_BW_NG=4"; do
  env $v timeout -k 10 200 python3 bench.py --workload mc --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $OUT/v.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('$OUT/v.json')); print('$v', round(d['phases']['combine_ms_per_step'],1), round(d['ms_per_step'],1))" >> $OUT/variants.txt
  echo "$v done"
done
