# PPR_DIAG of one MC job (per-kernel histograms printed at plan destruction): gpurun_out/mc_diag.err
mkdir -p gpurun_out
PPR_DIAG=1 PPR_TIMING=1 timeout -k 10 300 python3 -u bench.py --workload mc --steps 1 --warmup 0 --no-cpu-baseline \
  > gpurun_out/mc_diag.json 2> gpurun_out/mc_diag.err || exit 1
grep -E "ppr_diag|ppr_timing" gpurun_out/mc_diag.err | head -60
