set -e
cd $GRAFT_REPO_ROOT
PPR_MC_LEVEL_LOG=1 timeout -k 10 300 python -u bench.py --workload mc --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/mc_lv.json 2> gpurun_out/mc_lv.txt
python tools/mc_levels.py gpurun_out/mc_lv.txt > gpurun_out/mc_lv_summary.txt
