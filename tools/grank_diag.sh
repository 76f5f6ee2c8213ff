# GRank headline workload with PPR_DIAG: bucket histograms, spills, sources beyond the bucket cap
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/diag
PPR_DIAG=1 timeout -k 10 300 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > gpurun_out/diag/g.json 2> gpurun_out/diag/g.err
grep ppr_diag gpurun_out/diag/g.err > gpurun_out/diag/g.txt
