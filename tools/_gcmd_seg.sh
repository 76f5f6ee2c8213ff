set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 700 python3 tools/whatif.py "" "PPR_HUB_SEG=1" "PPR_HUB_SEG=1 PPR_SEG_BUCKET=512 PPR_SEG_T=1024" "PPR_HUB_SEG=1 PPR_SEG_BUCKET=1024 PPR_SEG_T=1024" "PPR_HUB_SEG=1 PPR_SEG_BUCKET=1024 PPR_SEG_T=2048" "PPR_HUB_SEG=1 PPR_SEG_BUCKET=2048 PPR_SEG_T=2048" "" > gpurun_out/wi/seg.txt 2>&1
echo seg done
PPR_DIAG=1 PPR_HUB_SEG=1 PPR_SEG_BUCKET=1024 PPR_SEG_T=1024 timeout -k 10 300 python3 tools/whatif.py --reps 1 "" > gpurun_out/wi/segdiag.txt 2>&1
cat gpurun_out/wi/seg.txt; grep ppr_diag gpurun_out/wi/segdiag.txt | tail -8
