# exact-sum A/B variants in one process (tools/whatif.py), PPR_DIAG phase split
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xs
timeout -k 10 900 python -u tools/whatif.py --reps 1 "" "PPR_SUM=chain" "PPR_XR_T=4096 PPR_XR_W=8" "PPR_XR_FILL=40" "PPR_XR_RMAX=1" "PPR_XR_RMAX=8" "PPR_DIAG=1" "" > gpurun_out/xs/whatif3.txt 2>&1
cat gpurun_out/xs/whatif3.txt | grep -v "^ppr_diag [ 0-9]"
