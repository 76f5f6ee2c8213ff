# exact-sum knob sweep (same process)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xs
timeout -k 10 1000 python -u tools/whatif.py --reps 1 "" "PPR_XR_RMAX=2" "PPR_XR_RMAX=4" "PPR_XR_FILL=50" "PPR_XR_FILL=70" "PPR_XR_T=4096" "PPR_HUB_BUDGET=134217728" "PPR_HUB_MIX=0" "" > gpurun_out/xs/whatif6.txt 2>&1
cat gpurun_out/xs/whatif6.txt
