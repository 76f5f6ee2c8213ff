# exact-sum knob sweep on RMAT-22 (same process, one timed job each)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xs
timeout -k 10 900 python -u tools/whatif.py --reps 1 "" "PPR_XR_RMAX=2" "PPR_XR_RMAX=4" "PPR_XR_RMAX=6" "PPR_XR_RMAX=10" "PPR_XR_FILL=45" "PPR_XR_FILL=72" "PPR_XR_T=4096" "PPR_HUB_BUCKET=320" "PPR_HUB_BUCKET=640" "" > gpurun_out/xs/sweep.txt 2>&1
cat gpurun_out/xs/sweep.txt
