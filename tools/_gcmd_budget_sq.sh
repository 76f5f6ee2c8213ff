set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 500 python3 tools/whatif.py "" PPR_HUB_BUDGET=16777216 PPR_HUB_BUDGET=8388608 "PPR_HUB_BUDGET=8388608 PPR_HUB_REGIONS=4" PPR_HUB_BUDGET=4194304 "" > gpurun_out/wi/budget.txt 2>&1
echo budget done
bash tools/sq_run.sh
