set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
PPR_DIAG=1 timeout -k 10 300 python3 tools/whatif.py --reps 1 "" > gpurun_out/wi/diag2.txt 2>&1
grep ppr_diag gpurun_out/wi/diag2.txt | tail -6
