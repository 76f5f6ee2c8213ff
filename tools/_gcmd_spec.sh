set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 600 python3 tools/whatif.py "" PPR_SPEC=0.5 PPR_SPEC=0.8 PPR_SPEC=0.95 "" > gpurun_out/wi/spec.txt 2>&1
cat gpurun_out/wi/spec.txt
for r in 0.5 0.8 0.95; do
PPR_DIAG=1 PPR_SPEC=$r timeout -k 10 300 python3 tools/whatif.py --reps 1 "" > gpurun_out/wi/specdiag_$r.txt 2>&1
grep "speculative\|hub final" gpurun_out/wi/specdiag_$r.txt
done
