# PPR_DIAG phase breakdown + PPR_WHATIF stage costs on RMAT-22 (tools/whatif.py), under gpurun_out/wi
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/wi
mkdir -p $OUT
PPR_DIAG=1 timeout -k 10 300 python3 tools/whatif.py --reps 1 "" > $OUT/diag.txt 2>&1
echo diag done
timeout -k 10 600 python3 tools/whatif.py "" PPR_WHATIF=1 PPR_WHATIF=2 PPR_WHATIF=4 PPR_WHATIF=8 PPR_WHATIF=16 PPR_WHATIF=32 PPR_WHATIF=64 "" ${EXTRA} > $OUT/wi.txt 2>&1
echo whatif done
cat $OUT/wi.txt
