set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 700 python3 tools/whatif.py "" PPR_TILE_SPLIT_LOGP=12 "PPR_SPEC=0.5 PPR_SPEC_FROM=6" PPR_NT=1 "" PPR_TILE_SPLIT_LOGP=12 > gpurun_out/wi/clean.txt 2>&1
cat gpurun_out/wi/clean.txt
