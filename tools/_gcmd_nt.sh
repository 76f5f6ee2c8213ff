set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 600 python3 tools/whatif.py "" PPR_NT=1 PPR_NT=2 PPR_NT=3 "" PPR_NT=1 > gpurun_out/wi/nt.txt 2>&1
cat gpurun_out/wi/nt.txt
