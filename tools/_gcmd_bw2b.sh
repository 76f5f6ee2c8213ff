set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bw2
timeout -k 10 900 python3 tools/whatif.py --reps 3 "" PPR_BW2=0 PPR_BW2=0 "" "" PPR_BW2=0 > gpurun_out/bw2/ab2.txt 2>&1
cat gpurun_out/bw2/ab2.txt
