set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/wi
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "speculative or tier_paths or multi" > gpurun_out/wi/spec_tests.txt 2>&1
tail -3 gpurun_out/wi/spec_tests.txt
PPR_TIMING=1 timeout -k 10 700 python3 tools/whatif.py "" "PPR_SPEC=0.5 PPR_SPEC_FROM=6" "PPR_SPEC=0.8 PPR_SPEC_FROM=6" "PPR_SPEC=0.5 PPR_SPEC_FROM=4" "PPR_SPEC=0.7 PPR_SPEC_FROM=8" "" > gpurun_out/wi/spec2.txt 2>&1
grep -v "^ppr_timing hub_planning" gpurun_out/wi/spec2.txt
