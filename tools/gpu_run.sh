#!/bin/bash
# tools/gpu_run.sh TAG STEP... -- one GPU-box session of named steps, each under its own time limit,
# outputs under gpurun_out/TAG/ (run through gpurun: tools/gpu_run.sh is the command it executes).
#   tests[:K]   pytest -m gpu tests (K: a -k filter)
#   bench       bench.py default line (no cpu / e2e legs unless FULL=1)
#   diag        bench.py one step with PPR_DIAG=1 PPR_TIMING=1
#   env:VAR=X   export VAR=X for the following steps
#   ab:VAR=X[,VAR2=Y]  one bench line (2 steps, 1 warmup) with those variables set, ms_per_step printed
# Stops at the first failing step (a GPU fault, abort or time limit ends the session).
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
for step in "$@"; do
  case "$step" in
    tests*)
      k=${step#tests}; k=${k#:}
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread ${k:+-k "$k"} \
        > "$out/pytest.txt" 2>&1 || { echo "tests failed rc=$?"; tail -30 "$out/pytest.txt"; exit 1; } ;;
    bench)
      extra="--no-cpu-baseline --no-e2e"; [ "${FULL:-0}" = 1 ] && extra=""
      timeout -k 10 600 python -u bench.py --steps ${STEPS:-3} --warmup 1 $extra > "$out/bench.json" 2> "$out/bench.err" \
        || { echo "bench failed rc=$?"; tail -20 "$out/bench.err"; exit 1; }
      cat "$out/bench.json" ;;
    diag)
      PPR_DIAG=1 PPR_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
        > "$out/diag.json" 2> "$out/diag.err" || { echo "diag failed rc=$?"; tail -20 "$out/diag.err"; exit 1; }
      grep -E "ppr_diag|ppr_timing" "$out/diag.err" | head -40 ;;
    env:*)
      export "${step#env:}" ;;
    ab:*)
      vars=${step#ab:}; name=$(echo "$vars" | tr ',=' '_-')
      env $(echo "$vars" | tr ',' ' ') timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e \
        > "$out/ab_$name.json" 2> "$out/ab_$name.err" || { echo "ab $vars failed rc=$?"; tail -20 "$out/ab_$name.err"; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['ms_per_step'],1), 'ms/job merge', round(d['roofline']['merge_ms_per_step'],1), 'frac', round(d['roofline']['frac'],4))" "$out/ab_$name.json" "$vars" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
