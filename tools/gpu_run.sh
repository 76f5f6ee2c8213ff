#!/bin/bash
# tools/gpu_run.sh TAG STEP... -- one GPU-box session of named steps, each under its own time limit,
# outputs under gpurun_out/TAG/ (run through gpurun: tools/gpu_run.sh is the command it executes).
#   tests[:K]   pytest -m gpu tests (K: a -k filter)
#   bench       bench.py default line (no cpu / e2e legs unless FULL=1)
#   e2e         tests/cpp/_dropin_test e2e (ppr::grank through include/ppr/grank.h, PPR_TIMING split)
#   diag        bench.py one step with PPR_DIAG=1 PPR_TIMING=1
#   prof        rocprofv3 --kernel-trace --stats over one job (+1 warmup): kernel_stats.csv, timeline
#   sq          two SQ counter passes (one rocprofv3 run each) over one job: sq_summary.txt
#   pmc         FETCH_SIZE and WRITE_SIZE passes over one job: pmc.json (tools/pmc_summary.py)
#   mctrace     kernel trace of one MC job, per-level breakdown (tools/mc_trace.py): mc_trace.txt
#   mclog       PPR_MC_LEVEL_LOG per-level times of one MC job (tools/mc_levels.py): mc_levels.txt
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
    e2e)
      PPR_TIMING=1 PPR_HEAP_PAD=64 timeout -k 10 300 tests/cpp/_dropin_test e2e ${E2E_SCALE:-22} 30 > "$out/e2e.json" \
        2> "$out/e2e.err" || { echo "e2e failed rc=$?"; tail -20 "$out/e2e.err"; exit 1; }
      cat "$out/e2e.json"; grep ppr_timing "$out/e2e.err" ;;
    diag)
      PPR_DIAG=1 PPR_TIMING=1 timeout -k 10 300 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
        > "$out/diag.json" 2> "$out/diag.err" || { echo "diag failed rc=$?"; tail -20 "$out/diag.err"; exit 1; }
      grep -E "ppr_diag|ppr_timing" "$out/diag.err" | head -40 ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp) ; export TMPDIR=/tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv rocpd -d "$out/prof" -o run -- python3 bench.py --steps 1 --warmup 1 \
        --no-cpu-baseline --no-e2e > "$out/prof.json" 2> "$out/prof.err" || { echo "prof failed rc=$?"; tail -20 "$out/prof.err"; exit 1; }
      ks=$(find "$out/prof" -name "*kernel_stats.csv" | head -1); cp "$ks" "$out/kernel_stats.csv"
      db=$(find "$out/prof" -name "*results.db" | head -1)
      python3 tools/timeline.py "$db" > "$out/timeline.txt" 2>/dev/null || true
      find "$out/prof" -name "*.db" -size +60M -delete
      head -25 "$out/kernel_stats.csv" | cut -d, -f1-8 ;;
    sq)
      export TMPDIR=/tmp
      P1="--steps 1 --warmup 0 --no-cpu-baseline --no-e2e"
      timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM \
        -d "$out/sqa" -o run -f csv -- python3 bench.py $P1 > "$out/sqa.log" 2>&1 || { echo "sq a failed"; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM \
        -d "$out/sqb" -o run -f csv -- python3 bench.py $P1 > "$out/sqb.log" 2>&1 || { echo "sq b failed"; exit 1; }
      python3 tools/sq_summary.py $(find "$out/sqa" "$out/sqb" -name "*counter_collection.csv") > "$out/sq_summary.txt"
      find "$out/sqa" "$out/sqb" -name "*counter_collection.csv" -size +20M -delete
      head -60 "$out/sq_summary.txt" ;;
    pmc)
      export TMPDIR=/tmp
      P1="--steps 1 --warmup 0 --no-cpu-baseline --no-e2e"
      timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$out/fetch" -o run -f csv -- python3 bench.py $P1 > "$out/fetch.json" 2> "$out/fetch.err" || { echo "fetch failed"; exit 1; }
      timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$out/write" -o run -f csv -- python3 bench.py $P1 > "$out/write.json" 2> "$out/write.err" || { echo "write failed"; exit 1; }
      python3 tools/pmc_summary.py $(find "$out/fetch" -name "*counter_collection.csv") $(find "$out/write" -name "*counter_collection.csv") 1 exact > "$out/pmc.json"
      python3 tools/stamp_build.py "$out/pmc.json"
      # per-kernel roofline join (needs the prof step's stats of this session; sq optional)
      if [ -f "$out/kernel_stats.csv" ]; then
        sqf=-; [ -f "$out/sq_summary.txt" ] && sqf="$out/sq_summary.txt"
        python3 tools/kernel_roofline.py "$out/kernel_stats.csv" $(find "$out/fetch" -name "*counter_collection.csv" | head -1) \
          $(find "$out/write" -name "*counter_collection.csv" | head -1) 2 1 "$sqf" "$out/prof.json" > "$out/kernel_roofline.json" \
          || echo "kernel_roofline failed"
      fi
      find "$out/fetch" "$out/write" -name "*counter_collection.csv" -size +20M -delete
      head -c 1500 "$out/pmc.json" ;;
    mctrace)
      export TMPDIR=/tmp
      timeout -k 10 400 rocprofv3 --kernel-trace -f csv -d "$out/mct" -o run -- python3 bench.py --workload mc --steps 1 --warmup 0 \
        --no-cpu-baseline --no-e2e > "$out/mct.json" 2> "$out/mct.err" || { echo "mctrace failed rc=$?"; tail -20 "$out/mct.err"; exit 1; }
      python3 tools/mc_trace.py $(find "$out/mct" -name "*kernel_trace.csv" | head -1) > "$out/mc_trace.txt"
      find "$out/mct" -name "*kernel_trace.csv" -size +40M -delete
      head -30 "$out/mc_trace.txt" ;;
    mclog)
      PPR_MC_LEVEL_LOG=1 timeout -k 10 300 python -u bench.py --workload mc --steps 1 --warmup 0 --no-cpu-baseline --no-e2e \
        > "$out/mclog.json" 2> "$out/mclog.err" || { echo "mclog failed rc=$?"; tail -20 "$out/mclog.err"; exit 1; }
      python3 tools/mc_levels.py "$out/mclog.err" > "$out/mc_levels.txt"; cat "$out/mc_levels.txt" ;;
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
