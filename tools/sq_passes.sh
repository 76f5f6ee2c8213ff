# SQ counter passes (one rocprofv3 run each, kernel trace off) over a short bench run
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--scale ${SCALE:-21} --iters ${ITERS:-6} --steps 1 --warmup 0 --no-cpu-baseline --no-e2e"
mkdir -p gpurun_out/sq
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d gpurun_out/sq/a -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/sq/a.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d gpurun_out/sq/b -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/sq/b.log 2>&1
python3 tools/sq_summary.py $(find gpurun_out/sq -name "*counter_collection.csv")
