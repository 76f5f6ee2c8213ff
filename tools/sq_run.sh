# SQ counter passes over one RMAT-22 GRank job (one rocprofv3 run per pass), summary under gpurun_out/sq
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--scale ${SCALE:-22} --iters ${ITERS:-30} --steps 1 --warmup 0 --no-cpu-baseline --no-e2e"
OUT=gpurun_out/sq
mkdir -p $OUT
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d $OUT/a -o run --output-format csv -- python3 bench.py $ARGS > $OUT/a.log 2>&1
echo pass a done
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $OUT/b -o run --output-format csv -- python3 bench.py $ARGS > $OUT/b.log 2>&1
echo pass b done
python3 tools/sq_summary.py $(find $OUT -name "*counter_collection.csv") > $OUT/sq_summary.txt
find $OUT -name "*counter_collection.csv" -delete
