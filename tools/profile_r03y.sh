# Round-3 final profile set (80 % table fill, per-group budget checks) of the headline workload in the exact summation mode, under gpurun_out/r03y: the plain bench line, a kernel
# trace (rocpd db + stats csv), the FETCH_SIZE and WRITE_SIZE passes and two SQ passes, each
# rocprofv3 pass in a run of its own (MI355X_MICROARCH.md "rocprofv3 PMC slots").
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r03y
mkdir -p $OUT
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
echo bench done; cat $OUT/bench.json | head -c 1500; echo
ARGS="--steps 1 --warmup 1 --no-cpu-baseline --no-e2e"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv rocpd -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.json 2> $OUT/trace.err
echo trace done
P1="--steps 1 --warmup 0 --no-cpu-baseline --no-e2e"
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run -f csv -- python3 bench.py $P1 > $OUT/fetch.json 2> $OUT/fetch.err
echo fetch done
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run -f csv -- python3 bench.py $P1 > $OUT/write.json 2> $OUT/write.err
echo write done
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -d $OUT/sqa -o run -f csv -- python3 bench.py $P1 > $OUT/sqa.log 2>&1
echo sq a done
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM -d $OUT/sqb -o run -f csv -- python3 bench.py $P1 > $OUT/sqb.log 2>&1
echo sq b done
python3 tools/sq_summary.py $(find $OUT/sqa $OUT/sqb -name "*counter_collection.csv") > $OUT/sq_summary.txt
python3 tools/pmc_summary.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") 1 exact > $OUT/pmc.json
python3 tools/timeline.py $(find $OUT/trace -name "*results.db" | head -1) > $OUT/timeline.txt || true
python3 tools/kernel_roofline.py $(find $OUT/trace -name "*kernel_stats.csv" | head -1) $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") 2 1 $OUT/sq_summary.txt > $OUT/kernel_roofline.json || true
find $OUT -name "*counter_collection.csv" -size +20M -delete
find $OUT -name "*.db" -size +60M -delete
ls -la $OUT
