# PMC passes over a short bench run (each pass in its own rocprofv3 run; see MI355X_MICROARCH.md)
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc1 -o p -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/pmc2 -o p -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc3 -o p -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc4 -o p -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc4.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU_ADD_U32 --output-format csv -d $OUT/pmc5 -o p -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/pmc5.log 2>&1 || true
