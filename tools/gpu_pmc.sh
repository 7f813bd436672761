# PMC passes over a short bench run (each pass in its own rocprofv3 run; see MI355X_MICROARCH.md)
# usage: CFG=c2|c3 [SUFFIX=_x EXTRA="--instances N"] bash tools/gpu_pmc.sh   -> gpurun_out/pmc_<cfg><suffix>/pass*/
set -e
CFG=${CFG:-c2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_$CFG${SUFFIX}
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-fresh ${EXTRA}"
P=$GRAFT_REPO_ROOT/bench.py
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- python3 $P --config $CFG --no-cpu-baseline ${EXTRA} > $OUT/trace.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/pass1 -o p -- python3 $P $ARGS > $OUT/pass1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --output-format csv -d $OUT/pass2 -o p -- python3 $P $ARGS > $OUT/pass2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pass3 -o p -- python3 $P $ARGS > $OUT/pass3.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pass4 -o p -- python3 $P $ARGS > $OUT/pass4.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_LDS_UNALIGNED_STALL --output-format csv -d $OUT/pass5 -o p -- python3 $P $ARGS > $OUT/pass5.log 2>&1
