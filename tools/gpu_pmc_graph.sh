# HBM traffic of the graph engine (configs c4/c5): FETCH_SIZE and WRITE_SIZE passes, each in
# its own rocprofv3 run (MI355X_MICROARCH.md HBM section), over one flush + one timed run.
# usage: CFG=c4|c5 [PASS_S=seconds per pass] [PMCG_ROOT=dir] bash tools/gpu_pmc_graph.sh   -> <root>/pmcg_<cfg>/pass{3,4}/
# (C5: ~10^6 dispatches per pass; the caller keeps a heartbeat file growing meanwhile)
set -e
CFG=${CFG:-c4}
OUT=${PMCG_ROOT:-$GRAFT_REPO_ROOT/gpurun_out}/pmcg_$CFG
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/bench.py
ARGS="--config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-parity"
timeout -s KILL ${PASS_S:-240} rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pass3 -o p -- python3 $P $ARGS > $OUT/pass3.log 2>&1
timeout -s KILL ${PASS_S:-240} rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pass4 -o p -- python3 $P $ARGS > $OUT/pass4.log 2>&1
