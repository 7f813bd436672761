# Kernel-trace profile of a graph-engine bench run: usage CFG=c4 ARGS="..." bash tools/gpu_prof_graph.sh
# (the per-dispatch trace stays in /tmp on the box -- C5 has ~370k dispatches per run; only the
# per-kernel stats and the run log come back under gpurun_out/)
set -e
CFG=${CFG:-c4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$CFG
TMP=/tmp/prof_$CFG
rm -rf $OUT $TMP; mkdir -p $OUT $TMP
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $TMP -o p -- python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu-baseline --no-parity $ARGS > $OUT/run.log 2>&1
find $TMP -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
