# Kernel-trace profile of a graph-engine bench run: usage CFG=c4 ARGS="..." bash tools/gpu_prof_graph.sh
set -e
CFG=${CFG:-c4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_$CFG
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o p -- python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu-baseline $ARGS > $OUT/run.log 2>&1
find $OUT -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
