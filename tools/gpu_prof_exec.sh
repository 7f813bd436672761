# Kernel-trace profile of a batch-engine bench run: usage CFG=c3 ARGS="..." TAG=x bash tools/gpu_prof_exec.sh
set -e
CFG=${CFG:-c3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-profx}_$CFG
rm -rf $OUT; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o p -- python3 $GRAFT_REPO_ROOT/bench.py --config $CFG --no-cpu-baseline $ARGS > $OUT/run.log 2>&1
