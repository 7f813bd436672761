set -e
# graph-engine kernel stats of the final tree (C4, C5)
CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c5 ARGS="--steps 1 --warmup 1" bash tools/gpu_prof_graph.sh
head -5 $GRAFT_REPO_ROOT/gpurun_out/prof_c5/kernel_stats.csv | cut -c1-150
