# Graph tests, the C4/C5 bench lines, their kernel stats and C4's HBM traffic (current tree).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r02t4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py \
  -x -q --timeout 300 --timeout-method thread > $O/pytest_graph.log 2>&1
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c5 ARGS="--steps 1 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c4 bash tools/gpu_pmc_graph.sh
