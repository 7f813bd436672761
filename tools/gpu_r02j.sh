# k_pick skips senders with nothing due (sender due word): graph + partition parity, C4 bench x2.
set -e
mkdir -p gpurun_out/r02j
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02j/pytest_graph.log 2>&1
for r in 1 2; do
timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02j/bench_c4_$r.json 2> gpurun_out/r02j/bench_c4_$r.err
done
CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
