# Partitioned mode on the device (2-3 ranks sharing the GPU over gloo) vs the oracle, then
# the graph suite (k_pick / k_marker / k_push now take the owned block range).
set -e
mkdir -p gpurun_out/r02i
timeout -k 10 500 python -u -m pytest tests/test_partition_gpu.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02i/pytest_part.log 2>&1
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02i/pytest_graph.log 2>&1
timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/r02i/bench_c4.json 2> gpurun_out/r02i/bench_c4.err
