# Graph engine: event-file-driven runs (streaming parsers, parallel send groups), all graph
# tests, C4 bench + kernel trace + per-kernel HBM traffic of the kept layout.
set -e
mkdir -p gpurun_out/r02h
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02h/pytest_graph.log 2>&1
timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 1 > gpurun_out/r02h/bench_c4.json 2> gpurun_out/r02h/bench_c4.err
CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c4 bash tools/gpu_pmc_graph.sh
