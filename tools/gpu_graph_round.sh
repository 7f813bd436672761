# Graph engine round measurement: graph parity tests, C4/C5 bench lines, kernel-trace
# profiles and the C4 HBM-traffic passes (each step under its own time limit).
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/graph_gpu.log 2>&1
timeout -k 10 300 python -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4.log 2>&1
timeout -k 10 300 python -u bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c5.log 2>&1
CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c5 ARGS="--steps 2 --warmup 1 --graph-steps 1000" bash tools/gpu_prof_graph.sh
CFG=c4 bash tools/gpu_pmc_graph.sh
