# Official round measurement: GPU tests, smoke, both benches (C2 with CPU baseline), PMC + traces.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/bench_c2_full.log 2>&1
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > gpurun_out/bench_c3_full.log 2>&1
CFG=c2 bash tools/gpu_pmc.sh
CFG=c3 bash tools/gpu_pmc.sh
