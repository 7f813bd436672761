# Full GPU suite with W4=5 as default, the default bench line (with cpu_baseline), C3/C2
# kernel-trace + PMC profiles of the current exec kernel.
set -e
mkdir -p gpurun_out/r02f
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02f/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r02f/bench_c3.json 2> gpurun_out/r02f/bench_c3.err
CFG=c3 bash tools/gpu_pmc.sh
CFG=c2 bash tools/gpu_pmc.sh
