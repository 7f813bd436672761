set -e
mkdir -p gpurun_out/r03s
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_trace_gpu.py tests/test_threaded_collect.py tests/test_gpu_limits.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03s/pytest.log 2>&1
VARIANTS="base old" CFGS="c3 c2" bash tools/gpu_ab_exec.sh
