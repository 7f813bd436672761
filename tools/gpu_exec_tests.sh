# Batch-engine GPU tests only (one pytest process).   usage: TAG=x bash tools/gpu_exec_tests.sh
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-exec}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_threaded_collect.py tests/test_trace_gpu.py \
  tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exec.log 2>&1
