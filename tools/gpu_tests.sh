# Every GPU test (one pytest process) and smoke(), logs under gpurun_out/<tag>/.
# usage: TAG=r02s bash tools/gpu_tests.sh
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-tests}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
