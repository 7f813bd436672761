set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > $O/pytest_parity.log 2>&1
echo "pytest rc=$?"
tail -3 $O/pytest_parity.log
