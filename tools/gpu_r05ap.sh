set -e
# final tree: the whole GPU suite, verbose log for profiles/
O=$GRAFT_REPO_ROOT/gpurun_out/r05ap
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
