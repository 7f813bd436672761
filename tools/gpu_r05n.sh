set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05n
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; tail -2 $O/smoke.log; exit $rc
