set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05g
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1500 $O/bench.log; exit $rc
