set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lanes_gpu.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err || exit $?
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
CFG=c3 SUFFIX=_r05 bash tools/gpu_pmc.sh || exit $?
CFG=c2 SUFFIX=_r05 bash tools/gpu_pmc.sh || exit $?
python3 tools/show_bench.py $O/bench_c3.json $O/bench_c2.json 2>/dev/null || tail -c 600 $O/bench_c3.json
