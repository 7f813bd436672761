set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05i
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench_c3.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --config c2 --steps 20 --warmup 3 > $O/bench_c2.log 2>&1 || exit $?
for f in $O/bench_c3.log $O/bench_c2.log; do python3 -c "
import json,sys
d=json.loads([x for x in open('$f') if x.startswith('{')][-1])
print(d['config']['workload'][:40], 'ms', round(d['ms_per_step'],4), 'value', '%.4g'%d['value'], 'parity', d['parity'], 'fresh', d['fresh_run'] and round(d['fresh_run']['fresh_run_ms'],3), 'kernel_ms', round(d['roofline']['kernel_ms'],4))
"; done
