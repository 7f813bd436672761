set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py -x -q --timeout 300 --timeout-method thread > $O/graph_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/graph_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
for v in "" "1"; do
CLSNAP_PICK_STAGE=$v timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/c4_$v$r.json 2>&1 || exit $?
done; done
for v in "" "1"; do
CLSNAP_PICK_STAGE=$v timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5_$v.json 2>&1 || exit $?
done
for f in $O/c4_*.json $O/c5_*.json; do python3 -c "
import json
d=json.loads([x for x in open('$f') if x.startswith('{')][-1])
print('$f'.split('/')[-1], 'ms', round(d['ms_per_step'],3), 'parity', d.get('parity'), d.get('phases',{}).get('drain',{}).get('us_per_tick'))
"; done
