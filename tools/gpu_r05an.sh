set -e
# recorded copies summed by k_finish (closures write the end cursor only): graph GPU tests, C4/C5 lines
O=$GRAFT_REPO_ROOT/gpurun_out/r05an
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tg.log 2>&1 || { tail -30 $O/tg.log; exit 1; }
tail -1 $O/tg.log
timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
for c in c4 c5; do python3 -c "import json; d=json.loads(open('$O/bench_$c.json').read().strip().splitlines()[-1]); print('$c', round(d['ms_per_step'],2), d['parity'], d['phases'], d['checks'])"; done
