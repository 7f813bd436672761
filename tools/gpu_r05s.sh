set -o pipefail
# fused push + pick drain ticks: graph GPU tests, then C5 with and without it, C4 once
O=$GRAFT_REPO_ROOT/gpurun_out/r05s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tg.log 2>&1; rc=$?; tail -3 $O/tg.log; [ $rc = 0 ] || exit $rc
for r in 1 2; do
CLSNAP_NO_PUSHPICK=1 timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5_off_$r.json 2> $O/c5_off_$r.err || exit $?
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5_on_$r.json 2> $O/c5_on_$r.err || exit $?
done
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_on.json 2> $O/c4_on.err || exit $?
python3 - $O <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ph = d.get("phases", {})
    print(f.split("/")[-1], "ms", round(d["ms_per_step"], 2), "parity", d.get("parity"),
          "drain_us", round(ph.get("drain", {}).get("us_per_tick", 0), 2),
          "traffic_us", round(ph.get("traffic", {}).get("us_per_tick", 0), 2), "status", d.get("status"))
PY
