set -e
# k_marker: every marker counts its close beside the creation-key load (this build) vs the committed build
O=$GRAFT_REPO_ROOT/gpurun_out/r05aq
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tg.log 2>&1 || { tail -30 $O/tg.log; exit 1; }
tail -1 $O/tg.log
for r in 1 2; do
for v in base new; do
if [ $v = base ]; then export CLSNAP_VARIANT=base; fi

timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err
unset CLSNAP_VARIANT
done; done
python3 - $O <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c*_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    ph = d["phases"]
    print(f.split("/")[-1], "ms", round(d["ms_per_step"], 3), "parity", d.get("parity"),
          "traffic_us", round(ph["traffic"]["us_per_tick"], 2), "drain_us", round(ph["drain"]["us_per_tick"], 2))
PY
