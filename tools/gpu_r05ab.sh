set -e
# C4: k_pick2 (two senders per thread, 4-B stage, one residency round) vs k_pick
O=$GRAFT_REPO_ROOT/gpurun_out/r05ab
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tg.log 2>&1 || { tail -30 $O/tg.log; exit 1; }
tail -1 $O/tg.log
for r in 1 2; do
CLSNAP_NO_PICK2=1 timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_off_$r.json 2> $O/c4_off_$r.err
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_on_$r.json 2> $O/c4_on_$r.err
done
python3 - $O <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/c4_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "ms", round(d["ms_per_step"], 3), "parity", d.get("parity"), d["phases"]["traffic"]["us_per_tick"])
PY
