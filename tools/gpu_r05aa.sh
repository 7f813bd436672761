set -e
# fork-when-dirty + start event on the main dispatch: parity/lanes tests, step gaps, bench lines
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_lanes_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1 || { tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for n in 131072 1048576; do timeout -k 10 120 python3 -u tools/step_gap.py $n 0 lanes; done
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --instances 131072 --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_c3_s17.json 2> $O/bench_c3_s17.err
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --dist-backend gloo --shared-device > $O/dist2_rehearsal.json 2> $O/dist2_rehearsal.err
python3 - $O <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(f.split("/")[-1], "ms", round(d["ms_per_step"], 4), "value %.3e" % d["value"], "parity", d.get("parity"),
          "kernel_ms", round(r.get("kernel_ms", 0), 4), "frac", round(r.get("frac", 0), 4), r.get("kernel"))
PY
