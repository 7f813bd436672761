set -e
# round-5 final tree: GPU suite + smoke, every bench line (C3 default = 200 timed replays)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05ag
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --instances 131072 --no-cpu-baseline > $O/bench_c3_s17.json 2> $O/bench_c3_s17.err
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-cpu-baseline --dist-backend gloo --shared-device > $O/dist2_rehearsal.json 2> $O/dist2_rehearsal.err
python3 - $O <<'PY'
import glob, json, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(f.split("/")[-1], "ms", round(d["ms_per_step"], 4), "value %.3e" % d["value"], "parity", d.get("parity"),
          "kernel_ms", round(r.get("kernel_ms", 0), 4), "frac", round(r.get("frac", 0), 4))
PY
