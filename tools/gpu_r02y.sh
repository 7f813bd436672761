# Batch-engine GPU tests on the current library (replays through a length-ordered slot
# map), then an interleaved A/B vs head (the committed tree).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r02zb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_threaded_collect.py tests/test_trace_gpu.py \
  tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exec.log 2>&1
for r in 1 2; do
  for v in head base; do
    if [ $v = base ]; then VAR=""; else VAR=$v; fi
    for c in c2 c3; do
      CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 3 --no-cpu-baseline \
        > $O/ab_${v}_${c}_$r.json 2>/dev/null
    done
  done
done
