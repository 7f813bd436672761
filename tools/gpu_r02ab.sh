# Batch-engine GPU tests on the current library, an interleaved A/B against head (the
# committed tree) on C2/C3, and the WRITE_SIZE of the current library on both.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r02ab}
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
cd /tmp && export TMPDIR=/tmp
for c in c2 c3; do
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w_$c -o p -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/w_$c.log 2>&1
done
