# Batch-engine parity tests on the current library (phase A/B loads issued together),
# then an interleaved A/B of exec-kernel variants on C2/C3 and a C4 FIFO-depth probe.
# usage: VARIANTS="cur lat" bash tools/gpu_r02n.sh
set -e
mkdir -p gpurun_out/r02n
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_threaded_collect.py tests/test_trace_gpu.py \
  tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r02n/pytest_exec.log 2>&1
for r in 1 2; do
  for v in ${VARIANTS:-cur lat}; do
    for c in c2 c3; do
      CLSNAP_VARIANT=$v timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 3 --no-cpu-baseline \
        > gpurun_out/r02n/ab_${v}_${c}_$r.json 2>/dev/null
    done
  done
done
for f in 16 4; do
  timeout -k 10 200 python -u bench.py --config c4 --graph-fifo $f --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/r02n/c4_fifo$f.json 2>/dev/null
done
