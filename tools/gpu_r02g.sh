# D=3 instantiation (8nodes), sender-side packed pop counters, lane offsets on use:
# parity tests, A/B of 5 vs 6 waves/SIMD for D=3/4.
set -e
mkdir -p gpurun_out/r02g
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_trace_gpu.py tests/test_gpu_limits.py tests/test_threaded_collect.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02g/pytest.log 2>&1
for r in 1 2; do for v in base w6; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  CLSNAP_VARIANT=$VAR timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02g/ab_${v}_c3_$r.json 2>/dev/null
  CLSNAP_VARIANT=$VAR timeout -k 10 120 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02g/ab_${v}_c2_$r.json 2>/dev/null
done; done
