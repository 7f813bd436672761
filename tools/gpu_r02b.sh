# Threaded-collector + graph tests (device drain), LDS ring-size sweep on C3 (occupancy),
# cycle attribution (prof build), C5 bench with the drain to completion.
set -e
mkdir -p gpurun_out/r02b
timeout -k 10 900 python -u -m pytest tests/test_threaded_collect.py tests/test_graph_gpu.py tests/test_gpu_parity.py -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r02b/pytest.log 2>&1
for s in 2 4 8; do
  timeout -k 10 120 python -u bench.py --fifo-slots $s --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02b/bench_c3_slots$s.json 2>/dev/null
done
CLSNAP_VARIANT=prof timeout -k 10 120 python tools/prof_c2.py c3 > gpurun_out/r02b/prof_cycles_c3.log 2>&1
CLSNAP_VARIANT=prof timeout -k 10 120 python tools/prof_c2.py c2 > gpurun_out/r02b/prof_cycles_c2.log 2>&1
timeout -k 10 600 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02b/bench_c5.json 2> gpurun_out/r02b/bench_c5.err
for r in 1 2; do for v in base rounds; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  CLSNAP_VARIANT=$VAR timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02b/ab_${v}_c3_$r.json 2>/dev/null
  CLSNAP_VARIANT=$VAR timeout -k 10 120 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02b/ab_${v}_c2_$r.json 2>/dev/null
done; done
