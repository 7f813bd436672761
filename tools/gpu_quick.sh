# Parity tests, C2/C3 benches (no CPU baseline), cycle attribution of the prof variant.
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1
timeout -k 10 120 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c3.log 2>&1
if [ -f chandy-lamport-distributed-snapshot-algorithm_amd/lib/libclsnap_prof.so ]; then
  CLSNAP_VARIANT=prof timeout -k 10 120 python tools/prof_c2.py c2 > gpurun_out/prof_cycles_c2.log 2>&1
  CLSNAP_VARIANT=prof timeout -k 10 120 python tools/prof_c2.py c3 > gpurun_out/prof_cycles_c3.log 2>&1
fi
