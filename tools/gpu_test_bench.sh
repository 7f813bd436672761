# One GPU round trip: parity tests, then the C2 and C3 benches (no CPU baseline).
mkdir -p gpurun_out
rm -f gpurun_out/pytest_gpu.log gpurun_out/bench*.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_c3.log 2>&1 || exit 3
