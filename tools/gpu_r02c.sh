# Graph engine with the 32-byte channel record: parity tests, C4 A/B vs the previous
# layout (lib/libclsnap_old.so), C5 with drain, C4 kernel trace + per-kernel HBM traffic.
set -e
mkdir -p gpurun_out/r02c
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02c/pytest_graph.log 2>&1
for r in 1 2; do for v in base old; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/r02c/ab_${v}_c4_$r.json 2>/dev/null
done; done
timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02c/bench_c5.json 2>/dev/null
CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c4 bash tools/gpu_pmc_graph.sh
