# Parity tests (default build), then A/B timing of library variants on C2 and C3.
# usage: VARIANTS="occ foo" bash tools/gpu_ab.sh
mkdir -p gpurun_out
rm -f gpurun_out/pytest_gpu.log gpurun_out/ab_*.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit 1
for v in base $VARIANTS; do
  for c in c2 c3; do
    if [ "$v" = base ]; then VAR=""; else VAR=$v; fi
    CLSNAP_VARIANT=$VAR timeout -k 10 120 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${v}_$c.log 2>&1 || exit 2
  done
done
