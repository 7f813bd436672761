# Full GPU suite (exec layout without the unused in-link LDS words; graph Logger trace),
# C2/C3 A/B of the W4=5 occupancy variant.
set -e
mkdir -p gpurun_out/r02d
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02d/pytest_gpu.log 2>&1
for r in 1 2; do for v in base w5; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  CLSNAP_VARIANT=$VAR timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02d/ab_${v}_c3_$r.json 2>/dev/null
  CLSNAP_VARIANT=$VAR timeout -k 10 120 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r02d/ab_${v}_c2_$r.json 2>/dev/null
done; done
