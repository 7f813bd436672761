# Batch-engine variant check: exec parity tests on the variant library, then interleaved A/B
# bench lines of base vs the variants.  usage: VARIANTS="x y" CFGS="c3 c2" TESTS=1 bash tools/gpu_ab_var.sh
set -e
mkdir -p gpurun_out
rm -f gpurun_out/abx_*.log gpurun_out/var_*.log
if [ -n "$TESTS" ]; then
  for v in $VARIANTS; do
    CLSNAP_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/var_$v.log 2>&1
  done
fi
VARIANTS="base $VARIANTS" bash tools/gpu_ab_exec.sh
