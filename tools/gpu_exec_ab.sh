# Exec-engine change check: the batch engine's GPU tests on the tree's library, then an
# interleaved A/B of C3/C2 bench lines against lib/libclsnap_<v>.so variants.
# usage: VARIANTS="old" TAG=r03i bash tools/gpu_exec_ab.sh
set -e
O=gpurun_out/${TAG:-exec}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_trace_gpu.py tests/test_threaded_collect.py tests/test_gpu_limits.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_exec.log 2>&1
for v in $VARIANTS; do
  CLSNAP_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
done
rm -f gpurun_out/abx_*.log
VARIANTS="base $VARIANTS" CFGS="${CFGS:-c3 c2}" bash tools/gpu_ab_exec.sh
