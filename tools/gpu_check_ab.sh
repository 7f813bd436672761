# Every GPU test + smoke on the tree (gpu_tests.sh), then variant parity + interleaved exec A/B
# (gpu_exec_ab.sh without repeating the exec tests).  usage: VARIANTS="x y" TAG=r03j bash tools/gpu_check_ab.sh
set -e
TAG=${TAG:-check} bash tools/gpu_tests.sh
O=gpurun_out/${TAG:-check}
for v in $VARIANTS; do
  CLSNAP_VARIANT=$v timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest_$v.log 2>&1
done
rm -f gpurun_out/abx_*.log
VARIANTS="base $VARIANTS" CFGS="${CFGS:-c3 c2}" bash tools/gpu_ab_exec.sh
