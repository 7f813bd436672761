# Partitioned-mode GPU test on the pre-revert graph kernels (lib/libclsnap_gdue.so, commit
# 33695fc), then the C4/C5 A/B of the k_marker no-marker fast path against gbase.
O=$GRAFT_REPO_ROOT/gpurun_out/r02r
mkdir -p $O
CLSNAP_VARIANT=gdue timeout -k 10 300 python -u -m pytest tests/test_partition_gpu.py -q --timeout 200 --timeout-method thread > $O/part_gdue.log 2>&1
echo "gdue rc=$?"
set -e
for r in 1 2; do
  for v in gbase base; do
    if [ $v = base ]; then VAR=""; else VAR=$v; fi
    CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/ab_${v}_c4_$r.json 2>/dev/null
  done
done
for v in gbase base; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/ab_${v}_c5.json 2>/dev/null
done
