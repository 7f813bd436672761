# Graph-engine GPU tests on the current library, then an interleaved A/B on C4/C5 against
# lib/libclsnap_${GV:-g12}.so.
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r02g}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py \
  -x -q --timeout 300 --timeout-method thread > $O/pytest_graph.log 2>&1
for r in 1 2; do
  for v in ${GV:-g12} base; do
    if [ $v = base ]; then VAR=""; else VAR=$v; fi
    CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/ab_${v}_c4_$r.json 2>/dev/null
  done
done
for v in ${GV:-g12} base; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/ab_${v}_c5.json 2>/dev/null
done
