# Graph-engine change check: graph/partition/trace GPU tests on the tree's library, then an
# interleaved A/B of C4/C5 bench lines against lib/libclsnap_<v>.so variants.
# usage: VARIANTS="prev" TAG=r03e bash tools/gpu_graph_ab.sh
set -e
O=gpurun_out/${TAG:-graph}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_partition_gpu.py tests/test_graph_trace_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest_graph.log 2>&1
VARIANTS="base $VARIANTS" CFGS="${CFGS:-c4 c5}" bash tools/gpu_ab_graph.sh
