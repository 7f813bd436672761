# Checks and interleaved A/Bs of the tree on one GPU (each step under its own limit, chained with set -e):
#   STEPS (space-separated, default all): launch exec graph abx abg
#   launch  bench.py --gpus 2 rank launch on the shared device (tests/test_bench_launch.py -m gpu)
#   exec    batch-engine GPU tests (parity, trace, threaded collect, limits)
#   vtest   batch-engine parity tests on each variant library of VTESTS
#   graph   graph-engine GPU tests (graph, graph trace, partition)
#   gvtest  the same tests on each graph variant library of GVTESTS
#   abx     interleaved A/B of batch-engine variants (VARIANTS, lib/libclsnap_<v>.so) on CFGS
#   abg     interleaved A/B of graph-engine variants (GVARIANTS) on C4 and C5
#   tprof   per-dispatch kernel trace of one C4 run per graph variant, summarised on the box
# usage: TAG=r04a STEPS="exec abx" VARIANTS="hwreg" bash tools/gpu_ab.sh
set -e
O=gpurun_out/${TAG:-r04}
mkdir -p $O
PYT="python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu"
for s in ${STEPS:-launch exec graph abx abg}; do
  case $s in
    launch) timeout -k 10 400 $PYT tests/test_bench_launch.py > $O/pytest_launch.log 2>&1 ;;
    exec) timeout -k 10 900 $PYT tests/test_gpu_parity.py tests/test_trace_gpu.py tests/test_threaded_collect.py \
            tests/test_gpu_limits.py > $O/pytest_exec.log 2>&1 ;;
    vtest) for v in ${VTESTS}; do
             CLSNAP_VARIANT=$v timeout -k 10 900 $PYT tests/test_gpu_parity.py -k "not random_scenarios" > $O/pytest_var_$v.log 2>&1
           done ;;
    gvtest) for v in ${GVTESTS}; do
             CLSNAP_VARIANT=$v timeout -k 10 900 $PYT tests/test_graph_gpu.py tests/test_graph_trace_gpu.py \
               tests/test_partition_gpu.py > $O/pytest_gvar_$v.log 2>&1
           done ;;
    graph) timeout -k 10 900 $PYT tests/test_graph_gpu.py tests/test_graph_trace_gpu.py tests/test_partition_gpu.py \
            > $O/pytest_graph.log 2>&1 ;;
    abx) for r in 1 2; do for v in base ${VARIANTS}; do
           if [ $v = base ]; then VAR=""; else VAR=$v; fi
           for c in ${CFGS:-c3 c2}; do
             CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config $c --steps 50 --warmup 5 \
               --no-cpu-baseline --no-collect ${EXTRA} > $O/abx_${v}_${c}_$r.log 2>&1
           done; done; done ;;
    abg) for r in 1 2; do for v in base ${GVARIANTS}; do
           if [ $v = base ]; then VAR=""; else VAR=$v; fi
           for c in ${GCFGS:-c4 c5}; do
             CLSNAP_VARIANT=$VAR timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 \
               --no-cpu-baseline > $O/abg_${v}_${c}_$r.log 2>&1
           done; done; done ;;
    tprof) for v in base ${GVARIANTS}; do  # per-dispatch tick kernel durations (tools/tick_profile.py)
             if [ $v = base ]; then VAR=""; else VAR=$v; fi
             for c in ${GCFGS:-c4}; do
               T=/tmp/tprof_${v}_$c; rm -rf $T; mkdir -p $T
               ( cd /tmp && export TMPDIR=/tmp CLSNAP_VARIANT=$VAR && timeout -s KILL 240 rocprofv3 --kernel-trace \
                   --output-format csv -d $T -o p -- python3 $GRAFT_REPO_ROOT/bench.py --config $c --steps 1 --warmup 0 \
                   --no-cpu-baseline --no-parity > $GRAFT_REPO_ROOT/$O/tprof_${v}_$c.log 2>&1 )
               python3 tools/tick_profile.py $(find $T -name "*kernel_trace.csv" | head -1) $O/tprof_${v}_$c.json \
                 >> $O/tprof_${v}_$c.log
             done; done ;;
  esac
  echo "step $s done" >> $O/steps.log
done
