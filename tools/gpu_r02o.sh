# Batch-engine parity tests on the current library (node snapshot records), an interleaved
# A/B of exec-kernel variants on C2/C3, and the store counters (VMEM_WR, WRITE_SIZE) of the
# current library.   usage: VARIANTS="cur rec nostore" bash tools/gpu_r02o.sh
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/r02o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_threaded_collect.py tests/test_trace_gpu.py \
  tests/test_gpu_limits.py -x -q --timeout 300 --timeout-method thread > $O/pytest_exec.log 2>&1
for r in 1 2; do
  for v in ${VARIANTS:-cur rec nostore}; do
    for c in c2 c3; do
      CLSNAP_VARIANT=$v timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 3 --no-cpu-baseline \
        > $O/ab_${v}_${c}_$r.json 2>/dev/null
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for c in c2 c3; do
  A="--config $c --steps 3 --warmup 1 --no-cpu-baseline"
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/pmc_${c}_a -o p -- python3 $GRAFT_REPO_ROOT/bench.py $A > $O/pmc_${c}_a.log 2>&1
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_${c}_w -o p -- python3 $GRAFT_REPO_ROOT/bench.py $A > $O/pmc_${c}_w.log 2>&1
done
