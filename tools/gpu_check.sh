# GPU tests + smoke, then bench lines of the given configs (each step under its own limit).
# usage: TAG=r03a CFGS="c3 c4" bash tools/gpu_check.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-check}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 1200 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
fi
for c in ${CFGS:-}; do
  timeout -k 10 600 python -u bench.py --config $c ${BENCH_ARGS} > $O/bench_$c.json 2> $O/bench_$c.err
done
