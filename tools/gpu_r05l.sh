set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05l
mkdir -p $O; rm -f $O/ab.log
for r in 1 2; do
timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes >> $O/ab.log 2>&1 || exit $?
CLSNAP_LANES_HEADER=$GRAFT_REPO_ROOT/tools/ab/cl_lanes_nopush.h timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes >> $O/ab.log 2>&1 || exit $?
done
cut -c1-120 $O/ab.log
CLSNAP_LANES_HEADER=$GRAFT_REPO_ROOT/tools/ab/cl_lanes_nopush.h timeout -k 10 600 python -u -m pytest tests/test_lanes_gpu.py -x -q --timeout 300 --timeout-method thread > $O/t.log 2>&1; rc=$?; tail -2 $O/t.log; exit $rc
