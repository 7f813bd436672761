set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05h
mkdir -p $O; rm -f $O/ab.log
for r in 1 2; do
for d in "LANES_TAIL=0" "LANES_TAIL=1"; do
CLSNAP_LANES_DEFS=$d timeout -k 10 120 python -u tools/lanes_ab.py c3 >> $O/ab.log 2>&1 || exit $?
done; done
cat $O/ab.log | cut -c1-120
timeout -k 10 600 python -u -m pytest tests/test_lanes_gpu.py -x -q --timeout 300 --timeout-method thread > $O/lanes_tests.log 2>&1
rc=$?; tail -3 $O/lanes_tests.log; exit $rc
