set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05l
mkdir -p $O; rm -f $O/ab.log
for r in 1 2; do
timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes >> $O/ab.log 2>&1 || exit $?
CLSNAP_LANES_HEADER=$GRAFT_REPO_ROOT/tools/ab/cl_lanes_lb2.h timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes >> $O/ab.log 2>&1 || exit $?
done
cut -c1-120 $O/ab.log
