set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05l
mkdir -p $O; rm -f $O/ab.log
for r in 1 2; do
timeout -k 10 120 python -u tools/lanes_ab.py c3 10 lanes >> $O/ab.log 2>&1 || exit $?
CLSNAP_LANES_HEADER=$GRAFT_REPO_ROOT/tools/ab/cl_lanes_noinl.h timeout -k 10 120 python -u tools/lanes_ab.py c3 10 lanes >> $O/ab.log 2>&1 || exit $?
done
sed -e 's/sums=.*//' $O/ab.log
