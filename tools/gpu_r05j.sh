set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05j
mkdir -p $O; rm -f $O/ab.log
for r in 1 2; do
for v in "" "noearly"; do
CLSNAP_VARIANT=$v timeout -k 10 120 python -u tools/lanes_ab.py c2 300 nodes >> $O/ab.log 2>&1 || exit $?
CLSNAP_VARIANT=$v timeout -k 10 120 python -u tools/lanes_ab.py c3 20 nodes >> $O/ab.log 2>&1 || exit $?
done; done
cut -c1-110 $O/ab.log
