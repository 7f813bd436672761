set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05p
mkdir -p $O; rm -f $O/ab.log
for n in 65536 131072 262144 524288; do
for e in nodes lanes; do
timeout -k 10 120 python -u tools/lanes_ab.py c3 20 $e $n >> $O/ab.log 2>&1 || exit $?
done; done
for e in nodes lanes; do timeout -k 10 120 python -u tools/lanes_ab.py c2 100 $e 131072 >> $O/ab.log 2>&1 || exit $?; done
cut -c1-80 $O/ab.log
