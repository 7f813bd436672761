set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05e
mkdir -p $O
timeout -k 10 300 python -u tools/lanes_check.py c3 > $O/lanes_a.log 2>&1
echo "a rc=$?"; grep rerun $O/lanes_a.log
CLSNAP_LANES_SPILL_NODES=1 timeout -k 10 300 python -u tools/lanes_check.py c3 > $O/lanes_b.log 2>&1
echo "b rc=$?"; cat $O/lanes_b.log
