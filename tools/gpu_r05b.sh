set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u tools/lanes_check.py c3 c2 > $O/lanes_check.log 2>&1
echo "rc=$?"; cat $O/lanes_check.log | tail -20
