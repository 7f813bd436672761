set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u tools/lanes_check.py c3s8 c3s2 c3 > $O/lanes_check.log 2>&1
echo "check rc=$?"; tail -8 $O/lanes_check.log


