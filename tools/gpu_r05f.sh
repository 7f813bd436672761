set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r05f
mkdir -p $O
for w in 3 4; do
CLSNAP_LANES_SPILL_NODES=1 CLSNAP_LANES_WAVES=$w timeout -k 10 300 python -u tools/lanes_check.py c3 > $O/lanes_w$w.log 2>&1
echo "w=$w rc=$?"; grep "engine=2\|equal" $O/lanes_w$w.log | cut -c1-150
done
