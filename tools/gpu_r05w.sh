set -e
# spilling instances on NP (default) or on the lanes spill kernel, 2^18 and 2^19
for n in 262144 524288; do
for r in 1 2; do
for v in "" SPILL_LANES; do
if [ -n "$v" ]; then export CLSNAP_$v=1; fi
timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes $n | sed -e 's/sums=.*//' -e "s/\$/ $v/"
unset CLSNAP_SPILL_LANES
done; done; done
