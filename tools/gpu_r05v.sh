set -e
# split A/B: spilling instances on NP (default) / lanes spill kernel / no split (all on the lanes spill kernel)
for n in 131072 1048576; do
for r in 1 2; do
for v in "" SPILL_LANES NO_SPLIT; do
if [ -n "$v" ]; then export CLSNAP_$v=1; fi
timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes $n | sed -e 's/sums=.*//' -e "s/\$/ $v/"
unset CLSNAP_SPILL_LANES CLSNAP_NO_SPLIT
done; done; done
