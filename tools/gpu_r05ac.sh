set -e
# the lanes spill kernel at the 3-wave target too (CLSNAP_SPILL_W3) vs the compiler's choice
for r in 1 2; do
timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes | sed -e 's/sums=.*//'
CLSNAP_SPILL_W3=1 timeout -k 10 120 python -u tools/lanes_ab.py c3 20 lanes | sed -e 's/sums=.*//' -e 's/$/ spill_w3/'
done
