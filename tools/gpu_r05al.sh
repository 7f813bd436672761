set -e
# lanes kernel: AMDGPU scheduling strategies for the hipRTC compile (A/B)
for r in 1 2; do
for v in "" "-amdgpu-sched-strategy=max-ilp" "-amdgpu-sched-strategy=max-memory-clause" "-amdgpu-sched-strategy=iterative-ilp" "-amdgpu-schedule-metric-bias=0"; do
if [ -n "$v" ]; then export CLSNAP_JIT_MLLVM="$v"; fi
timeout -k 10 180 python -u tools/lanes_ab.py c3 20 lanes | sed -e 's/sums=\(.\{40\}\).*/sums=\1/' -e "s/\$/ $v/" || echo "failed $v"
unset CLSNAP_JIT_MLLVM
done; done
