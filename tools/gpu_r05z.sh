set -e
# fork stream2 per replay (CLSNAP_FORK_ALL=1, round-5 tree) or only after other work on the main stream
for r in 1 2; do
for n in 131072 1048576; do
timeout -k 10 120 python3 -u tools/step_gap.py $n 0 lanes | sed -e 's/$/ fork_dirty/'
CLSNAP_FORK_ALL=1 timeout -k 10 120 python3 -u tools/step_gap.py $n 0 lanes | sed -e 's/$/ fork_all/'
done; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_lanes_gpu.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -1
