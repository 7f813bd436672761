# Bench lines against the refreshed exec-kernel profiles (valu/traffic entries), and the
# C4 per-kernel HBM traffic of the due-word k_pick.
set -e
mkdir -p gpurun_out/r02l
timeout -k 10 300 python -u bench.py > gpurun_out/r02l/bench_c3.json 2> gpurun_out/r02l/bench_c3.err
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/r02l/bench_c2.json 2> gpurun_out/r02l/bench_c2.err
CFG=c4 bash tools/gpu_pmc_graph.sh
