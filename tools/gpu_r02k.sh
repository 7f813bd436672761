# Round-2 measurement of the current tree: all GPU tests, smoke, benches (C3 default with
# the CPU baseline, C2, C4, C5), kernel traces and PMC passes of the exec kernel (C3, C2).
set -e
mkdir -p gpurun_out/r02k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r02k/pytest_gpu.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02k/smoke.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r02k/bench_c3.json 2> gpurun_out/r02k/bench_c3.err
timeout -k 10 300 python -u bench.py --config c2 > gpurun_out/r02k/bench_c2.json 2> gpurun_out/r02k/bench_c2.err
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/r02k/bench_c4.json 2> gpurun_out/r02k/bench_c4.err
timeout -k 10 300 python -u bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r02k/bench_c5.json 2> gpurun_out/r02k/bench_c5.err
CFG=c3 bash tools/gpu_pmc.sh
CFG=c2 bash tools/gpu_pmc.sh
