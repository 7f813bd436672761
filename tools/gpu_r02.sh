# Round-2 measurement pass: GPU parity tests, the default bench line (north_star batch,
# with cpu_baseline), kernel-trace + PMC passes of it, and a 2-rank rehearsal of the
# multi-GPU path on one card (gloo collective, both ranks on cuda:0).
set -e
mkdir -p gpurun_out/r02
R=$GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r02/pytest_gpu.log 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r02/bench_c3.json 2> gpurun_out/r02/bench_c3.err
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > gpurun_out/r02/bench_c2.json 2> gpurun_out/r02/bench_c2.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --dist-backend gloo --shared-device > gpurun_out/r02/dist2_rehearsal.json 2> gpurun_out/r02/dist2_rehearsal.err
CFG=c3 bash tools/gpu_pmc.sh
