# Round measurement of the current tree (each GPU step under its own limit, chained):
#   bench lines: c3 (default, with cpu_baseline), c2, c4, c5; 2-rank rehearsal on one card;
#   exec-kernel PMC + kernel stats (c3, c2); graph kernel stats (c4, c5) and C4 HBM traffic.
# usage: TAG=r02f bash tools/gpu_final.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final}
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err
timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --dist-backend gloo --shared-device > $O/dist2_rehearsal.json 2> $O/dist2_rehearsal.err
CFG=c3 bash tools/gpu_pmc.sh
CFG=c2 bash tools/gpu_pmc.sh
CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c5 ARGS="--steps 1 --warmup 1" bash tools/gpu_prof_graph.sh
CFG=c4 bash tools/gpu_pmc_graph.sh
