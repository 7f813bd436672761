# Round measurement of the current tree, in two gpurun calls (each GPU step under its own
# limit, chained with set -e):
#   PART=bench  bench lines: c3 (default, with cpu_baseline), c3 at the per-GPU share of an
#               8-GPU node (2^17 instances), c2, c4 and c5 (with their cpu baselines), and a
#               2-rank gloo rehearsal of the multi-GPU path on one card
#   PART=prof   exec-kernel PMC + kernel stats (c3, c3 at 2^17, c2: tools/make_profiles.py
#               turns gpurun_out/pmc_* into profiles/); graph kernel stats (c4, c5) and C4's
#               HBM traffic, summarised on the box
#   PART=c5traffic  C5's HBM traffic with the drain (two ~9-minute counter passes)
#   PART=graph  the graph lines, kernel stats and C4 traffic only (after a graph-engine change)
# usage: TAG=r03f PART=bench bash tools/gpu_final.sh
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-final}
mkdir -p $O
if [ "${PART:-bench}" = c5traffic ]; then
  ( while true; do date >> $O/heartbeat.log; sleep 30; done ) &
  HB=$!
  PASS_S=540 PMCG_ROOT=/tmp CFG=c5 bash tools/gpu_pmc_graph.sh || { kill $HB; exit 1; }
  kill $HB
  PMCG_DIR=/tmp/pmcg_c5 OUT_DIR=$O/profiles python3 tools/graph_traffic.py c5 100000 4100 drain > $O/traffic_c5.log
elif [ "${PART:-bench}" = graph ]; then
  # the graph configs again after a graph-engine change: bench lines, kernel stats, C4 traffic
  timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
  timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
  CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
  CFG=c5 ARGS="--steps 1 --warmup 1" bash tools/gpu_prof_graph.sh
  PMCG_ROOT=/tmp CFG=c4 bash tools/gpu_pmc_graph.sh
  PMCG_DIR=/tmp/pmcg_c4 OUT_DIR=$O/profiles python3 tools/graph_traffic.py c4 1048576 80 > $O/traffic_c4.log
elif [ "${PART:-bench}" = bench ]; then
  timeout -k 10 300 python -u bench.py > $O/bench_c3.json 2> $O/bench_c3.err
  timeout -k 10 300 python -u bench.py --instances 131072 --no-cpu-baseline > $O/bench_c3_s17.json 2> $O/bench_c3_s17.err
  timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err
  timeout -k 10 300 python -u bench.py --config c4 --steps 10 --warmup 2 > $O/bench_c4.json 2> $O/bench_c4.err
  timeout -k 10 300 python -u bench.py --config c5 --steps 1 --warmup 1 > $O/bench_c5.json 2> $O/bench_c5.err
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 \
    bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu-baseline --dist-backend gloo --shared-device > $O/dist2_rehearsal.json 2> $O/dist2_rehearsal.err
else
  CFG=c3 bash tools/gpu_pmc.sh
  CFG=c3 SUFFIX=_s17 EXTRA="--instances 131072" bash tools/gpu_pmc.sh
  CFG=c2 bash tools/gpu_pmc.sh
  CFG=c4 ARGS="--steps 3 --warmup 1" bash tools/gpu_prof_graph.sh
  CFG=c5 ARGS="--steps 1 --warmup 1" bash tools/gpu_prof_graph.sh
  # (the graph passes' per-dispatch CSVs stay in /tmp on the box: C5 has ~10^6 dispatches;
  # only the traffic summaries come back, under $O/profiles)
  PMCG_ROOT=/tmp CFG=c4 bash tools/gpu_pmc_graph.sh
  PMCG_DIR=/tmp/pmcg_c4 OUT_DIR=$O/profiles python3 tools/graph_traffic.py c4 1048576 80 > $O/traffic_c4.log
  # (C5's traffic passes run ~20 min: PART=c5traffic, a call of their own)
fi
