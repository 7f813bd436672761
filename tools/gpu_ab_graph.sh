# Interleaved A/B timing of graph-engine library variants on C4 and C5 (two rounds).
# usage: VARIANTS="old r1s9" bash tools/gpu_ab_graph.sh   (lib/libclsnap_<v>.so; "base" = lib/libclsnap.so)
mkdir -p gpurun_out
rm -f gpurun_out/abg_*.log
for r in 1 2; do
for v in ${VARIANTS:-base old}; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  for c in ${CFGS:-c4 c5}; do
    CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abg_${v}_${c}_$r.log 2>&1 || exit 2
  done
done
done
