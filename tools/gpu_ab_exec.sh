# Interleaved A/B of library variants on C2 and C3 (bench lines only; two rounds).
# usage: VARIANTS="base old" [CFGS="c2 c3"] [EXTRA="--instances 131072"] [SFX=_s17] bash tools/gpu_ab_exec.sh
mkdir -p gpurun_out
for r in 1 2; do
for v in ${VARIANTS:-base old}; do
  if [ $v = base ]; then VAR=""; else VAR=$v; fi
  for c in ${CFGS:-c2 c3}; do
    CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline ${EXTRA} > gpurun_out/abx_${v}_${c}${SFX}_$r.log 2>&1 || exit 2
  done
done
done
