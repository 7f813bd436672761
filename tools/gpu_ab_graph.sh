mkdir -p gpurun_out
for r in 1 2; do
for v in new old; do
  if [ $v = new ]; then VAR=""; else VAR=old; fi
  for c in c4 c5; do
    CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/abg_${v}_${c}_$r.log 2>&1 || exit 2
  done
done
done
