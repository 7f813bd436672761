# Cycle attribution (prof variants) of the exec kernel, per config.  usage: VARIANTS="prof profold" bash tools/gpu_prof_ab.sh
mkdir -p gpurun_out
for v in ${VARIANTS:-prof profold}; do
  for c in ${CFGS:-c3 c2}; do
    CLSNAP_VARIANT=$v timeout -k 10 200 python -u tools/prof_c2.py $c > gpurun_out/prof_${v}_$c.log 2>&1 || exit 2
  done
done
