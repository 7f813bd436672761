# Interleaved A/B of exec-kernel variants on C2/C3 (bench lines only).
set -e
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r02ac}
mkdir -p $O
for r in 1 2; do
  for v in ${VARIANTS:-head pushA pushB}; do
    for c in c2 c3; do
      CLSNAP_VARIANT=$v timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 3 --no-cpu-baseline \
        > $O/ab_${v}_${c}_$r.json 2>/dev/null
    done
  done
done
