# Every GPU test + smoke on the current library, then an interleaved A/B of the exec-kernel
# variants rec (node records) and tsm (+ close stores only for channels that recorded).
set -e
TAG=r02t bash tools/gpu_tests.sh
O=$GRAFT_REPO_ROOT/gpurun_out/r02t
for r in 1 2; do
  for v in rec tsm; do
    for c in c2 c3; do
      CLSNAP_VARIANT=$v timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 3 --no-cpu-baseline \
        > $O/ab_${v}_${c}_$r.json 2>/dev/null
    done
  done
done
