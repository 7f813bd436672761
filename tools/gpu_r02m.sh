# A/B of the sender due word (lib/libclsnap_predue.so = the tree before it) on C4 and C5,
# then a kernel-trace summary of one C5 run (trace kept in /tmp: 600k dispatches).
set -e
mkdir -p gpurun_out/r02m gpurun_out/prof_c5r02
for r in 1 2; do
  for v in predue base; do
    if [ $v = base ]; then VAR=""; else VAR=$v; fi
    CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/r02m/ab_${v}_c4_$r.json 2>/dev/null
    CLSNAP_VARIANT=$VAR timeout -k 10 200 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02m/ab_${v}_c5_$r.json 2>/dev/null
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pc5 -o p -- python3 $GRAFT_REPO_ROOT/bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c5r02/run.log 2>&1
find /tmp/pc5 -name "*kernel_stats.csv" -exec cp {} $GRAFT_REPO_ROOT/gpurun_out/prof_c5r02/kernel_stats.csv \;
