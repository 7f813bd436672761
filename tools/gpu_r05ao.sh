set -e
# the pop's second FIFO load dropped (CLSNAP_VARIANT=ablnrt: the next head's receiveTime faked as
# t + 1, timing only -- results wrong by construction) vs the tree, C4 and C5
O=$GRAFT_REPO_ROOT/gpurun_out/r05ao
mkdir -p $O
for r in 1 2; do
for v in base ablnrt; do
if [ $v = ablnrt ]; then export CLSNAP_VARIANT=ablnrt; fi
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline --no-parity > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || true
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-parity > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || true
unset CLSNAP_VARIANT
for c in c4 c5; do python3 -c "import json; d=json.loads(open('$O/${c}_${v}_$r.json').read().strip().splitlines()[-1]); print('$c $v', round(d['ms_per_step'],2), d['phases']['traffic']['us_per_tick'], d['phases']['drain']['us_per_tick'])" || true; done
done; done
