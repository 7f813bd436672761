set -e
# C5: the closure's begin-cursor read dropped (CLSNAP_VARIANT=ablrec, timing only: the recorded
# counter is wrong by construction) vs the tree
O=$GRAFT_REPO_ROOT/gpurun_out/r05am
mkdir -p $O
for r in 1 2; do
for v in base ablrec; do
if [ $v = ablrec ]; then export CLSNAP_VARIANT=ablrec; fi
timeout -k 10 300 python -u bench.py --config c5 --no-cpu-baseline --no-parity > $O/c5_${v}_$r.json 2> $O/c5_${v}_$r.err || true
unset CLSNAP_VARIANT
python3 -c "import json; d=json.loads(open('$O/c5_${v}_$r.json').read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'],1), d['phases']['drain']['us_per_tick'])"
done; done
