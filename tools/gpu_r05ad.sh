set -e
# C4 pop-line ablations (timing only, results wrong by construction): 1 = no tokcnt atomic,
# 4 = no route load (receiver and in-position hashed from the channel)
O=$GRAFT_REPO_ROOT/gpurun_out/r05ad
mkdir -p $O
for r in 1 2; do
for a in 0 1 4; do
CLSNAP_ABL_PICK=$a timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $O/c4_abl${a}_$r.json 2> $O/c4_abl${a}_$r.err || true
python3 -c "import json; d=json.loads(open('$O/c4_abl${a}_$r.json').read().strip().splitlines()[-1]); print('abl $a', round(d['ms_per_step'],3), d['phases']['traffic']['us_per_tick'], d.get('parity'))"
done; done
