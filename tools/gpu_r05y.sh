set -e
# the 8-GPU share (2^17): kernel timeline of back-to-back split reruns, and the bench line over more steps
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05y
mkdir -p $O
n=131072
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr$n -o tr -- python3 -u $R/tools/step_gap.py $n 0 lanes > $O/gap$n.log 2>&1
f=$(ls $O/tr$n/*/tr_kernel_trace.csv $O/tr$n/tr_kernel_trace.csv 2>/dev/null | head -n1 || true)
grep step_ms $O/gap$n.log
python3 $R/tools/trace_gaps.py $f
python3 - $f <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if "lanes" in r["Kernel_Name"] or "cl_exec" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[-12]["Start_Timestamp"])
for r in rows[-12:]:
    print(r["Kernel_Name"][:28], r.get("Queue_Id"), (int(r["Start_Timestamp"]) - t0) / 1e3, (int(r["End_Timestamp"]) - t0) / 1e3)
PY
cd $R
for r in 1 2; do
timeout -k 10 300 python -u bench.py --instances 131072 --steps 200 --warmup 20 --no-cpu-baseline --no-fresh --no-collect > $O/s17_$r.json 2> $O/s17_$r.err
python3 -c "import json,sys; d=json.loads(open('$O/s17_$r.json').read().strip().splitlines()[-1]); print('s17 steps 200', d['ms_per_step'], d['roofline']['kernel_ms'])"
done
