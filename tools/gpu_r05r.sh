set -o pipefail
# kernel timeline of back-to-back split reruns (2^17 and 2^20, C3 scenario)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05r
mkdir -p $O
for n in 131072 1048576; do
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/tr$n -o tr -- python3 -u $R/tools/step_gap.py $n 0 lanes > $O/gap$n.log 2>&1 || exit $?
f=$(ls $O/tr$n/*/tr_kernel_trace.csv $O/tr$n/tr_kernel_trace.csv 2>/dev/null | head -n1 || true)
cat $O/gap$n.log | grep step_ms
python3 $R/tools/trace_gaps.py $f
done
