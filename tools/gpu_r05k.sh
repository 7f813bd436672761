set -e
CFG=c3 SUFFIX=_r05k bash tools/gpu_pmc.sh
cd $GRAFT_REPO_ROOT
for k in clsnap_lanes_nospill cl_exec_kernel; do echo "== $k"; python3 tools/pmc_summary.py gpurun_out/pmc_c3_r05k $k; done > gpurun_out/pmc_c3_r05k/summary.txt
grep -E "clsnap_lanes|cl_exec" gpurun_out/pmc_c3_r05k/trace/p_kernel_stats.csv | cut -c1-200
cat gpurun_out/pmc_c3_r05k/summary.txt
