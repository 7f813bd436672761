set -e
CFG=c3 SUFFIX=_r05lanes bash tools/gpu_pmc.sh
cd $GRAFT_REPO_ROOT
python3 tools/pmc_summary.py gpurun_out/pmc_c3_r05lanes clsnap_lanes > gpurun_out/pmc_c3_r05lanes/summary.txt || true
