# Round check of the current tree: every GPU test + smoke (gpu_tests.sh), then the bench
# lines (gpu_final.sh PART=bench).  usage: TAG=r03h bash tools/gpu_round.sh
set -e
TAG=${TAG:-round} bash tools/gpu_tests.sh
TAG=${TAG:-round} PART=bench bash tools/gpu_final.sh
