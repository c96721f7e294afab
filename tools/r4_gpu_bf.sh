set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 bash tools/tree_ab.sh ab/x1 ab/base > gpurun_out/r4_bf_ab.txt 2>&1 || exit 3
