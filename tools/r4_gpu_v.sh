set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_gbw_ab.txt 2>&1 || exit 1
