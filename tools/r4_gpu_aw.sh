set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/tree_ab.sh ab/base ab/v256 ab/v1024 > gpurun_out/r4_aw_ab.txt 2>&1 || exit 3
