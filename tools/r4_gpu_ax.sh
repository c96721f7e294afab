set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash tools/tree_ab.sh ab/base ab/s3 > gpurun_out/r4_ax_ab.txt 2>&1 || exit 3
