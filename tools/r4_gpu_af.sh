set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/branch_times.py > gpurun_out/r4_defer2_branch_times.txt 2>&1 || exit 1
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_defer2_ab.txt 2>&1 || exit 2
