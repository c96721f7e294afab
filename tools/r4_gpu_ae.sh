set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/branch_times.py > gpurun_out/r4_defer_branch_times.txt 2>&1 || exit 1
