set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/wgrad_split_sweep.py > gpurun_out/r4_wgrad_sweep.txt 2>&1 || exit 1
