set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 1100 bash tools/legs_ab.sh ab/old . > gpurun_out/r4_bc_ab.txt 2>&1 || exit 3
