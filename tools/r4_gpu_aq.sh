set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/as_dbg.py > gpurun_out/r4_as_dbg.txt 2>&1 || exit 1
bash tools/r4_gpu_an.sh
