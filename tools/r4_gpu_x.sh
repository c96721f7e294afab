set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python3 -u tools/hbm_write_probe.py > gpurun_out/r4_hbm_write.txt 2>&1 || exit 1
