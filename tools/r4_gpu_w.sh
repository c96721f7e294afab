set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/dgrad_probe.py > gpurun_out/r4_dgrad_probe3.txt 2>&1 || exit 1
