set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/dgrad_probe.py dil res_skip w_ih > gpurun_out/r4_big_probe.txt 2>&1 || exit 1
echo "== BIG" >> gpurun_out/r4_big_probe.txt
BIG=1 timeout -k 10 200 python3 -u tools/dgrad_probe.py dil res_skip w_ih >> gpurun_out/r4_big_probe.txt 2>&1 || exit 2
