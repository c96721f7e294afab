set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/wgrad_split_sweep.py > gpurun_out/r4_wgrad_sweep.txt 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_wgsweep_prof -o wg -- python3 tools/wgrad_split_sweep.py --splits > gpurun_out/r4_wgsweep_prof.log 2>&1 || exit 2
