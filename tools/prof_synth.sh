set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_synth -o run -- python3 tools/synth_probe.py 1 > gpurun_out/prof_synth.log 2>&1
find gpurun_out/prof_synth -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/synth_kernel_stats.csv
