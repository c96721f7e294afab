set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/deftrace -o d -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data --no-transformer > gpurun_out/deftrace.log 2>&1 || exit 1
python3 tools/trace_summary.py gpurun_out/deftrace/d_kernel_trace.csv > gpurun_out/r4_deftrace_summary.txt 2>&1
