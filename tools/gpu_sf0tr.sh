# kernel trace of graph-replayed SeparateF0 steps and its per-queue timeline
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sf0tr -o sf0 -- python3 tools/sf0_trace.py > gpurun_out/sf0tr.log 2>&1 || exit 1
python3 tools/sf0_trace.py --show gpurun_out/sf0tr/sf0_kernel_trace.csv 40 > gpurun_out/sf0tr_show.txt
