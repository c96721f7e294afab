#!/bin/bash
# round-6 GPU check: kernel stats of the graph-replayed SeparateF0 step on the final tree
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sf0z -o sf0 -- python3 tools/sf0_trace.py > gpurun_out/sf0z.log 2>&1
rc=$?; tail -3 gpurun_out/sf0z.log; [ $rc -eq 0 ] || exit $rc
python3 tools/sf0_trace.py --show gpurun_out/sf0z/sf0_kernel_trace.csv > gpurun_out/sf0z_show.txt 2>&1; head -3 gpurun_out/sf0z_show.txt
