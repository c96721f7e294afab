#!/bin/bash
# round-6 GPU check: the K loop without MFMAs; the Transformer leg by four-phase routing
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/p8_bench.py > gpurun_out/p8_bench4.txt 2>&1 || exit 6
tail -2 gpurun_out/p8_bench4.txt
timeout -k 10 900 python -u tools/flag_ab.py --tf "ensvs_set_p8=6" "ensvs_set_p8=7" "ensvs_set_p8=4" > gpurun_out/ab_tf_p8.txt 2>&1
rc=$?; cat gpurun_out/ab_tf_p8.txt; exit $rc
