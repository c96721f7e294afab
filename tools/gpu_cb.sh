#!/bin/bash
# round-6 GPU check: Transformer leg A/B of its 128-tile launches (M = 8 192, N = 256) on the
# 64 x 64 kernel (ensvs_set_small(3))
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u tools/flag_ab.py --tf "ensvs_set_small=1" "ensvs_set_small=3" > gpurun_out/small3_tf_ab.txt 2>&1
rc=$?; tail -6 gpurun_out/small3_tf_ab.txt; exit $rc
