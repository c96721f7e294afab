#!/bin/bash
# round-6 GPU check: main line A/B of the N <= 128 launches on the 64 x 64 kernel
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u tools/flag_ab.py "ensvs_set_small=1" "ensvs_set_small=2" > gpurun_out/small2_ab.txt 2>&1
rc=$?; tail -6 gpurun_out/small2_ab.txt; exit $rc
