#!/bin/bash
# round-6 GPU check: the short-K N = 512 launches on the four-phase / 128 x 128 kernels
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/p8_shortk_bench.py > gpurun_out/p8_shortk.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/p8_shortk.txt | cut -c1-220; exit $rc
