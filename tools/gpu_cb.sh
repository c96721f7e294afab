#!/bin/bash
# round-6 GPU check: the main step's N = 128 launches on the 128 x 128 / 64 x 64 kernels
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/n128_bench.py > gpurun_out/n128_bench.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/n128_bench.txt | cut -c1-220; exit $rc
