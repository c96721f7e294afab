#!/bin/bash
# round-6 GPU check: the four-phase kernel on the N = 256 launches (120 tiles of 256 x 256) --
# per-launch times, bitwise tests, main-line / SeparateF0 A/B
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/p8h_bench.py > gpurun_out/p8h_short_bench.txt 2>&1 || exit 4
grep -v amdgpu gpurun_out/p8h_short_bench.txt
timeout -k 10 550 python -u tools/flag_ab.py "ensvs_set_p8h=129" "ensvs_set_p8h=1" > gpurun_out/ab_p8h_short.txt 2>&1
rc=$?; cat gpurun_out/ab_p8h_short.txt; exit $rc
