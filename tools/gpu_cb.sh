#!/bin/bash
# round-6 GPU check: the 128 x 256 kernel restricted to long-K plain launches; the four-phase
# kernel's K loop without loads
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu -rf -x tests/test_gemm_p8h_gpu.py > gpurun_out/p8h_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/p8h_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/p8h_bench.py > gpurun_out/p8h_bench.txt 2>&1 || exit 5
cat gpurun_out/p8h_bench.txt
timeout -k 10 200 python -u tools/p8_bench.py > gpurun_out/p8_bench2.txt 2>&1 || exit 6
tail -2 gpurun_out/p8_bench2.txt
timeout -k 10 500 python -u tools/flag_ab.py "ensvs_set_p8h=0" "ensvs_set_p8h=1" > gpurun_out/ab_p8h.txt 2>&1
rc=$?; tail -4 gpurun_out/ab_p8h.txt; exit $rc
