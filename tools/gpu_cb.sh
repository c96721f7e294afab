#!/bin/bash
# round-6 GPU check: the 128 x 256 kernel's RELU_MASK instance -- tests, per-launch times
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu -rf -x tests/test_gemm_p8h_gpu.py > gpurun_out/p8h_rm_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/p8h_rm_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/p8h_bench.py > gpurun_out/p8h_rm_bench.txt 2>&1
rc=$?; grep -v amdgpu gpurun_out/p8h_rm_bench.txt | cut -c1-160; exit $rc
