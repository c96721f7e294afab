#!/bin/bash
# round-6 GPU check: the 128 x 256 / 64 x 64 routing bitwise tests
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu -rf -x tests/test_gemm_p8h_gpu.py > gpurun_out/p8h_small_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/p8h_small_tests.log | tail -20; exit $rc
