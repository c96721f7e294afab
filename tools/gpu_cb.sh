#!/bin/bash
# round-6 GPU check: the 128 x 256 kernel's epilogue with operands prefetched 8 rows ahead --
# bitwise tests, per-launch times
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu -rf -x tests/test_gemm_p8h_gpu.py > gpurun_out/p8h_epi_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/p8h_epi_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 550 python -u tools/flag_ab.py "ensvs_set_p8h=3" "ensvs_set_p8h=1" > gpurun_out/ab_p8h_ops.txt 2>&1
rc=$?; cat gpurun_out/ab_p8h_ops.txt; exit $rc
