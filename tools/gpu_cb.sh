#!/bin/bash
# scratch GPU experiment (round 6): four-phase GEMM bench, torch.library ops, production golden,
# GEMM bitwise tests.  A heartbeat file keeps long single tests (compiles) from reading as hung;
# every step still has its own time limit.
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
export ENSVS_RECORD_DIR=gpurun_out/r6_errors
timeout -k 10 300 python -u tools/p8_bench.py 30 > gpurun_out/p8_bench.log 2>&1
rc=$?; tail -10 gpurun_out/p8_bench.log; [ $rc -ne 0 ] && exit $rc
T="python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu -rf"
timeout -k 10 700 $T -x tests/test_torch_ops_gpu.py > gpurun_out/r6_tests_b.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/r6_tests_b.log | tail -30; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 500 $T tests/test_production_golden_gpu.py tests/test_gemm_bf16a_gpu.py tests/test_dropin_gpu.py > gpurun_out/r6_tests_a.log 2>&1
rc2=$?; tail -8 gpurun_out/r6_tests_a.log; exit $(( rc > rc2 ? rc : rc2 ))
