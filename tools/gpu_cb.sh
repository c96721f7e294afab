#!/bin/bash
# scratch GPU experiment (round 6): four-phase GEMM bench, GEMM bitwise tests, production
# golden, torch.library ops
set -o pipefail
mkdir -p gpurun_out
export ENSVS_RECORD_DIR=gpurun_out/r6_errors
timeout -k 10 300 python -u tools/p8_bench.py 30 > gpurun_out/p8_bench.log 2>&1
rc=$?; tail -12 gpurun_out/p8_bench.log; [ $rc -ne 0 ] && exit $rc
T="python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu -rf"
timeout -k 10 400 $T tests/test_gemm_bf16a_gpu.py tests/test_production_golden_gpu.py > gpurun_out/r6_tests_a.log 2>&1
rc=$?; tail -8 gpurun_out/r6_tests_a.log; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 500 $T tests/test_torch_ops_gpu.py tests/test_dropin_gpu.py > gpurun_out/r6_tests_b.log 2>&1
rc2=$?; tail -25 gpurun_out/r6_tests_b.log; exit $(( rc > rc2 ? rc : rc2 ))
