#!/bin/bash
# scratch GPU experiment (round 6): lean-epilogue four-phase GEMM bench, torch.library ops,
# step A/B: hipBLASLt route vs the engine (p8 for the gate GEMMs / for every eligible launch)
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u tools/p8_bench.py 30 > gpurun_out/p8_bench.log 2>&1
rc=$?; tail -11 gpurun_out/p8_bench.log; [ $rc -ne 0 ] && exit $rc
T="python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu -rf"
timeout -k 10 700 $T tests/test_torch_ops_gpu.py > gpurun_out/r6_tests_b.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error |error:" gpurun_out/r6_tests_b.log | tail -30; case $rc in 124|137|134|139) exit $rc;; esac
timeout -k 10 900 python -u tools/flag_ab.py "" "BLAS=0" "BLAS=0,ensvs_set_p8=2" > gpurun_out/r6_blas_ab.txt 2>&1
rc2=$?; cat gpurun_out/r6_blas_ab.txt | tail -8; [ $rc2 -ne 0 ] && exit $rc2
timeout -k 10 900 python -u tools/flag_ab.py --sf0 "" "BLAS=0" "BLAS=0,ensvs_set_p8=2" > gpurun_out/r6_blas_ab_sf0.txt 2>&1
rc3=$?; cat gpurun_out/r6_blas_ab_sf0.txt | tail -8
exit $(( rc > rc3 ? rc : rc3 ))
