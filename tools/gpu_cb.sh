#!/bin/bash
# round-6 GPU check: the four-phase kernel's generic epilogue in two passes (no spills) --
# bitwise tests, per-launch times, main / SeparateF0 / Transformer A/B of mode 6 vs 7
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu -rf -x tests/test_gemm_p8h_gpu.py tests/test_gemm_big_gpu.py > gpurun_out/gen_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/gen_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/p8_bench.py > gpurun_out/p8_bench_gen.txt 2>&1 || exit 6
grep generic gpurun_out/p8_bench_gen.txt
timeout -k 10 550 python -u tools/flag_ab.py "ensvs_set_p8=6" "ensvs_set_p8=7" > gpurun_out/ab_gen_main.txt 2>&1 || exit 7
cat gpurun_out/ab_gen_main.txt
timeout -k 10 300 python -u tools/flag_ab.py --tf "ensvs_set_p8=6" "ensvs_set_p8=7" > gpurun_out/ab_gen_tf.txt 2>&1
rc=$?; cat gpurun_out/ab_gen_tf.txt; exit $rc
