#!/bin/bash
# round-6 GPU check: odd-channel fp32 weight gradients through bf16 copies (kernels.WGRAD_CAST)
# -- the wgrad / production tests, then the main line A/B
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -rf -x tests/test_gemm_gpu.py tests/test_production_golden_gpu.py tests/test_graph_cache_gpu.py tests/test_reductions_gpu.py > gpurun_out/wcast_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/wcast_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u tools/flag_ab.py "WGRAD_CAST=0" "WGRAD_CAST=1" > gpurun_out/wcast_ab.txt 2>&1
rc=$?; cat gpurun_out/wcast_ab.txt | tail -8; exit $rc
