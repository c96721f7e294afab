set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gemm_bf16a_gpu.py -k "addscale_dma or gate_bwd_dma" > gpurun_out/r4_ao_tests.log 2>&1
echo rc=$? >> gpurun_out/r4_ao_tests.log
