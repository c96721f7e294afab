set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gemm_bf16a_gpu.py tests/test_diffnet_gpu.py > gpurun_out/r4_u_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/dgrad_probe.py > gpurun_out/r4_dgrad_probe2.txt 2>&1 || exit 2
