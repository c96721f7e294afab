set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemm_bf16a_gpu.py tests/test_diffnet_gpu.py tests/test_gemm_big_gpu.py tests/test_encoders_gpu.py > gpurun_out/r4_az_tests.log 2>&1 || exit 1
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_az_ab.txt 2>&1 || exit 3
