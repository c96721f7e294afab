set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py tests/test_diffnet_gpu.py > gpurun_out/r4_al_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/wgrad_bench.py > gpurun_out/r4_wgrad_big_bench2.txt 2>&1 || exit 2
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_wgrad_big_ab2.txt 2>&1 || exit 4
