set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "l2norm" > gpurun_out/r4_be_tests.log 2>&1 || exit 1
timeout -k 10 1000 bash tools/tree_ab.sh ab/base ab/pb2 ab/bn . > gpurun_out/r4_be_ab.txt 2>&1 || exit 3
