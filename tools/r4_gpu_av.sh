set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_encoders_gpu.py tests/test_multitrack_gpu.py tests/test_timing_gpu.py > gpurun_out/r4_av_tests.log 2>&1 || exit 1
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_av_ab.txt 2>&1 || exit 3
