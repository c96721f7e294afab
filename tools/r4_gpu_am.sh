set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_encoders_gpu.py tests/test_multitrack_gpu.py tests/test_bf16_copies_gpu.py tests/test_singletrack_gpu.py > gpurun_out/r4_am_tests.log 2>&1 || exit 1
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_bn_ab.txt 2>&1 || exit 2
