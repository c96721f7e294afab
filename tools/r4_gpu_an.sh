set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_gemm_bf16a_gpu.py tests/test_diffnet_gpu.py tests/test_bf16_copies_gpu.py > gpurun_out/r4_an_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/dgrad_probe.py dil gate_bwd > gpurun_out/r4_as_probe.txt 2>&1 || exit 2
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_as_ab.txt 2>&1 || exit 3
