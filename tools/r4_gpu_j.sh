set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_lstm_gpu.py tests/test_bf16_copies_gpu.py tests/test_encoders_gpu.py tests/test_multitrack_gpu.py > gpurun_out/r4_j_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/lstm_mfma_bench.py > gpurun_out/r4_lstm_mfma_bench_j.txt 2>&1 || exit 2
timeout -k 10 600 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_lstm_ab_j.txt 2>&1 || exit 3
