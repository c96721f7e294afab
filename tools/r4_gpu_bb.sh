set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_graph_train_gpu.py tests/test_multitrack_gpu.py tests/test_bench_size_gpu.py tests/test_ddp_gpu.py tests/test_precision_trajectory_gpu.py > gpurun_out/r4_bb_tests.log 2>&1 || exit 1
