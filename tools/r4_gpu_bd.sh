set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread tests/test_graph_train_gpu.py tests/test_multitrack_gpu.py tests/test_bench_size_gpu.py > gpurun_out/r4_bd_tests.log 2>&1 || exit 1
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_bd_ab.txt 2>&1 || exit 3
