# Tiled weight repack: bitwise tests, repack timing, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_pack_gpu.py tests/test_multitrack_gpu.py tests/test_graph_train_gpu.py -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/pack_bench.py > gpurun_out/cb_pack.txt 2>&1 || exit 2
timeout -k 10 900 python -u tools/flag_ab.py "PACK_TILED=0" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
