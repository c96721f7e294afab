# bn_stats_final with unconditional partial loads: bitwise tests, standalone timing, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reductions_gpu.py tests/test_encoders_gpu.py tests/test_multitrack_gpu.py tests/test_graph_train_gpu.py -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cb_bnprof -o bn -- python3 tools/bn_stats_probe.py > gpurun_out/cb_bn.log 2>&1 || exit 2
timeout -k 10 900 bash tools/lib_ab.sh ab/libensvs_HEAD.so "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
