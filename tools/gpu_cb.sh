# BatchNorm statistics merge in one load round trip: parity tests and A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_reductions_gpu.py tests/test_encoders_gpu.py tests/test_multitrack_gpu.py -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/flag_ab.py "layers.BN_STATS=0" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
