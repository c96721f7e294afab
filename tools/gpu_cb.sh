# SeparateF0 decoder start order: parity test and A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_separate_f0.py -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 900 python tools/flag_ab.py --sf0 "acoustic_models.DEC_ORDER=0" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
