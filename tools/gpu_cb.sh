# SeparateF0 bf16-copy / deferred decoder gradients: parity tests, then an interleaved A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_separate_f0.py -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_lstm_gpu.py -k coop tests/test_reductions_gpu.py >> gpurun_out/cb_tests.log 2>&1 || exit 2
timeout -k 10 900 python tools/flag_ab.py --sf0 "acoustic_models.DEC_LATER=0" "acoustic_models.DEC_PAD=0" "" "layers.COOP_BF16=0,acoustic_models.DEC_PAD=0,acoustic_models.DEC_LATER=0" > gpurun_out/cb_ab.txt 2>&1 || exit 3
