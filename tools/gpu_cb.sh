#!/bin/bash
# round-6 GPU check: cooperative LSTM backward publishing from wave 0 -- coop tests, SeparateF0 A/B
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu -rf -x tests/test_lstm_gpu.py tests/test_separate_f0.py > gpurun_out/coop_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/coop_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
SF0=1 timeout -k 10 1000 bash tools/tree_ab.sh ab/head . > gpurun_out/ab_coop_pub.txt 2>&1
rc=$?; cat gpurun_out/ab_coop_pub.txt; exit $rc
