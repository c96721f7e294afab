#!/bin/bash
# round-6 GPU check: GEMM bitwise tests, the K loop without loads, the real-data leg
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread -m gpu -rf -x tests/test_gemm_p8h_gpu.py > gpurun_out/p8_tests.log 2>&1
rc=$?; grep -E "FAIL|passed|failed|Error" gpurun_out/p8_tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/p8_bench.py > gpurun_out/p8_bench3.txt 2>&1 || exit 6
tail -2 gpurun_out/p8_bench3.txt
timeout -k 10 700 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-synth --no-sf0 \
  --no-census --no-config2 --no-shapes --no-transformer > gpurun_out/realdata.json 2> gpurun_out/realdata.err
rc=$?; python3 -c "
import json; d=json.loads(open('gpurun_out/realdata.json').read().strip().splitlines()[-1])
r=d.get('real_data', {}); print({k: r.get(k) for k in ('value','s_per_epoch','feeder_wait_s_per_epoch','ratio_to_same_shapes_back_to_back','ratio_to_fixed_shape','eager_value','steps_per_epoch')})
"; exit $rc
