#!/bin/bash
# Interleaved A/B of the LSTM routing in the full training step (bench.py train leg only):
# ENSVS_LSTM_BATCH = "" (exact kernels), "64", "64,128".  Prints ms_per_step per run.
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for hs in "" "64" "64,128"; do
    ENSVS_LSTM_BATCH=$hs timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-synth --no-sf0 --no-census --no-config2 > gpurun_out/ab_${rep}_${hs}.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_${rep}_${hs}.json').read().strip().splitlines()[-1]); print('batch=[$hs]', round(d['ms_per_step'],3), 'ms')"
  done
done
