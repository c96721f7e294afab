#!/bin/bash
# Interleaved whole-step A/B of library builds (ENSVS_LIB; "" = the in-tree build): bench
# train leg (graph replay, 30 x 1024, 20 steps), two rounds.  tools/lib_ab.sh LIB1 LIB2 ...
cd "$(dirname "$0")/.."
for rep in 1 2; do
  for lib in "" "$@"; do
    ENSVS_LIB=$lib timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline \
      --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('lib=[$lib]', round(d['ms_per_step'], 3), 'ms')" || exit 1
  done
done
