#!/bin/bash
# Interleaved whole-step A/B of source trees (each with its own built libensvs.so), e.g. a
# `git archive` of an earlier commit unpacked under ab/: bench train leg (graph replay,
# 30 x 1024, 20 steps), two rounds.  tools/tree_ab.sh DIR1 DIR2 ...  ("." = this tree)
cd "$(dirname "$0")/.."
root=$(pwd)
for rep in 1 2; do
  for d in "$@"; do
    (cd "$root/$d" && ENSVS_LIB= timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data 2>/dev/null) | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('tree=[$d]', round(d['ms_per_step'], 3), 'ms')" || exit 1
  done
done
