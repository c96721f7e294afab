#!/bin/bash
# Interleaved whole-step A/B of source trees (each with its own built libensvs.so), e.g. a
# `git archive` of an earlier commit unpacked under ab/: bench train leg (graph replay,
# 30 x 1024, 20 steps), two rounds.  tools/tree_ab.sh DIR1 DIR2 ...  ("." = this tree)
# SF0=1: time the recipe-default SeparateF0 leg instead (its ms_per_step).
cd "$(dirname "$0")/.."
root=$(pwd)
if [ -n "$SF0" ]; then legs=""; key=separate_f0; else legs="--no-sf0"; key=""; fi
for rep in 1 2; do
  for d in "$@"; do
    (cd "$root/$d" && ENSVS_LIB= timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 \
      --no-cpu-baseline --no-synth $legs --no-census --no-config2 --no-shapes --no-real-data \
      --no-transformer 2>/dev/null) | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); d=d['$key'] if '$key' else d; print('tree=[$d]', round(d['ms_per_step'], 3), 'ms', '$key')" || exit 1
  done
done
