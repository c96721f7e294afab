#!/bin/bash
# Interleaved A/B of source trees over the bench's training legs (main line, 60 x 512,
# ragged, config 2, interaction loss, on-disk data path): tools/legs_ab.sh DIR1 DIR2 ...
cd "$(dirname "$0")/.."
root=$(pwd)
for rep in 1 2; do
  for d in "$@"; do
    (cd "$root/$d" && ENSVS_LIB= timeout -k 10 400 python -u bench.py --no-cpu-baseline \
      --no-synth --no-sf0 --no-census --no-transformer 2>/dev/null) | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
s = d['shapes']
print('tree=[$d] main %.3f p60 %.3f ragged %.3f c2 %.3f il %.3f real %.3f M' % (d['ms_per_step'],
      s['p60x512']['ms_per_step'], s['ragged_p30x1024']['ms_per_step'], d['config2']['ms_per_step'],
      d['interaction_loss']['ms_per_step'], d['real_data']['value'] / 1e6))" || exit 1
  done
done
