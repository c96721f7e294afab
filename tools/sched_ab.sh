#!/bin/bash
# A/B of step-schedule knobs on the bench (dev): library (ENSVS_LIB), hardware queues,
# auxiliary weight-gradient streams, branch priority.  One config per line of $1:
# "<name> VAR=value ...".   gpurun -- 'bash tools/sched_ab.sh tools/ab_cfgs.txt'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
rm -f gpurun_out/ab.txt
while read -r n rest; do
  [ -z "$n" ] && continue
  env $rest timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-synth --no-cpu-baseline --no-config2 $BENCH_ARGS > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); print('$n', round(d['ms_per_step'],2))" >> gpurun_out/ab.txt
done < "$1"
