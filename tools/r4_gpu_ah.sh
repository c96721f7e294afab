set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in base same aux; do
  case $v in base) d=ab/base; e="";; same) d=.; e="ENSVS_DEFER_SAME=1";; *) d=.; e="";; esac
  (cd $d && env $e timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data --no-transformer 2>/dev/null) | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'], 3), 'ms')" >> gpurun_out/r4_defer_same.txt || exit 1
done
done
