set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for v in base aux side0 side2; do
  if [ $v = base ]; then d=ab/base; e=""; else d=.; e=""; fi
  if [ $v = side0 ]; then e="ENSVS_AUX_SIDE=0"; fi
  if [ $v = side2 ]; then e="ENSVS_AUX_SIDE=2"; fi
  (cd $d && env $e timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data --no-transformer 2>/dev/null) | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'], 3), 'ms')" >> gpurun_out/r4_defer_var.txt || exit 1
done
done
