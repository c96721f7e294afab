set -o pipefail
cd $GRAFT_REPO_ROOT
echo "env GPU_MAX_HW_QUEUES=[${GPU_MAX_HW_QUEUES:-unset}]" > gpurun_out/r4_hwq.txt
for rep in 1 2; do
for v in base4 base8 defer4 defer8; do
  case $v in base*) d=ab/base;; *) d=.;; esac
  q=${v: -1}
  (cd $d && GPU_MAX_HW_QUEUES=$q timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data --no-transformer 2>/dev/null) | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'], 3), 'ms')" >> gpurun_out/r4_hwq.txt || exit 1
done
done
