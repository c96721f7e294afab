set -o pipefail
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for d in ab/base .; do
  (cd $d && timeout -k 10 240 python -u bench.py --eager --steps 10 --warmup 3 --no-cpu-baseline --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data --no-transformer 2>/dev/null) | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('eager tree=[$d]', round(d['ms_per_step'], 3), 'ms')" >> gpurun_out/r4_defer_eager.txt || exit 1
done
done
