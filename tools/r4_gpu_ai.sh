set -o pipefail
cd $GRAFT_REPO_ROOT
ENSVS_AUX_SIDE=0 timeout -k 10 300 python3 -u tools/branch_times.py > gpurun_out/r4_side0_bt.txt 2>&1 || exit 1
for rep in 1 2; do
for v in base side0; do
  case $v in base) d=ab/base; e="";; side0) d=.; e="ENSVS_AUX_SIDE=0";; esac
  (cd $d && env $e timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-synth --no-sf0 --no-census --no-config2 --no-shapes --no-real-data --no-transformer 2>/dev/null) | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$v', round(d['ms_per_step'], 3), 'ms')" >> gpurun_out/r4_side0.txt || exit 1
done
done
