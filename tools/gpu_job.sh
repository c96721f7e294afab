#!/bin/bash
# One parametrised GPU-box job (replaces round 4's one-off tools/r4_gpu_*.sh):
#   gpurun -- 'bash tools/gpu_job.sh TAG STEP [STEP ...]'
# STEP is one of
#   tests:<pytest args>     -m gpu tests (-x -v, thread timeout) -> gpurun_out/TAG_tests<i>.log
#   bench:<bench.py args>   one bench line                        -> gpurun_out/TAG_bench<i>.json
#   prof:<bench.py args>    rocprofv3 --kernel-trace --stats of a bench run -> gpurun_out/TAG_prof<i>/
#   py:<script + args>      any python script                     -> gpurun_out/TAG_py<i>.txt
#   ab:<dir> <dir> ...      interleaved whole-tree A/B (tools/tree_ab.sh) -> gpurun_out/TAG_ab<i>.txt
#   smoke                   __graft_entry__.smoke()               -> gpurun_out/TAG_smoke.log
#   gloo2:<bench.py args>   2 ranks on the one GPU over gloo (bench.py --gpus 2, the N > 1 line
#                           rehearsed)                              -> gpurun_out/TAG_gloo2_<i>.json
# Inside a STEP, commas stand for spaces (bench:--no-synth,--no-shapes), since the job's
# arguments are split on spaces.
# Every step has its own time limit; the job stops at the first failing step.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &  # a long quiet step is not a hang
HB=$!
trap "kill $HB" EXIT
tag=$1; shift
i=0
for step in "$@"; do
  i=$((i + 1)); kind=${step%%:*}; args=${step#*:}; args=${args//,/ }
  case $kind in
    tests) timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $args \
             > gpurun_out/${tag}_tests$i.log 2>&1 ;;
    bench) timeout -k 10 900 python -u bench.py $args > gpurun_out/${tag}_bench$i.json \
             2> gpurun_out/${tag}_bench$i.err ;;
    prof)  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
             -d gpurun_out/${tag}_prof$i -o prof -- python3 bench.py $args > gpurun_out/${tag}_prof$i.log 2>&1 ;;
    py)    timeout -k 10 900 python -u $args > gpurun_out/${tag}_py$i.txt 2>&1 ;;
    ab)    timeout -k 10 1100 bash tools/tree_ab.sh $args > gpurun_out/${tag}_ab$i.txt 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
             > gpurun_out/${tag}_smoke.log 2>&1 ;;
    gloo2) ENSVS_BENCH_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 \
             --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 $args \
             > gpurun_out/${tag}_gloo2_$i.json 2> gpurun_out/${tag}_gloo2_$i.err ;;
    *) echo "unknown step $step"; exit 8 ;;
  esac
  rc=$?
  echo "step $i ($kind) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
