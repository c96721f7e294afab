#!/bin/bash
# round-6 GPU check: main-line A/B of the p8 stagger and SQ counters of the K loop
set -o pipefail
mkdir -p gpurun_out/pmc
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for m in 2 6; do
  timeout -s KILL 90 rocprofv3 --pmc $SQ -d gpurun_out/pmc/sq_m$m -o sq --output-format csv -- python3 tools/p8_pmc.py dgrad $m > gpurun_out/pmc/sq_m$m.log 2>&1 || exit 1
done
timeout -k 10 500 python -u tools/flag_ab.py "ensvs_set_p8=2" "ensvs_set_p8=6" > gpurun_out/ab_stag.txt 2>&1
rc=$?; tail -5 gpurun_out/ab_stag.txt; exit $rc
