#!/bin/bash
# round-6 GPU check: PMC passes over the 128 x 256 kernel's launches (tools/pmc_gemm_cases.sh)
set -o pipefail
mkdir -p gpurun_out
( while sleep 45; do date >> gpurun_out/hb.txt; done ) &
HB=$!
trap "kill $HB" EXIT
CASES="skip_sum cond_dgrad res_fwd" bash tools/pmc_gemm_cases.sh || exit 1
for c in skip_sum cond_dgrad res_fwd; do
  echo "### $c"; cat gpurun_out/pmc_$c.txt | grep -v amdgpu
  python3 tools/pmc_table.py gpurun_out/pmc_${c}_1 gpurun_out/pmc_${c}_2 gpurun_out/pmc_${c}_3 gpurun_out/pmc_${c}_4 --match conv_gemm
done > gpurun_out/pmc_p8h.txt 2>&1
cat gpurun_out/pmc_p8h.txt
