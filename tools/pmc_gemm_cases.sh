#!/bin/bash
# PMC passes over the step's GEMM shapes (tools/gemm_pmc.py): an SQ pass, an SQ + TCC pass and
# the HBM FETCH_SIZE / WRITE_SIZE passes per case (CASES="..." to pick); summaries by
# tools/pmc_table.py.   gpurun -- 'bash tools/pmc_gemm_cases.sh'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
for c in ${CASES:-gate_fwd gate_bwd dil_dgrad wgrad_cond wgrad_dil}; do
  timeout -k 10 60 python3 tools/gemm_pmc.py $c > gpurun_out/pmc_$c.txt 2>&1 || exit 1
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_${c}_$i -o p -- python3 tools/gemm_pmc.py $c > gpurun_out/pmc_${c}_$i.log 2>&1 || exit 1
  done
done
