set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 -u tools/wgrad_bench.py > gpurun_out/r4_wgrad_bench_new.txt 2>&1 || exit 1
ENSVS_LIB=$GRAFT_REPO_ROOT/ab/base/ensemble_svs_with_interactions_amd/libensvs.so timeout -k 10 200 python3 -u tools/wgrad_bench.py > gpurun_out/r4_wgrad_bench_base.txt 2>&1 || exit 2
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="TCC_HIT_sum TCC_MISS_sum SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
for c in gate_bwd dil_dgrad wgrad_dil; do
  i=0
  for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $P --output-format csv -d gpurun_out/pmc_${c}_$i -o p -- python3 tools/gemm_pmc.py $c > gpurun_out/pmc_${c}_$i.log 2>&1 || exit 3
  done
  python3 tools/pmc_table.py gpurun_out/pmc_${c}_1 gpurun_out/pmc_${c}_2 gpurun_out/pmc_${c}_3 gpurun_out/pmc_${c}_4 > gpurun_out/r4_pmc_$c.txt
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cases -o cases -- python3 tools/gemm_pmc.py wgrad_dil > gpurun_out/prof_cases.log 2>&1
timeout -k 10 200 python3 -u tools/branch_times.py > gpurun_out/r4_branch_times.txt 2>&1
timeout -k 10 200 python3 -u tools/lstm_phase_probe.py > gpurun_out/r4_lstm_phase.txt 2>&1
