# PMC passes over tools/gemm_one.py (dev tool): bash tools/pmc_gemm.sh [M N K taps]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT --output-format csv -d gpurun_out/pmc1 -o p -- python3 tools/gemm_one.py "$@" > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pmc2 -o p -- python3 tools/gemm_one.py "$@" > gpurun_out/pmc2.log 2>&1
