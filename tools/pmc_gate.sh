# PMC passes over tools/gate_probe.py (dev tool; MI355X_MICROARCH.md HBM/rocprofv3 section:
# one counter group per pass).  bash tools/pmc_gate.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="python3 tools/gate_probe.py 5 gate_gf16"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES --output-format csv -d gpurun_out/pg1 -o p -- $P > gpurun_out/pg1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/pg2 -o p -- $P > gpurun_out/pg2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pg3 -o p -- $P > gpurun_out/pg3.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pg4 -o p -- $P > gpurun_out/pg4.log 2>&1
