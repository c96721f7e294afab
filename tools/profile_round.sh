# Round profile artifacts (run on the GPU box from the repo root):
#   kernel stats of the default bench command, and the gate-GEMM HBM traffic (FETCH_SIZE /
#   WRITE_SIZE in separate passes, MI355X_MICROARCH.md HBM section) -> tools/gate_gemm_pmc.json
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python3 tools/gate_gemm_pmc.py > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o pmc -- python3 tools/gate_gemm_pmc.py > gpurun_out/pmc_write.log 2>&1
python3 tools/pmc_summary.py gpurun_out/pmc_fetch/pmc_counter_collection.csv gpurun_out/pmc_write/pmc_counter_collection.csv gpurun_out/gate_gemm_pmc.json conv_gemm_b16_big_kernel
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gate -o gate -- python3 tools/gate_gemm_pmc.py > gpurun_out/prof_gate.log 2>&1
