# Full round check on the GPU box: all -m gpu tests, smoke, the default bench line, and the
# gate-GEMM PMC traffic passes.   gpurun -- 'bash tools/round_run.sh'
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/rr_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rr_smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/rr_bench.json 2> gpurun_out/rr_bench.err || exit 1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o pmc -- python3 tools/gate_gemm_pmc.py > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o pmc -- python3 tools/gate_gemm_pmc.py > gpurun_out/pmc_write.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_fetch/pmc_counter_collection.csv gpurun_out/pmc_write/pmc_counter_collection.csv gpurun_out/gate_gemm_pmc.json conv_gemm_b16_big_kernel
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gate -o gate -- python3 tools/gate_gemm_pmc.py > gpurun_out/prof_gate.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_train -o train -- python3 bench.py --no-synth --no-cpu-baseline --no-config2 --steps 8 > gpurun_out/prof_train.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_step_fetch -o pmc -- python3 tools/step_pmc.py > gpurun_out/pmc_step_fetch.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_step_write -o pmc -- python3 tools/step_pmc.py > gpurun_out/pmc_step_write.log 2>&1 || exit 1
python3 tools/step_pmc_sum.py gpurun_out/pmc_step_fetch/pmc_counter_collection.csv gpurun_out/pmc_step_write/pmc_counter_collection.csv gpurun_out/step_pmc.json
