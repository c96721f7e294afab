set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py tests/test_gemm_bf16a_gpu.py tests/test_bf16_copies_gpu.py > gpurun_out/r4_c_tests.log 2>&1 || exit 1
timeout -k 10 600 bash tools/tree_ab.sh ab/base . ab/norond > gpurun_out/r4_wgrad_ab.txt 2>&1 || exit 2
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_step_fetch -o pmc -- python3 tools/step_pmc.py > gpurun_out/pmc_step_fetch.log 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_step_write -o pmc -- python3 tools/step_pmc.py > gpurun_out/pmc_step_write.log 2>&1 || exit 4
python3 tools/step_pmc_sum.py gpurun_out/pmc_step_fetch/pmc_counter_collection.csv gpurun_out/pmc_step_write/pmc_counter_collection.csv gpurun_out/r4_step_pmc_map.json
