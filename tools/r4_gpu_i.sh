set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_lstm_gpu.py tests/test_bf16_copies_gpu.py tests/test_encoders_gpu.py tests/test_multitrack_gpu.py tests/test_separate_f0.py > gpurun_out/r4_i_tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/lstm_mfma_bench.py > gpurun_out/r4_lstm_mfma_bench_i.txt 2>&1 || exit 2
timeout -k 10 600 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_lstm_ab_i.txt 2>&1 || exit 3
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_synth_fetch -o pmc -- python3 tools/synth_pmc.py > gpurun_out/pmc_synth_fetch.log 2>&1 || exit 4
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_synth_write -o pmc -- python3 tools/synth_pmc.py > gpurun_out/pmc_synth_write.log 2>&1 || exit 5
python3 tools/step_pmc_sum.py gpurun_out/pmc_synth_fetch/pmc_counter_collection.csv gpurun_out/pmc_synth_write/pmc_counter_collection.csv gpurun_out/r4_synth_pmc.json 1 > /dev/null
