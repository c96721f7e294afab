set -o pipefail
export ENSVS_BENCH_BACKEND=gloo
timeout -k 10 600 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_coop_fault_gpu.py tests/test_ardec_gpu.py tests/test_lstm_gpu.py tests/test_ddp_gpu.py > gpurun_out/r4_coop_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 3 --eager > gpurun_out/r4_gloo2_eager.json 2> gpurun_out/r4_gloo2_eager.err || exit 2
timeout -k 10 300 python -u bench.py --gpus 2 --steps 5 --warmup 2 --overlap-ddp > gpurun_out/r4_gloo2_overlap2.json 2> gpurun_out/r4_gloo2_overlap2.err || exit 3
