set -o pipefail
mkdir -p gpurun_out/r4_errors
ENSVS_RECORD_DIR=gpurun_out/r4_errors timeout -k 10 300 python -u -m pytest -x -v -s --timeout 280 --timeout-method thread tests/test_precision_trajectory_gpu.py > gpurun_out/r4_traj.log 2>&1
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r4_bench_a.json 2> gpurun_out/r4_bench_a.err || exit 2
