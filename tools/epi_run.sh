cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_bf16a_gpu.py tests/test_gemm_big_gpu.py tests/test_gemm_gpu.py tests/test_inference_gpu.py tests/test_multitrack_gpu.py tests/test_diffnet_gpu.py -m gpu > gpurun_out/epi_tests.log 2>&1 || exit 1
timeout -k 10 100 python -u tools/small_gemm_probe.py > gpurun_out/epi_sgp.log 2>&1 || exit 1
ENSVS_GATE8=0 timeout -k 10 100 python -u tools/small_gemm_probe.py > gpurun_out/epi_sgp0.log 2>&1 || exit 1
timeout -k 10 100 python -u tools/gate_probe.py 20 gate_gf16 > gpurun_out/epi_gate.log 2>&1 || exit 1
ENSVS_GATE8=0 timeout -k 10 100 python -u tools/gate_probe.py 20 gate_gf16 > gpurun_out/epi_gate0.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/synth_probe.py 1 6 > gpurun_out/epi_synth.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-synth --no-cpu-baseline --no-config2 > gpurun_out/epi_bench.json 2> gpurun_out/epi_bench.err
