# generic plain-GEMM routing to hipBLASLt: parity tests and A/Bs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_blas_gpu.py tests/test_separate_f0.py tests/test_multitrack_gpu.py tests/test_diffnet_gpu.py tests/test_gemm_bf16a_gpu.py tests/test_bench_size_gpu.py -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/flag_ab.py "BLAS:generic=0" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
timeout -k 10 900 python -u tools/flag_ab.py --sf0 "BLAS:generic=0" "" >> gpurun_out/cb_ab.txt 2>&1 || exit 4
