# Every plain bf16 GEMM (>= 2^24 MACs) on hipBLASLt: GPU tests, then the step A/B (3 rounds)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/flag_ab.py "BLAS:generic=0" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
timeout -k 10 600 python -u tools/flag_ab.py "BLAS:generic=0" "" > gpurun_out/cb_ab2.txt 2>&1 || exit 4
