set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gemm_gpu.py -k "pack or embed or phoneme" > gpurun_out/r4_ay_tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -u tools/census.py 400 > gpurun_out/r4_census_pack.txt 2>&1 || exit 2
timeout -k 10 700 bash tools/tree_ab.sh ab/base . > gpurun_out/r4_ay_ab.txt 2>&1 || exit 3
