# BLAS cast on: GPU tests, SeparateF0 A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/cb_tests.log 2>&1 || exit 1
timeout -k 10 900 python -u tools/flag_ab.py --sf0 "BLAS:cast=0" "" > gpurun_out/cb_ab.txt 2>&1 || exit 3
