set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_transformer.py > gpurun_out/r4_n_tests.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tfprof2 -o tf -- python3 tools/tf_leg.py > gpurun_out/r4_tf_prof2.log 2>&1 || exit 2
