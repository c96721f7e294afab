# Round check: every -m gpu test, smoke, the default bench line (each under its own limit)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/fin_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.log 2>&1 || exit 2
timeout -k 10 600 python -u bench.py > gpurun_out/fin_bench.json 2> gpurun_out/fin_bench.err || exit 3
