# Round-4 closing run: every -m gpu test, smoke, the default bench line, the main step's
# kernel trace and its HBM counters (separate --pmc passes).   gpurun -- 'bash tools/r4_final.sh'
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
if [ "$1" != "--bench-only" ]; then
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r4f_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4f_smoke.log 2>&1 || exit 2
fi
b0=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r4f_bench.json 2> gpurun_out/r4f_bench.err || exit 3
echo "bench wall $(( $(date +%s) - b0 )) s" >> gpurun_out/r4f_bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4f_prof_train -o train -- python3 bench.py --no-synth --no-cpu-baseline --no-config2 --no-sf0 --no-shapes --no-real-data --no-transformer --no-census --steps 8 > gpurun_out/r4f_prof_train.log 2>&1 || exit 4
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4f_pmc_fetch -o pmc -- python3 tools/step_pmc.py > gpurun_out/r4f_pmc_fetch.log 2>&1 || exit 5
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4f_pmc_write -o pmc -- python3 tools/step_pmc.py > gpurun_out/r4f_pmc_write.log 2>&1 || exit 6
python3 tools/step_pmc_sum.py gpurun_out/r4f_pmc_fetch/pmc_counter_collection.csv gpurun_out/r4f_pmc_write/pmc_counter_collection.csv gpurun_out/r4f_step_pmc.json
