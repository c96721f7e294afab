# SeparateF0 census (serial, per launch) and kernel stats of the bench's SF0 leg
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u tools/census.py 60 sf0 > gpurun_out/cb_census_sf0.txt 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cb_sf0prof -o sf0 -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-synth --no-census --no-config2 --no-shapes --no-real-data --no-transformer > gpurun_out/cb_sf0prof.log 2>&1 || exit 2
