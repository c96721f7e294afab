set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/census.py 400 train mgc > gpurun_out/r4_census_mgc.txt 2>&1 || exit 2
