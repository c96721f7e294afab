set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tfprof -o tf -- python3 tools/tf_leg.py > gpurun_out/r4_tf_prof.log 2>&1 || exit 1
