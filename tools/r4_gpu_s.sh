set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u tools/tf_leg.py > gpurun_out/r4_tf_leg.json 2> gpurun_out/r4_tf_leg.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tfprof3 -o tf -- python3 tools/tf_leg.py > gpurun_out/r4_tf_prof3.log 2>&1 || exit 2
