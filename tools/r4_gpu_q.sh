set -o pipefail
cd $GRAFT_REPO_ROOT
echo "== full lib" > gpurun_out/r4_q.txt
timeout -k 10 200 python3 -u tools/tf_large_t_err.py 2>&1 | grep -v amdgpu.ids | head -8 >> gpurun_out/r4_q.txt || exit 1
echo "== full lib, HIP_LAUNCH_BLOCKING=1" >> gpurun_out/r4_q.txt
HIP_LAUNCH_BLOCKING=1 timeout -k 10 200 python3 -u tools/tf_large_t_err.py 2>&1 | grep -v amdgpu.ids | head -8 >> gpurun_out/r4_q.txt || exit 2
