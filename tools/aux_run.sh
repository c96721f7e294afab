set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_multitrack_gpu.py tests/test_dropin_gpu.py tests/test_singletrack_gpu.py -m gpu > gpurun_out/aux_tests.log 2>&1
for q in 4 8; do for a in 0 1; do
  GPU_MAX_HW_QUEUES=$q ENSVS_AUX_WGRAD=$a timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-synth --no-cpu-baseline --no-config2 > gpurun_out/aux_q${q}_a${a}.json 2>gpurun_out/aux_q${q}_a${a}.err
done; done
