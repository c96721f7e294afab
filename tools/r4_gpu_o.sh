set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_attention_ops_gpu.py > gpurun_out/r4_o_ops.log 2>&1
echo "ops rc=$?" >> gpurun_out/r4_o_ops.log
cd ab/base && timeout -k 10 300 python3 -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_transformer.py -k large_t > ../../gpurun_out/r4_o_base.log 2>&1
echo "base rc=$?" >> ../../gpurun_out/r4_o_base.log
