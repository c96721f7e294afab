set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -u -c "
import sys, json
sys.argv = ['bench.py']
import bench
bench._imports()
import torch
dev = torch.device('cuda', 0)
r = bench.transformer_train(dev)
r['cpu_baseline'] = bench.transformer_cpu_baseline()
print(json.dumps(r))
" > gpurun_out/r4_transformer_leg.json 2> gpurun_out/r4_transformer_leg.err || exit 1
timeout -k 10 300 python3 -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_transformer.py > gpurun_out/r4_l_tests.log 2>&1 || exit 2
