"""Tier-2 Transformer encoder training leg alone (bench.transformer_train), for profiling:
    rocprofv3 --kernel-trace --stats -d gpurun_out/tf -- python3 tools/tf_leg.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = sys.argv[:1]
import bench  # noqa: E402

bench._imports()
import torch  # noqa: E402

print(json.dumps(bench.transformer_train(torch.device("cuda", 0), steps=5, warm=2)))
