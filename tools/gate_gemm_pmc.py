"""Launch only the dominant kernel of the bench (mgc DiffNet block gate GEMM, bf16,
M = 30 x 1024 frames, N = 512, K = 1024) 23 times, for rocprofv3 --pmc passes
(FETCH_SIZE / WRITE_SIZE per dispatch).  Dev tool:
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o pmc -- python3 tools/gate_gemm_pmc.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ensemble_svs_with_interactions_amd import configs, engine  # noqa: E402

engine.set_gemm_precision("bf16")
dev = torch.device("cuda", 0)
torch.manual_seed(20250321)
model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
sec, _, flops = bench.gate_gemm_timing(model, 30, 1024, dev, iters=20)
print(f"gate GEMM {sec * 1e6:.1f} us/launch, {flops / sec / 1e12:.1f} TFLOP/s", flush=True)
