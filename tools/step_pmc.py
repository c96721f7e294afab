"""HBM traffic of one bench training step (30 pairs x 1024 frames, bf16), for rocprofv3 --pmc
passes: 3 eager warm-up steps, then K = 4 eager steps bracketed by marker kernels
(torch.cuda._sleep), so tools/step_pmc_sum.py can sum FETCH_SIZE / WRITE_SIZE over the
dispatches of the measured steps only.  Run each counter in its own pass:
  rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT -o pmc -- python3 tools/step_pmc.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step  # noqa: E402

K = 4
engine.set_gemm_precision("bf16")
dev = torch.device("cuda", 0)
torch.manual_seed(20250321)
model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
b = data.synthetic_batch(30, 1024, 1000)
g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
args = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"), b["lengths"].tolist())
for _ in range(3):
    train_step(model, opt, *args)
torch.cuda.synchronize()
torch.cuda._sleep(1000)
for _ in range(K):
    train_step(model, opt, *args)
torch.cuda._sleep(1000)
torch.cuda.synchronize()
print(f"steps {K}", flush=True)
