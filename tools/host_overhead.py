"""Host-issue vs GPU time of the bench train step: if the host spends as long issuing a
step as the GPU spends executing it, the step is launch-bound (candidate for graphs)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step  # noqa: E402

dev = torch.device("cuda", 0)
engine.set_gemm_precision("bf16")
torch.manual_seed(0)
model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
b = data.synthetic_batch(30, 1024, 1000)
g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
args = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"), b["lengths"].tolist())
for _ in range(3):
    train_step(model, opt, *args)
torch.cuda.synchronize()
for conc in (True, False):
    engine.set_concurrency(conc)
    train_step(model, opt, *args)
    torch.cuda.synchronize()
    host = []
    t0 = time.time()
    for _ in range(5):
        h0 = time.time()
        train_step(model, opt, *args)
        host.append(time.time() - h0)
    torch.cuda.synchronize()
    wall = (time.time() - t0) / 5
    print(f"concurrency={conc}: wall {wall*1e3:.2f} ms/step, host issue {sum(host)/5*1e3:.2f} ms/step "
          f"(min {min(host)*1e3:.2f})", flush=True)
