"""Per-parameter gradient error of test_transformer.py::test_gpu_large_t_against_oracle's case
(fp32 mode): max |got - ref| / max(max |ref|, floor), printed per parameter (dev tool)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from golden_util import params_from_shapes  # noqa: E402
from oracle import ensvs_oracle as O  # noqa: E402
from ensemble_svs_with_interactions_amd import engine  # noqa: E402
from ensemble_svs_with_interactions_amd.transformer import TransformerEncoder  # noqa: E402

engine.set_gemm_precision("fp32")
cfg = dict(in_dim=86, out_dim=60, hidden_dim=192, attention_dim=768, num_heads=2,
           num_layers=2, kernel_size=3, dropout=0.0)
torch.manual_seed(3)
mod = TransformerEncoder(**cfg).cuda()
P = params_from_shapes({k: list(v.shape) for k, v in mod.state_dict().items()})
mod.load_state_dict(P)
B, T = 3, 1000
g = torch.Generator().manual_seed(9)
x = torch.randn(B, T, cfg["in_dim"], generator=g)
R = torch.randn(B, T, cfg["out_dim"], generator=g)
lengths = [1000, 731, 402]
grads = []
for rep in range(3):
    mod.zero_grad(set_to_none=True)
    out = mod(x.cuda(), lengths)
    (out * R.cuda()).sum().backward()
    torch.cuda.synchronize()
    grads.append({k: p.grad.detach().clone() for k, p in mod.named_parameters()})
for rep in (1, 2):
    print("run-to-run max grad diff", rep,
          max((grads[rep][k] - grads[0][k]).abs().max().item() for k in grads[0]))
P64 = {k: v.double().requires_grad_() for k, v in P.items()}
ref = O.transformer_encoder(P64, cfg, x.double(), lengths)
print("out rel", ((out.detach().cpu().double() - ref.detach()).norm() / ref.detach().norm()).item())
(ref * R.double()).sum().backward()
fl = 1e-2 * max(float(np.abs(P64[k].grad.numpy()).max()) for k in P64)
for k, p in mod.named_parameters():
    r = P64[k].grad
    e = (p.grad.cpu().double() - r).abs().max().item() / max(r.abs().max().item(), fl)
    print(f"{k:45s} {e:.2e}")
