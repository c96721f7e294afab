"""SeparateF0 full-size gradient diagnostic (dev tool): HIP grads vs the CPU oracle's
autograd grads on the sf0_forward_full fixture, per-parameter relative L2, worst first."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from oracle import ensvs_oracle as O  # noqa: E402
from golden_util import load_case, params_from_shapes, rel_l2  # noqa: E402
from ensemble_svs_with_interactions_amd import configs, engine  # noqa: E402
from gpu_util import build  # noqa: E402

engine.set_gemm_precision(sys.argv[1] if len(sys.argv) > 1 else "fp32")
a, meta = load_case("sf0_forward_full")
cfg = configs.multitrack_separate_f0(num_speakers=4)
model = build(cfg, meta["shapes"])
for m in (model.mgc_model, model.vuv_model, model.bap_model, model.encoder):
    m.lstm.dropout = 0.0
model.train()
d = lambda k: torch.from_numpy(np.ascontiguousarray(a[k])).cuda()  # noqa: E731
t = lambda k: torch.from_numpy(np.ascontiguousarray(a[k]))  # noqa: E731
model._replay_draws = dict(lf0_main=d("draw::lf0_main").view(-1), lf0_sub=d("draw::lf0_sub").view(-1))
(om, rm), (os_, rs) = model(d("x_main"), d("x_sub"), (d("spk_main"), d("spk_sub")),
                            lengths=a["lengths"].tolist(), ys=[d("y_main"), d("y_sub")])
sum((x * d(f"R{i}")).sum() for i, x in enumerate((om, rm, os_, rs))).backward()
P = params_from_shapes(meta["shapes"], requires_grad=True)
(o1, r1), (o2, r2) = O.separate_f0_forward(
    P, cfg, t("x_main"), t("x_sub"), (t("spk_main").long(), t("spk_sub").long()),
    a["lengths"].tolist(), [t("y_main"), t("y_sub")],
    dict(lf0_main=t("draw::lf0_main"), lf0_sub=t("draw::lf0_sub")), training=True, bn_updates={})
sum((x * t(f"R{i}")).sum() for i, x in enumerate((o1, r1, o2, r2))).backward()
for n, (x, y) in enumerate(((om, o1), (rm, r1), (os_, o2), (rs, r2))):
    print("out", n, rel_l2(x.detach().cpu(), y.detach()))
res = []
for k, p in model.named_parameters():
    g = p.grad.cpu() if p.grad is not None else torch.zeros(p.shape)
    res.append((rel_l2(g, P[k].grad), k))
for r, k in sorted(res, reverse=True)[:25]:
    print(f"{r:.3e} {k}")
