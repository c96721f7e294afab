"""Where the training step's device copies come from (dev tool): counts torch-level copies
(Tensor.copy_ / .to / .cuda / torch.tensor(..., device) / torch.as_tensor) issued during one
eager step, by call site.   python tools/copy_census.py
"""
import collections
import os
import sys
import traceback

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step  # noqa: E402

SITES = collections.Counter()


def _site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "ensemble_svs_with_interactions_amd" in fr.filename:
            return f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.line}"
    return "?"


def wrap(obj, name):
    orig = getattr(obj, name)

    def f(*a, **k):
        SITES[(name, _site())] += 1
        return orig(*a, **k)
    setattr(obj, name, f)
    return orig


def main():
    dev = torch.device("cuda")
    engine.set_gemm_precision("bf16")
    torch.manual_seed(0)
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    opt = FusedAdam(model)
    b = data.synthetic_batch(30, 1024, 3)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    args = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
            b["lengths"].tolist())
    train_step(model, opt, *args)
    torch.cuda.synchronize()
    for name in ("copy_", "to", "cuda", "clone"):
        wrap(torch.Tensor, name)
    for name in ("tensor", "as_tensor", "zeros", "empty", "full", "ones", "arange"):
        wrap(torch, name)
    train_step(model, opt, *args)
    torch.cuda.synchronize()
    for (name, site), n in SITES.most_common(40):
        print(f"{n:5d} {name:10s} {site}")


if __name__ == "__main__":
    main()
