"""Capture GraphedTrainStep on the tiny model (dev tool for graph-capture issues)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from ensemble_svs_with_interactions_amd import configs, engine  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep  # noqa: E402
from golden_util import load_case  # noqa: E402
from gpu_util import build  # noqa: E402
from test_multitrack_gpu import _batch  # noqa: E402

engine.set_gemm_precision("bf16")
a, meta = load_case("train_step_tiny")
xm, xs, ym, s0, s1, lens = _batch(a)
model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True), meta["shapes"])
opt = FusedAdam(model, lr=meta["lr"])
print("aux", engine._STATE["aux"], flush=True)
gs = GraphedTrainStep(model, opt, xm, xs, ym, s0, s1, lens, warmup=1)
loss, norm = gs.step()
print("ok", loss.item(), flush=True)
