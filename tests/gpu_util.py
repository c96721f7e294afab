"""Helpers for GPU parity tests: build this package's modules with seeded params."""
import torch

from ensemble_svs_with_interactions_amd import configs, engine
from golden_util import params_from_shapes


def build(cfg, shapes, prefix="", device="cuda"):
    mod = configs.instantiate(cfg)
    P = params_from_shapes(shapes)
    sd = {k[len(prefix):]: v for k, v in P.items() if k.startswith(prefix)}
    missing, unexpected = mod.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith("num_batches_tracked") or k.rsplit(".", 1)[-1] in
               engine_schedule_names() for k in missing), missing
    return mod.to(device)


def engine_schedule_names():
    from oracle.weights import SCHEDULE_BUFFERS
    return SCHEDULE_BUFFERS


def grads_by_name(mod, prefix=""):
    return {prefix + k: p.grad for k, p in mod.named_parameters() if p.grad is not None}
