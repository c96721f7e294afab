"""BASELINE.md §3 check (build container only; the reference never travels): the CPU
restatement (oracle, as bench.py's cpu_baseline runs it) must train within +-20 % of the
reference's own train_step on the same host, threads, shapes and draws.

  PYTHONDONTWRITEBYTECODE=1 python tools/cpu_baseline_check.py [--pairs 10] [--frames 1024]

Both sides: full-size multi-track diffusion model, fp32, median of 5 steps after 2 warm-up
steps, torch.set_num_threads(8).  Prints one JSON line.
"""
import argparse
import json
import logging
import os
import platform
import subprocess
import sys
import time
import types

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)

import gen_goldens as G  # noqa: E402  (stub loader + reference import + draw injection)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from ensemble_svs_with_interactions_amd import configs, data  # noqa: E402
from oracle import ensvs_oracle as O  # noqa: E402
from oracle.weights import seeded_state_dict  # noqa: E402


def draws_for(P, T, rng):
    return dict(lf0_main=(torch.rand(P, T // 4, 1, generator=rng) < 0.5).float() * 2,
                lf0_sub=(torch.rand(P, T // 4, 1, generator=rng) < 0.5).float() * 2,
                mgc_t=torch.randint(0, 100, (P,), generator=rng),
                mgc_noise=torch.randn(P, 1, 60, T, generator=rng),
                bap_t=torch.randint(0, 100, (P,), generator=rng),
                bap_noise=torch.randn(P, 1, 5, T, generator=rng))


def time_reference(P, T, steps):
    cfg = configs.multitrack_diffusion(num_speakers=4)
    model, _ = G.build_ref(cfg)
    model.vuv_model.lstm.dropout = 0.0
    b = data.synthetic_batch(P, T, 7)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, betas=(0.9, 0.999), weight_decay=0.0)
    mc = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5])
    oc = types.SimpleNamespace(clip_norm=1.0)
    log = logging.getLogger("cpu_check")
    rng = torch.Generator().manual_seed(3)
    ts = []
    for _ in range(steps):
        d = {k: v.numpy() for k, v in draws_for(P, T, rng).items()}
        t0 = time.time()
        with G.queue_draws(d, T):
            G.ref_train_step(log, model, mc, oc, opt, None, True,
                             (G.T_(b["x_main"]), G.T_(b["x_sub"])),
                             [G.T_(b["y_main"]), G.T_(b["y_sub"])],
                             (G.T_(b["spk_main"]).int(), G.T_(b["spk_sub"]).int()),
                             (G.T_(b["lengths"]), G.T_(b["lengths"])), None, None,
                             feats_criterion="l1", pitch_reg_weight=0.0, logf0_diff_weight=0.0,
                             mgc_diff_weight=0.0)
        ts.append(time.time() - t0)
    return ts


def time_oracle(P, T, steps):
    """The same loop as bench.py's cpu_baseline (oracle, fast=True)."""
    cfg = configs.multitrack_diffusion(num_speakers=4)
    model = configs.instantiate(cfg)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    del model
    Pm = {k: torch.from_numpy(v) for k, v in seeded_state_dict(shapes, 1).items()}
    for pre in ("mgc_model.", "bap_model."):
        for k, v in O.diffusion_schedule().items():
            Pm[pre + k] = v
    trainable = [k for k in Pm if "running" not in k and k.rsplit(".", 1)[-1] not in
                 O.diffusion_schedule()]
    b = data.synthetic_batch(P, T, 7)
    x = (torch.from_numpy(b["x_main"]), torch.from_numpy(b["x_sub"]))
    y = (torch.from_numpy(b["y_main"]), torch.from_numpy(b["y_sub"]))
    spk = (torch.from_numpy(b["spk_main"]), torch.from_numpy(b["spk_sub"]))
    rng = torch.Generator().manual_seed(3)
    state, ts = {}, []
    for s in range(steps):
        for k in trainable:
            Pm[k] = Pm[k].detach().requires_grad_()
        d = draws_for(P, T, rng)
        t0 = time.time()
        preds, _ = O.model_forward(Pm, cfg, x[0], x[1], spk, b["lengths"], y, d,
                                   bn_updates={}, fast=True)
        loss = O.masked_l1_loss(preds, y[0], b["lengths"], cfg["stream_sizes"])
        loss.backward()
        grads = {k: Pm[k].grad for k in trainable}
        params = {k: Pm[k].detach() for k in trainable}
        O.clip_and_adam(params, grads, state, step=s + 1)
        Pm.update(params)
        ts.append(time.time() - t0)
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=10)
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--threads", type=int, default=8)
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    P, T = args.pairs, args.frames
    out = {}
    for name, fn in (("reference", time_reference), ("oracle", time_oracle)):
        ts = fn(P, T, 7)
        med = float(np.median(ts[2:]))
        out[name] = dict(frames_per_s=P * T / med, step_s=med, steps_s=[round(t, 3) for t in ts])
    out["ratio_oracle_over_reference"] = out["oracle"]["frames_per_s"] / \
        out["reference"]["frames_per_s"]
    cpu = subprocess.run(["lscpu"], capture_output=True, text=True).stdout
    model = [ln.split(":", 1)[1].strip() for ln in cpu.splitlines() if ln.startswith("Model name")]
    out.update(pairs=P, frames=T, threads=args.threads, cpu=model[0] if model else platform.processor(),
               torch=torch.__version__)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
