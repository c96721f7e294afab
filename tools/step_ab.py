"""Interleaved A/B of step-schedule switches on the bench workload (graph replay, 30 x 1024,
bf16): python tools/step_ab.py concurrency -> ms/step with the switch off / on,
two rounds, fresh model and capture per run."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep  # noqa: E402

SWITCHES = {"concurrency": engine.set_concurrency}


def run(steps=20):
    dev = torch.device("cuda", 0)
    torch.manual_seed(20250321)
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    b = data.synthetic_batch(30, 1024, 1000)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    gs = GraphedTrainStep(model, opt, g("x_main"), g("x_sub"), g("y_main"), g("spk_main"),
                          g("spk_sub"), b["lengths"].tolist(), warmup=1)
    for _ in range(3):
        gs.step()
    torch.cuda.synchronize()
    t0 = time.time()
    for _ in range(steps):
        loss, _ = gs.step()
    torch.cuda.synchronize()
    return (time.time() - t0) / steps * 1e3, loss.item()


if __name__ == "__main__":
    engine.set_gemm_precision("bf16")
    name = sys.argv[1]
    for rnd in range(2):
        for on in (False, True):
            SWITCHES[name](on)
            ms, loss = run()
            print(f"{name}={int(on)} round {rnd}: {ms:.3f} ms/step (loss {loss:.6f})", flush=True)
            torch.cuda.empty_cache()
