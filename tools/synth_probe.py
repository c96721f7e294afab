"""Acoustic-inference time vs batch size at T=2000 (dev tool): whole model.inference and
the captured reverse diffusion of the mgc stream alone.   python tools/synth_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: E402


def tmed(fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev).eval()
    T = 2000
    for B in [int(v) for v in (sys.argv[1:] or ["1", "2", "6"])]:
        b = data.synthetic_batch(B, T, 5 + B)
        g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
        xm, xs, s0, s1 = g("x_main"), g("x_sub"), g("spk_main"), g("spk_sub")
        f = lambda: model.inference(xm, xs, spks=(s0, s1), lengths=[T] * B)  # noqa: E731
        f()
        t_all = tmed(f)
        gd = model.mgc_model
        E = gd.encoder_out_dim if hasattr(gd, "encoder_out_dim") else 256
        cond = torch.randn(B * (T + 4), E, device=dev)
        r = lambda: gd._reverse_graph(cond, E, B, T + 4)  # noqa: E731
        try:
            r()
            t_rev = tmed(r)
        except Exception as e:  # probe only
            t_rev = float("nan")
            print("reverse probe failed:", e)
        print(f"B={B}: inference {t_all:7.1f} ms | mgc reverse graph {t_rev:7.1f} ms", flush=True)


if __name__ == "__main__":
    main()
