"""Pair inference time (T = 2000) with the branch streams concurrent vs serial, before and
after a captured training step in the same process (dev tool): whether mgc / bap reverse
diffusions overlap, or their streams share a hardware queue.
  python tools/infer_streams_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import configs, data, engine  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, GraphedTrainStep  # noqa: E402


def tmed(fn, reps=3):
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2] * 1e3


def infer_times(model, dev, tag):
    T, B = 2000, 1
    b = data.synthetic_batch(B, T, 6)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    xm, xs, s0, s1 = g("x_main"), g("x_sub"), g("spk_main"), g("spk_sub")
    model.eval()
    f = lambda: model.inference(xm, xs, spks=(s0, s1), lengths=[T] * B)  # noqa: E731
    out = {}
    for conc in (True, False):
        engine.set_concurrency(conc)
        f()
        out["concurrent" if conc else "serial"] = tmed(f)
    engine.set_concurrency(True)
    model.train()
    print(tag, {k: round(v, 1) for k, v in out.items()}, flush=True)


def main():
    dev = torch.device("cuda")
    torch.manual_seed(int(os.environ.get("PROBE_SEED", "0")))
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    if os.environ.get("PROBE_FRESH", "1") == "1":
        infer_times(model, dev, "fresh")
    if os.environ.get("PROBE_BRANCHES_FIRST", "0") == "1":
        with engine.Branches(dev) as br:
            for i in range(4):
                with br.on(i):
                    pass
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    b = data.synthetic_batch(30, 1024, 1000)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    targs = (g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub"),
             b["lengths"].tolist())
    if os.environ.get("PROBE_EAGER_TRAIN", "0") == "1":
        from ensemble_svs_with_interactions_amd.train import train_step
        for _ in range(int(os.environ.get("PROBE_STEPS", "2"))):
            train_step(model, opt, *targs)
    else:
        st = GraphedTrainStep(model, opt, *targs, warmup=1)
        for _ in range(int(os.environ.get("PROBE_STEPS", "2"))):
            st.step()
    torch.cuda.synchronize()
    infer_times(model, dev, "after training")
    from ensemble_svs_with_interactions_amd import diffsinger
    diffsinger.USE_GRAPHS["on"] = False
    infer_times(model, dev, "after training, eager reverse diffusion")
    diffsinger.USE_GRAPHS["on"] = True
    import bench
    bench._imports()
    bench.gate_gemm_timing(model, 30, 1024, dev)
    infer_times(model, dev, "after gate_gemm_timing")
    syn = bench.synth_rtf(model, dev, reps=3)
    print("bench synth pair acoustic_ms", round(syn["pair"]["acoustic_ms"], 1), flush=True)
    infer_times(model, dev, "after bench synth")
    engine.set_concurrency(False)
    syn = bench.synth_rtf(model, dev, reps=3)
    engine.set_concurrency(True)
    print("bench synth (serial) pair acoustic_ms", round(syn["pair"]["acoustic_ms"], 1),
          flush=True)


if __name__ == "__main__":
    main()
