"""Per-launch census of one training step (dev tool): every libensvs entry point of one eager,
serial bench step (30 pairs x 1024 frames) timed with HIP events and tagged with the GEMM /
weight-gradient shape that issued it; aggregated by (entry point, shape), largest total
first.   python tools/census.py [rows] [synth]
synth: the mgc DiffNet's 100-step reverse diffusion of one (main, sub) pair at 2 000 frames
(eager, the launches the inference graph captures) instead of the training step; voc: one
uSFGAN generator pass over one 2 000-frame track (480 000 samples); post: the bench's
per-track post-acoustic processing and uSFGAN inputs of one 2 000-frame track; vocleg: the
bench's whole 6-part vocoder leg (post-processing per track, one batched generator pass);
sf0: the training step of the recipe-default SeparateF0 model instead.
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ensemble_svs_with_interactions_amd import _lib, configs, data, engine  # noqa: E402
from ensemble_svs_with_interactions_amd import kernels as K  # noqa: E402
from ensemble_svs_with_interactions_amd.train import FusedAdam, train_step  # noqa: E402

ROWS = int(sys.argv[1]) if len(sys.argv) > 1 else 45
SYNTH = len(sys.argv) > 2 and sys.argv[2] == "synth"
VOC = len(sys.argv) > 2 and sys.argv[2] == "voc"
POST = len(sys.argv) > 2 and sys.argv[2] in ("post", "vocleg")
VOCLEG = len(sys.argv) > 2 and sys.argv[2] == "vocleg"
SF0 = len(sys.argv) > 2 and sys.argv[2] == "sf0"
# sites: the training step with column-sum / weight-gradient launches tagged by the product's
# Python call site (which layer issues them)
SITES = len(sys.argv) > 2 and sys.argv[2] == "sites"
ONLY = sys.argv[3] if len(sys.argv) > 3 else None  # rows of one branch only (lf0/mgc/bap/vuv)
REC = []
TAG = [None]
ON = [False]
BR = [None]  # branch index of the enclosing engine.Branches.on(i) region (None: outside)
BR_NAMES = {0: "lf0", 1: "mgc", 2: "bap", 3: "vuv"}
orig_call = _lib.call
orig_on = engine.Branches.on


class _br:
    def __init__(self, ctx, i):
        self.ctx, self.i = ctx, i

    def __enter__(self):
        self.old = BR[0]
        BR[0] = self.i
        return self.ctx.__enter__()

    def __exit__(self, *exc):
        BR[0] = self.old
        return self.ctx.__exit__(*exc)


engine.Branches.on = lambda self, i: _br(orig_on(self, i), i)


def call(name, *args):
    if not ON[0]:
        return orig_call(name, *args)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    orig_call(name, *args)
    e.record()
    tag = TAG[0]
    if name in ("ensvs_lstm_mfma_fwd", "ensvs_lstm_mfma_bwd"):
        tag = f"H={args[6]} T={args[5]}"
    elif name == "ensvs_colsum":
        tag = f"M={args[2]} groups={args[3]} N={args[4]}{' centred' if args[5] else ''}"
        if SITES:
            tag += " @" + _site()
    elif name in ("ensvs_lstm_fwd", "ensvs_lstm_bwd"):
        tag = f"H={args[7]} B={args[5]} T={args[6]}"
    elif name in ("ensvs_lstm_coop_fwd", "ensvs_lstm_coop_bwd"):
        tag = f"H={args[6]} B={args[4]} T={args[5]}"
    REC.append((name, tag, s, e, BR[0]))


def _site():
    import traceback
    fr = [f for f in traceback.extract_stack()[:-3]
          if "ensemble_svs_with_interactions_amd" in f.filename
          and not f.filename.endswith(("kernels.py", "_lib.py"))]
    return " < ".join(f"{os.path.basename(f.filename)}:{f.name}:{f.lineno}" for f in fr[-2:][::-1])


def tagged(fn, fmt):
    def w(*a, **k):
        old = TAG[0]
        TAG[0] = fmt(*a, **k)
        try:
            return fn(*a, **k)
        finally:
            TAG[0] = old
    return w


def gemm_tag(segs, B, Tout, N, W, Y, ldy, **k):
    sg = "+".join(f"{s.K}x{s.taps}{'b' if s.x.dtype == torch.bfloat16 else 'f'}" for s in segs)
    return f"gemm M={B * Tout} N={N} K=[{sg}] epi={k.get('epi', 0)}"


def wgrad_tag(dy, ldy, x, ldx, B, Tout, Tin, N, Kc, taps, *a, **k):
    return (f"wgrad M={B * Tout} N={N} K={Kc}x{taps} "
            f"{'b' if dy.dtype == torch.bfloat16 else 'f'}" + (" @" + _site() if SITES else ""))


import importlib  # noqa: E402
import pkgutil  # noqa: E402
import ensemble_svs_with_interactions_amd as pkg  # noqa: E402

for m in [m for m in pkgutil.iter_modules(pkg.__path__) if not m.name.startswith("lib")]:
    mod = importlib.import_module(f"{pkg.__name__}.{m.name}")
    if getattr(mod, "call", None) is orig_call:
        mod.call = call
_lib.call = call
K.gemm = tagged(K.gemm, gemm_tag)
K.wgrad = tagged(K.wgrad, wgrad_tag)


def run_synth(dev):
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev).eval()
    gd = model.mgc_model
    B, T = 1, 2004
    E = gd.denoise_fn.E
    cond = torch.randn(B * T, E, device=dev)
    x = torch.randn(B * T, gd.out_dim, device=dev)
    noise = torch.randn(B * T, gd.out_dim, device=dev)
    gd._reverse(x, cond, E, B, T, lambda k: noise)
    torch.cuda.synchronize()
    ON[0] = True
    gd._reverse(x, cond, E, B, T, lambda k: noise)
    torch.cuda.synchronize()
    ON[0] = False


def run_voc(dev):
    from ensemble_svs_with_interactions_amd import usfgan
    voc = configs.instantiate(configs.usfgan_generator()).to(dev)
    voc.remove_weight_norm()
    wrapper = usfgan.USFGANWrapper({"data": dict(configs.USFGAN_DATA),
                                    "generator": {"aux_context_window": 2}}, voc)
    T = 2000
    f0 = 200.0 + 20.0 * torch.rand(1, T, device=dev)
    aux = torch.randn(1, T, voc.aux_channels, device=dev)
    wrapper.inference_batch(f0, aux)
    torch.cuda.synchronize()
    ON[0] = True
    wrapper.inference_batch(f0, aux)
    torch.cuda.synchronize()
    ON[0] = False


def run_post(dev):
    import types
    import numpy as np
    from ensemble_svs_with_interactions_amd import postprocess, scalers
    T = 2000
    b = data.synthetic_batch(1, T, 5)
    xm = torch.from_numpy(b["x_main"]).to(dev)[0]
    feats = torch.randn(T, 67, device=dev)
    mean_, var_ = np.zeros(67), np.full(67, 0.25)
    sc = scalers.StandardScaler(mean_, var_)
    cfg = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5], num_windows=1,
                                has_dynamic_features=[False] * 4)
    post = dict(frame_period=5, post_filter_type="gv", trajectory_smoothing=True,
                trajectory_smoothing_cutoff=50, trajectory_smoothing_cutoff_f0=20,
                vuv_threshold=0.3)

    def one():
        f = feats.clone()
        postprocess.inverse_transform(sc, f)
        st = postprocess.postprocess_acoustic(dev, f, xm, {}, {}, cfg, sc, pitch_idx=51, **post)
        return postprocess.usfgan_inputs(*st, sine_f0_type="f0", vuv_threshold=0.3)
    if VOCLEG:
        from ensemble_svs_with_interactions_amd import usfgan
        voc = configs.instantiate(configs.usfgan_generator()).to(dev)
        voc.remove_weight_norm()
        wrapper = usfgan.USFGANWrapper({"data": dict(configs.USFGAN_DATA),
                                        "generator": {"aux_context_window": 2}}, voc)
        single = one

        def one():
            f0s, auxs = zip(*[single() for _ in range(6)])
            return wrapper.inference_batch(torch.cat(f0s, 1).t().contiguous(),
                                           torch.stack(auxs))
    one()
    torch.cuda.synchronize()
    ON[0] = True
    one()
    torch.cuda.synchronize()
    ON[0] = False


def main():
    dev = torch.device("cuda")
    engine.set_concurrency(False)
    if POST:
        run_post(dev)
        return report()
    if VOC:
        run_voc(dev)
        return report()
    if SYNTH:
        run_synth(dev)
        return report()
    torch.manual_seed(20250321)
    cfg = configs.multitrack_separate_f0 if SF0 else configs.multitrack_diffusion
    model = configs.instantiate(cfg(num_speakers=4)).to(dev)
    opt = FusedAdam(model, lr=1e-4, clip_norm=1.0)
    P, T = 30, 1024
    b = data.synthetic_batch(P, T, 1000)
    g = lambda k: torch.from_numpy(b[k]).to(dev).contiguous()  # noqa: E731
    xm, xs, ym, s0, s1 = g("x_main"), g("x_sub"), g("y_main"), g("spk_main"), g("spk_sub")
    lens = b["lengths"].tolist()
    for _ in range(2):
        train_step(model, opt, xm, xs, ym, s0, s1, lens)
    torch.cuda.synchronize()
    ON[0] = True
    train_step(model, opt, xm, xs, ym, s0, s1, lens)
    torch.cuda.synchronize()
    ON[0] = False
    report()


def report():
    agg = collections.defaultdict(lambda: [0, 0.0])
    tot = 0.0
    per_br = collections.defaultdict(float)
    for name, tag, s, e, br in REC:
        ms = s.elapsed_time(e)
        a = agg[(name, tag)]
        a[0] += 1
        a[1] += ms
        tot += ms
        per_br[BR_NAMES.get(br, "other")] += ms
        if ONLY and BR_NAMES.get(br, "other") != ONLY:
            a[0] -= 1
            a[1] -= ms
    print(f"{len(REC)} launches, {tot:.2f} ms (event-bracketed, serial eager "
          f"{'reverse diffusion' if SYNTH else ('vocoder' if VOC else ('post' if POST else 'step'))})")
    print("per branch: " + "  ".join(f"{k} {v:.2f} ms" for k, v in sorted(per_br.items())))
    for (name, tag), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:ROWS]:
        if n <= 0:  # (entries of other branches only, with ONLY set)
            continue
        print(f"{ms:8.3f} ms {n:4d}x {ms / n * 1e3:8.1f} us  {name:28s} {tag or ''}")


if __name__ == "__main__":
    main()
