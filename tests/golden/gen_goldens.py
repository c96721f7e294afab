"""Generate the golden fixtures in tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container (the reference lives at /root/reference and
never travels):   python tests/golden/gen_goldens.py

The reference package is imported with a stub loader for absent,
non-arithmetic dependencies (pyworld, librosa, hydra, ...).
Parameters come from oracle/weights.py (seeded by key), random draws
(AR-decoder dropout masks, diffusion t / noise) are injected so that the
oracle and the HIP path can replay them.  Fixtures store inputs, draws and
outputs only; weights are regenerated from the seed.

Deviation recorded for capture: nn.LSTM's internal inter-layer dropout of
the V/UV model (p=0.1) draws from torch's C++ RNG and cannot be replayed, so
training-mode goldens run it with dropout=0.
"""
import importlib.abc
import importlib.machinery
import json
import logging
import os
import sys
import tempfile
import types
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, "/root/reference")
sys.dont_write_bytecode = True

STUB_ROOTS = {"pyworld", "pysptk", "librosa", "pyloudnorm", "nnmnkwii", "mlflow", "h5py",
              "torchaudio", "tkinter", "hydra", "omegaconf", "tensorboard", "pysinsy", "soundfile"}


class _AnyObj:
    def __call__(self, *a, **k):
        return _AnyObj()

    def __getattr__(self, n):
        return _AnyObj()

    def __mro_entries__(self, bases):
        return (object,)


class _Any(types.ModuleType):
    def __getattr__(self, n):
        if n.startswith("__"):
            raise AttributeError(n)
        return _AnyObj()


class _Finder(importlib.abc.MetaPathFinder, importlib.abc.Loader):
    def find_spec(self, name, path, target=None):
        if name.split(".")[0] in STUB_ROOTS:
            return importlib.machinery.ModuleSpec(name, self, is_package=True)

    def create_module(self, spec):
        return _Any(spec.name)

    def exec_module(self, m):
        m.__path__ = []


sys.meta_path.insert(0, _Finder())
_tb = types.ModuleType("torch.utils.tensorboard")
_tb.SummaryWriter = object
sys.modules["torch.utils.tensorboard"] = _tb
import matplotlib  # noqa: E402

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402

plt.style.use = lambda *a, **k: None

import torch  # noqa: E402
import torch.nn.functional as TF  # noqa: E402

import nnsvs.acoustic_models.tacotron_f0 as ref_tacotron_f0  # noqa: E402
import nnsvs.diffsinger.diffusion as ref_diffusion  # noqa: E402
from nnsvs.acoustic_models.util import pad_inference_multitrack  # noqa: E402
from nnsvs.bin.train_acoustic_multitrack import train_step as ref_train_step  # noqa: E402
from nnsvs import train_util as ref_train_util  # noqa: E402
from nnsvs.util import make_non_pad_mask as ref_make_non_pad_mask  # noqa: E402

from ensemble_svs_with_interactions_amd import configs, data  # noqa: E402
from oracle.weights import seeded_state_dict  # noqa: E402

SEED = 20250321
torch.set_num_threads(8)


# ------------------------------------------------------------ injection

class _DropoutF:
    """Proxy for tacotron_f0.F whose dropout() replays queued keep masks."""

    def __init__(self):
        self.queue = []
        self.log = []

    def __getattr__(self, n):
        return getattr(TF, n)

    def dropout(self, x, p=0.5, training=True, inplace=False):
        m = self.queue.pop(0)
        self.log.append(m)
        return x * m


DROP = _DropoutF()
ref_tacotron_f0.F = DROP


class inject_diffusion:
    """Replace torch.randint / torch.randn_like / torch.randn with queued draws."""

    def __init__(self, ints=(), normals=()):
        self.ints = list(ints)
        self.normals = list(normals)

    def __enter__(self):
        self.saved = (torch.randint, torch.randn_like, torch.randn)
        torch.randint = lambda *a, **k: self.ints.pop(0)
        torch.randn_like = lambda x, **k: self.normals.pop(0)
        torch.randn = lambda *a, **k: self.normals.pop(0)
        # p_sample binds noise_fn=torch.randn at definition time (diffusion.py:194)
        self.saved_defaults = ref_diffusion.GaussianDiffusion.p_sample.__wrapped__.__defaults__
        ref_diffusion.GaussianDiffusion.p_sample.__wrapped__.__defaults__ = (torch.randn,) + \
            self.saved_defaults[1:]
        return self

    def __exit__(self, *exc):
        torch.randint, torch.randn_like, torch.randn = self.saved
        ref_diffusion.GaussianDiffusion.p_sample.__wrapped__.__defaults__ = self.saved_defaults
        assert not self.ints and not self.normals, "unconsumed draws"


def build_ref(cfg_mine, seed=SEED):
    cfg = configs.to_reference_targets(cfg_mine)
    torch.manual_seed(0)
    model = configs.instantiate(cfg)
    shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
    sd = seeded_state_dict(shapes, seed)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()},
                                                strict=False)
    assert not unexpected
    return model, shapes


def rng_for(name):
    return np.random.default_rng([SEED, zlib.crc32(name.encode())])


def grad_summary(module, prefix=""):
    """{key: [sum, abs-sum, l2]} of every parameter gradient (float64)."""
    out = {}
    for k, p in module.named_parameters():
        g = p.grad
        if g is None:
            out[prefix + k] = [0.0, 0.0, 0.0]
        else:
            g = g.double()
            out[prefix + k] = [g.sum().item(), g.abs().sum().item(), g.norm().item()]
    return out


def save(name, arrays, meta):
    path = os.path.join(HERE, name + ".npz")
    arrays = {k: np.asarray(v) for k, v in arrays.items()}
    arrays["meta_json"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(path, **arrays)
    print(f"{name}: {os.path.getsize(path) / 1e6:.2f} MB")


def T_(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def ar_masks(name, B, Tr):
    r = rng_for(name)
    return (r.random((B, Tr, 1)) < 0.5).astype(np.float32) * 2.0


# ---------------------------------------------------------------- cases

def case_diffnet(model, which, B, T, full_grads):
    gd = getattr(model, which + "_model")
    net = gd.denoise_fn
    M = net.in_dim
    E = net.residual_layers[0].conditioner_projection.in_channels
    r = rng_for("diffnet_" + which)
    spec = r.standard_normal((B, 1, M, T)).astype(np.float32) * 0.5
    t = r.integers(0, 100, size=B).astype(np.int64)
    cond = r.standard_normal((B, E, T)).astype(np.float32)
    R = r.standard_normal((B, 1, M, T)).astype(np.float32)
    spec_t = T_(spec).requires_grad_()
    cond_t = T_(cond).requires_grad_()
    net.zero_grad()
    out = net(spec_t, T_(t), cond_t)
    (out * T_(R)).sum().backward()
    arrays = dict(spec=spec, t=t, cond=cond, R=R, out=out.detach().numpy(),
                  d_spec=spec_t.grad.numpy(), d_cond=cond_t.grad.numpy())
    for k in full_grads:
        arrays["grad::" + k] = dict(net.named_parameters())[k].grad.numpy()
    meta = dict(prefix=f"{which}_model.denoise_fn.", grad_summary=grad_summary(net))
    save(f"diffnet_{which}", arrays, meta)


def case_ffconvlstm(model, which, B, T, lengths):
    enc = {"mgc": model.mgc_model.encoder, "bap": model.bap_model.encoder,
           "vuv": model.vuv_model}[which]
    prefix = {"mgc": "mgc_model.encoder.", "bap": "bap_model.encoder.", "vuv": "vuv_model."}[which]
    enc.train()
    if which == "vuv":
        enc.lstm.dropout = 0.0
    batch = data.synthetic_batch(B, T, SEED + 7, lengths=lengths)
    if which == "vuv":
        x = np.concatenate([batch["x_main"], batch["y_main"][:, :, :60],
                            batch["y_main"][:, :, 60:61]], -1)
    else:
        x = np.concatenate([batch["x_main"], batch["y_main"][:, :, 60:61]], -1)
    r = rng_for("ffconvlstm_" + which)
    spk = (0.3 * r.standard_normal((B, 1, enc.emb.embedding_dim))).astype(np.float32)
    spk_t = T_(spk).requires_grad_()
    enc.zero_grad()
    out = enc(T_(x), T_(batch["lengths"]), spk_embs=spk_t.expand(B, T, -1))
    R = r.standard_normal(tuple(out.shape)).astype(np.float32)
    (out * T_(R)).sum().backward()
    bn = {k: v.numpy().copy() for k, v in enc.state_dict().items() if "running" in k}
    arrays = dict(x=x, lengths=batch["lengths"], spk=spk, R=R, out=out.detach().numpy(),
                  d_spk=spk_t.grad.numpy(), **{"bn::" + k: v for k, v in bn.items()})
    meta = dict(prefix=prefix, grad_summary=grad_summary(enc))
    save(f"ffconvlstm_{which}", arrays, meta)


def case_lf0(model, B, T, lengths):
    lm = model.lf0_model
    lm.train()
    model._set_lf0_params()
    batch = data.synthetic_batch(B, T, SEED + 11, lengths=lengths)
    r = rng_for("lf0")
    E = model.speaker_embedding.emb.embedding_dim
    s0 = (0.3 * r.standard_normal((B, 1, E))).astype(np.float32)
    s1 = (0.3 * r.standard_normal((B, 1, E))).astype(np.float32)
    s0_t, s1_t = T_(s0).requires_grad_(), T_(s1).requires_grad_()
    masks = ar_masks("lf0_masks", B, T // 4)
    DROP.queue = [T_(masks[:, t]) for t in range(T // 4)]
    lm.zero_grad()
    lf0, res = lm(T_(batch["x_main"]), T_(batch["x_sub"]), s0_t.expand(B, T, -1),
                  s1_t.expand(B, T, -1), T_(batch["lengths"]))
    assert not DROP.queue
    R1 = r.standard_normal(tuple(lf0.shape)).astype(np.float32)
    R2 = r.standard_normal(tuple(res.shape)).astype(np.float32)
    ((lf0 * T_(R1)).sum() + (res * T_(R2)).sum()).backward()
    bn = {k: v.numpy().copy() for k, v in lm.state_dict().items() if "running" in k}
    arrays = dict(x_main=batch["x_main"], x_sub=batch["x_sub"], lengths=batch["lengths"],
                  spk_main=s0, spk_sub=s1, masks=masks, R1=R1, R2=R2,
                  lf0=lf0.detach().numpy(), res=res.detach().numpy(),
                  d_spk_main=s0_t.grad.numpy(), d_spk_sub=s1_t.grad.numpy(),
                  **{"bn::" + k: v for k, v in bn.items()})
    meta = dict(prefix="lf0_model.", grad_summary=grad_summary(lm),
                lf0_stats={k: getattr(model, k) for k in configs.LF0_STATS})
    save("lf0_model", arrays, meta)


def model_draws(name, P, T, cfg):
    r = rng_for(name)
    d = dict(lf0_main=ar_masks(name + "_lm", P, T // 4), lf0_sub=ar_masks(name + "_ls", P, T // 4),
             mgc_t=r.integers(0, 100, size=P).astype(np.int64),
             mgc_noise=r.standard_normal((P, 1, 60, T)).astype(np.float32),
             bap_t=r.integers(0, 100, size=P).astype(np.int64),
             bap_noise=r.standard_normal((P, 1, 5, T)).astype(np.float32))
    return d


def queue_draws(d, T):
    DROP.queue = [T_(d["lf0_main"][:, t]) for t in range(T // 4)] + \
                 [T_(d["lf0_sub"][:, t]) for t in range(T // 4)]
    return inject_diffusion(ints=[T_(d["mgc_t"]), T_(d["bap_t"])],
                            normals=[T_(d["mgc_noise"]), T_(d["bap_noise"])])


def case_model_forward_full():
    cfg = configs.multitrack_diffusion(num_speakers=4)
    model, shapes = build_ref(cfg)
    model.train()
    model.vuv_model.lstm.dropout = 0.0
    P, T = 2, 32
    batch = data.synthetic_batch(P, T, SEED + 13, lengths=[32, 28])
    d = model_draws("fwd_full", P, T, cfg)
    with queue_draws(d, T):
        ((mgc, lf0, vuv, bap), res), sub = model(
            T_(batch["x_main"]), T_(batch["x_sub"]),
            (T_(batch["spk_main"]).int(), T_(batch["spk_sub"]).int()),
            lengths=T_(batch["lengths"]), ys=[T_(batch["y_main"]), T_(batch["y_sub"])])
    assert sub == (None, None) and not DROP.queue
    arrays = dict(**{k: v for k, v in batch.items()}, **{"draw::" + k: v for k, v in d.items()},
                  mgc_noise_out=mgc[0].detach().numpy(), mgc_recon=mgc[1].detach().numpy(),
                  lf0=lf0.detach().numpy(), vuv=vuv.detach().numpy(),
                  bap_noise_out=bap[0].detach().numpy(), bap_recon=bap[1].detach().numpy(),
                  res=res.detach().numpy())
    save("model_forward_full", arrays, dict(shapes={k: list(v) for k, v in shapes.items()}))
    return model, shapes


def case_train_step_tiny(steps=2, lr=1e-3, logf0_diff_weight=0.0, name="train_step_tiny"):
    """logf0_diff_weight > 0: the interaction-loss recipe (output_subtrack model,
    train_acoustic_multitrack.py:175-182, 296)."""
    il = logf0_diff_weight > 0
    cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True, output_subtrack=il)
    model, shapes = build_ref(cfg)
    model.vuv_model.lstm.dropout = 0.0
    P, T = 3, 48
    batch = data.synthetic_batch(P, T, SEED + 17, lengths=[48, 40, 32])
    opt = torch.optim.Adam(model.parameters(), lr=lr, betas=(0.9, 0.999), weight_decay=0.0)
    model_config = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5])
    optim_config = types.SimpleNamespace(clip_norm=1.0)
    logger = logging.getLogger("golden")
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}
    arrays = dict(**{k: v for k, v in batch.items()})
    meta = dict(shapes={k: list(v) for k, v in shapes.items()}, lr=lr, steps=steps)
    losses, norms = [], []
    for s in range(steps):
        d = model_draws(f"tiny_step{s}", P, T, cfg)
        for k, v in d.items():
            arrays[f"draw{s}::{k}"] = v
        # record the grad norm that clip_grad_norm_ returns
        norm_box = {}
        orig = torch.nn.utils.clip_grad_norm_

        def clip(params, max_norm, *a, **k):
            n = orig(params, max_norm, *a, **k)
            norm_box["n"] = float(n)
            return n
        torch.nn.utils.clip_grad_norm_ = clip
        try:
            with queue_draws(d, T):
                loss, metrics = ref_train_step(
                    logger, model, model_config, optim_config, opt, None, True,
                    (T_(batch["x_main"]), T_(batch["x_sub"])),
                    [T_(batch["y_main"]), T_(batch["y_sub"])],
                    (T_(batch["spk_main"]).int(), T_(batch["spk_sub"]).int()),
                    (T_(batch["lengths"]), T_(batch["lengths"])),
                    None, None, feats_criterion="l1", pitch_reg_weight=0.0,
                    logf0_diff_weight=logf0_diff_weight, mgc_diff_weight=0.0)
        finally:
            torch.nn.utils.clip_grad_norm_ = orig
        losses.append(float(loss))
        norms.append(norm_box["n"])
        if il:
            meta.setdefault("interaction_losses", []).append(
                float(metrics["Loss_LogF0_Interaction"]))
        after = {k: v.detach().clone() for k, v in model.state_dict().items()}
        if s == 0:
            for k in after:
                if after[k].dtype == torch.float32:
                    arrays[f"delta0::{k}"] = (after[k] - before[k]).numpy()
    for k, v in model.state_dict().items():
        if v.dtype == torch.float32:
            arrays[f"final::{k}"] = v.numpy()
    meta.update(losses=losses, grad_norms=norms, logf0_diff_weight=logf0_diff_weight)
    save(name, arrays, meta)


GRAD_SAMPLE = 2048


def grad_sample_index(key, numel):
    """Fixed sample of element indices of one parameter's gradient (at most GRAD_SAMPLE):
    a full-width model's gradients are 94 MB, so the fixture keeps a seeded subset of every
    tensor (enough for a per-tensor relative-L2 estimate) plus its exact sum / abs / l2."""
    if numel <= GRAD_SAMPLE:
        return np.arange(numel, dtype=np.int64)
    return np.sort(rng_for("gsample_" + key).choice(numel, GRAD_SAMPLE, replace=False))


def case_train_step_full(steps=2, lr=1e-4, P=2, T=64, lengths=(64, 52), name="train_step_full"):
    """The reference train_step (train_acoustic_multitrack.py:40-392) on the recipe-width
    model (multitrack_acoustic_nnsvs_world_multi_ar_f0_diff_mgcbap.yaml), V/UV LSTM dropout
    0 (see the module docstring): losses, grad norms, per-step loss metrics, step-0 gradient
    summaries + sampled elements of every parameter gradient, final BN running statistics.
    name="train_step_prod": the same at the bench's sequence length (T = 1024, 256 free-running
    AR-decoder steps per track), the fixture the bf16 production route is checked against."""
    cfg = configs.multitrack_diffusion(num_speakers=4)
    model, shapes = build_ref(cfg)
    model.vuv_model.lstm.dropout = 0.0
    batch = data.synthetic_batch(P, T, SEED + 23, lengths=list(lengths))
    opt = torch.optim.Adam(model.parameters(), lr=lr, betas=(0.9, 0.999), weight_decay=0.0)
    model_config = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5])
    optim_config = types.SimpleNamespace(clip_norm=1.0)
    logger = logging.getLogger("golden")
    arrays = dict(**{k: v for k, v in batch.items()})
    meta = dict(shapes={k: list(v) for k, v in shapes.items()}, lr=lr, steps=steps,
                grad_sample=GRAD_SAMPLE)
    losses, norms, feats = [], [], []
    for s in range(steps):
        d = model_draws(("full" if name == "train_step_full" else name) + f"_step{s}", P, T, cfg)
        for k, v in d.items():
            arrays[f"draw{s}::{k}"] = v
        norm_box = {}
        orig = torch.nn.utils.clip_grad_norm_

        def clip(params, max_norm, *a, **k):
            n = orig(params, max_norm, *a, **k)
            norm_box["n"] = float(n)
            return n
        torch.nn.utils.clip_grad_norm_ = clip
        try:
            with queue_draws(d, T):
                loss, metrics = ref_train_step(
                    logger, model, model_config, optim_config, opt, None, True,
                    (T_(batch["x_main"]), T_(batch["x_sub"])),
                    [T_(batch["y_main"]), T_(batch["y_sub"])],
                    (T_(batch["spk_main"]).int(), T_(batch["spk_sub"]).int()),
                    (T_(batch["lengths"]), T_(batch["lengths"])),
                    None, None, feats_criterion="l1", pitch_reg_weight=0.0,
                    logf0_diff_weight=0.0, mgc_diff_weight=0.0)
        finally:
            torch.nn.utils.clip_grad_norm_ = orig
        losses.append(float(loss))
        norms.append(norm_box["n"])
        feats.append(float(metrics["Loss_Feats"]))
        if s == 0:
            # gradients as the optimizer saw them (after clipping they are scaled in place
            # by clip_grad_norm_: undo the scale so the fixture holds the raw gradient)
            coef = min(1.0, 1.0 / (norm_box["n"] + 1e-6))
            summ = {}
            for k, p in model.named_parameters():
                g = p.grad.detach().double().reshape(-1) / coef
                summ[k] = [g.sum().item(), g.abs().sum().item(), g.norm().item()]
                idx = grad_sample_index(k, g.numel())
                arrays[f"gidx::{k}"] = idx.astype(np.int32)
                arrays[f"gval::{k}"] = g[torch.from_numpy(idx)].numpy()
            meta["grad_summary"] = summ
    for k, v in model.state_dict().items():
        if "running" in k:
            arrays[f"final::{k}"] = v.numpy()
    meta.update(losses=losses, grad_norms=norms, loss_feats=feats)
    save(name, arrays, meta)


def case_inference_bap(model):
    gd = model.bap_model
    gd.eval()
    B, T = 1, 32
    batch = data.synthetic_batch(B, T, SEED + 19)
    cond_in = np.concatenate([batch["x_main"], batch["y_main"][:, :, 60:61]], -1)
    r = rng_for("inference_bap")
    spk = (0.3 * r.standard_normal((B, 1, 256))).astype(np.float32)
    noises = r.standard_normal((101, B, 1, 5, T)).astype(np.float32)
    with torch.no_grad(), inject_diffusion(normals=[T_(n) for n in noises]):
        out = gd.inference(T_(cond_in), T_(batch["lengths"]), spk_embs=T_(spk).expand(B, T, -1))
    save("inference_bap", dict(cond_in=cond_in, lengths=batch["lengths"], spk=spk, noises=noises,
                               out=out.numpy()), {})


def case_model_inference_tiny():
    cfg = configs.multitrack_diffusion(num_speakers=4, tiny=True)
    model, shapes = build_ref(cfg)
    model.eval()
    arrays, meta = {}, {}
    for T in (28, 29, 30, 31):
        batch = data.synthetic_batch(1, T, SEED + 23 + T)
        pad = 4 - T % 4
        Tp = T + pad
        r = rng_for(f"inf_tiny_{T}")
        masks = ar_masks(f"inf_tiny_masks_{T}", 2, Tp // 4)
        nm = r.standard_normal((101, 1, 1, 60, Tp)).astype(np.float32)
        nb = r.standard_normal((101, 1, 1, 5, Tp)).astype(np.float32)
        DROP.queue = [T_(masks[0:1, t]) for t in range(Tp // 4)] + \
                     [T_(masks[1:2, t]) for t in range(Tp // 4)]
        with torch.no_grad(), inject_diffusion(normals=[T_(n) for n in nm] + [T_(n) for n in nb]):
            out = model.inference(T_(batch["x_main"]), T_(batch["x_sub"]),
                                  spks=(T_(batch["spk_main"]).int(), T_(batch["spk_sub"]).int()),
                                  lengths=T_(batch["lengths"]))
        assert not DROP.queue
        for k in ("x_main", "x_sub", "spk_main", "spk_sub", "lengths"):
            arrays[f"T{T}::{k}"] = batch[k]
        arrays[f"T{T}::masks"] = masks
        arrays[f"T{T}::noise_mgc"] = nm
        arrays[f"T{T}::noise_bap"] = nb
        arrays[f"T{T}::out"] = out.numpy()
        meta[f"T{T}"] = dict(pad=pad, out_shape=list(out.shape))
    meta["shapes"] = {k: list(v) for k, v in shapes.items()}
    save("model_inference_tiny", arrays, meta)


def sf0_ref(tiny):
    """The SeparateF0 recipe model with the decoders' / encoder's nn.LSTM inter-layer
    dropout off (torch's C++ RNG cannot be replayed; module docstring)."""
    model, shapes = build_ref(configs.multitrack_separate_f0(num_speakers=4, tiny=tiny))
    for m in (model.mgc_model, model.vuv_model, model.bap_model, model.encoder):
        m.lstm.dropout = 0.0
    return model, shapes


def sf0_queue(d, T):
    DROP.queue = [T_(d["lf0_main"][:, t]) for t in range(T // 4)] + \
                 [T_(d["lf0_sub"][:, t]) for t in range(T // 4)]


def case_sf0_forward(tiny, P, T, lengths, name):
    """MultiTrackMultistreamSeparateF0ParametricModel.forward in training mode (teacher
    forcing) through the reference API, then backward of sum(out_main * R0 + res_main * R1
    + out_sub * R2 + res_sub * R3): outputs, BatchNorm running statistics after the call and
    the parameter gradients (all of them for the tiny model, summaries for the full one)."""
    model, shapes = sf0_ref(tiny)
    model.train()
    batch = data.synthetic_batch(P, T, SEED + 29, lengths=lengths)
    d = dict(lf0_main=ar_masks(name + "_lm", P, T // 4), lf0_sub=ar_masks(name + "_ls", P, T // 4))
    sf0_queue(d, T)
    model.zero_grad()
    (om, rm), (os_, rs) = model(T_(batch["x_main"]), T_(batch["x_sub"]),
                                (T_(batch["spk_main"]).int(), T_(batch["spk_sub"]).int()),
                                lengths=T_(batch["lengths"]),
                                ys=[T_(batch["y_main"]), T_(batch["y_sub"])])
    assert not DROP.queue
    r = rng_for(name)
    Rs = [r.standard_normal(tuple(t.shape)).astype(np.float32) for t in (om, rm, os_, rs)]
    sum((t * T_(R)).sum() for t, R in zip((om, rm, os_, rs), Rs)).backward()
    arrays = dict(**{k: v for k, v in batch.items()}, **{"draw::" + k: v for k, v in d.items()},
                  out_main=om.detach().numpy(), res_main=rm.detach().numpy(),
                  out_sub=os_.detach().numpy(), res_sub=rs.detach().numpy(),
                  **{f"R{i}": R for i, R in enumerate(Rs)})
    for k, v in model.state_dict().items():
        if "running" in k:
            arrays["bn::" + k] = v.numpy().copy()
    if tiny:
        for k, p_ in model.named_parameters():
            arrays["grad::" + k] = (p_.grad if p_.grad is not None
                                    else torch.zeros_like(p_)).numpy()
    meta = dict(shapes={k: list(v) for k, v in shapes.items()}, grad_summary=grad_summary(model),
                lengths=list(lengths))
    save(name, arrays, meta)


def case_sf0_train_tiny(steps=2, lr=1e-3):
    """Two reference train steps (train_acoustic_multitrack.py:40-392: deterministic-loss
    branch, feats_criterion l1, clip 1.0, Adam) of the tiny SeparateF0 model."""
    model, shapes = sf0_ref(True)
    P, T = 3, 48
    batch = data.synthetic_batch(P, T, SEED + 31, lengths=[48, 40, 32])
    opt = torch.optim.Adam(model.parameters(), lr=lr, betas=(0.9, 0.999), weight_decay=0.0)
    model_config = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5])
    optim_config = types.SimpleNamespace(clip_norm=1.0)
    logger = logging.getLogger("golden")
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}
    arrays = dict(**{k: v for k, v in batch.items()})
    meta = dict(shapes={k: list(v) for k, v in shapes.items()}, lr=lr, steps=steps)
    losses, norms = [], []
    for s in range(steps):
        d = dict(lf0_main=ar_masks(f"sf0_step{s}_lm", P, T // 4),
                 lf0_sub=ar_masks(f"sf0_step{s}_ls", P, T // 4))
        for k, v in d.items():
            arrays[f"draw{s}::{k}"] = v
        norm_box = {}
        orig = torch.nn.utils.clip_grad_norm_

        def clip(params, max_norm, *a, **k):
            n = orig(params, max_norm, *a, **k)
            norm_box["n"] = float(n)
            return n
        torch.nn.utils.clip_grad_norm_ = clip
        try:
            sf0_queue(d, T)
            loss, _ = ref_train_step(
                logger, model, model_config, optim_config, opt, None, True,
                (T_(batch["x_main"]), T_(batch["x_sub"])),
                [T_(batch["y_main"]), T_(batch["y_sub"])],
                (T_(batch["spk_main"]).int(), T_(batch["spk_sub"]).int()),
                (T_(batch["lengths"]), T_(batch["lengths"])),
                None, None, feats_criterion="l1", pitch_reg_weight=0.0,
                logf0_diff_weight=0.0, mgc_diff_weight=0.0)
            assert not DROP.queue
        finally:
            torch.nn.utils.clip_grad_norm_ = orig
        losses.append(float(loss))
        norms.append(norm_box["n"])
        if s == 0:
            after = {k: v.detach().clone() for k, v in model.state_dict().items()}
            for k in after:
                if after[k].dtype == torch.float32:
                    arrays[f"delta0::{k}"] = (after[k] - before[k]).numpy()
    for k, v in model.state_dict().items():
        if v.dtype == torch.float32:
            arrays[f"final::{k}"] = v.numpy()
    meta.update(losses=losses, grad_norms=norms)
    save("sf0_train_tiny", arrays, meta)


def case_sf0_inference_tiny():
    model, shapes = sf0_ref(True)
    model.eval()
    arrays, meta = {}, {}
    for T in (29, 32):
        batch = data.synthetic_batch(2, T, SEED + 37 + T, lengths=[T, T - 5])
        pad = 4 - T % 4
        Tp = T + pad
        masks = ar_masks(f"sf0_inf_{T}_lm", 2, Tp // 4), ar_masks(f"sf0_inf_{T}_ls", 2, Tp // 4)
        sf0_queue(dict(lf0_main=masks[0], lf0_sub=masks[1]), Tp)
        with torch.no_grad():
            out = model.inference(T_(batch["x_main"]), T_(batch["x_sub"]),
                                  spks=(T_(batch["spk_main"]).int(), T_(batch["spk_sub"]).int()),
                                  lengths=T_(batch["lengths"]))
        assert not DROP.queue
        for k in ("x_main", "x_sub", "spk_main", "spk_sub", "lengths"):
            arrays[f"T{T}::{k}"] = batch[k]
        arrays[f"T{T}::masks_main"] = masks[0]
        arrays[f"T{T}::masks_sub"] = masks[1]
        arrays[f"T{T}::out"] = out.numpy()
        meta[f"T{T}"] = dict(pad=pad, out_shape=list(out.shape))
    save("sf0_inference_tiny", arrays, meta)


def st_draws(name, P, T):
    r = rng_for(name)
    return dict(lf0_main=ar_masks(name + "_lm", P, T // 4),
                mgc_t=r.integers(0, 100, size=P).astype(np.int64),
                mgc_noise=r.standard_normal((P, 1, 60, T)).astype(np.float32),
                bap_t=r.integers(0, 100, size=P).astype(np.int64),
                bap_noise=r.standard_normal((P, 1, 5, T)).astype(np.float32))


def st_queue(d, T):
    DROP.queue = [T_(d["lf0_main"][:, t]) for t in range(T // 4)]
    return inject_diffusion(ints=[T_(d["mgc_t"]), T_(d["bap_t"])],
                            normals=[T_(d["mgc_noise"]), T_(d["bap_noise"])])


def case_st_forward_full():
    """BASELINE config 2: single-track NPSSMDNMultistreamParametricModel (multistream.py:
    1025-1243) training forward at full size, teacher-forced lf0 decoder."""
    model, shapes = build_ref(configs.singletrack_diffusion())
    model.train()
    model.vuv_model.lstm.dropout = 0.0
    P, T = 2, 32
    batch = data.synthetic_batch(P, T, SEED + 29, lengths=[32, 28])
    d = st_draws("st_fwd_full", P, T)
    with st_queue(d, T):
        (mgc, lf0, vuv, bap), res = model(T_(batch["x_main"]), T_(batch["lengths"]),
                                          T_(batch["y_main"]))
    assert not DROP.queue
    arrays = dict(x=batch["x_main"], y=batch["y_main"], lengths=batch["lengths"],
                  **{"draw::" + k: v for k, v in d.items()},
                  mgc_noise_out=mgc[0].detach().numpy(), mgc_recon=mgc[1].detach().numpy(),
                  lf0=lf0.detach().numpy(), vuv=vuv.detach().numpy(),
                  bap_noise_out=bap[0].detach().numpy(), bap_recon=bap[1].detach().numpy(),
                  res=res.detach().numpy())
    save("st_forward_full", arrays, dict(shapes={k: list(v) for k, v in shapes.items()}))


def case_st_train_tiny(steps=2, lr=1e-3):
    """2 steps of the reference single-track train_step (nnsvs/bin/train_acoustic.py:33-274,
    feats_criterion l1, no AMP) on the tiny single-track config."""
    from nnsvs.bin.train_acoustic import train_step as ref_st_train_step
    model, shapes = build_ref(configs.singletrack_diffusion(tiny=True))
    model.vuv_model.lstm.dropout = 0.0
    P, T = 3, 48
    batch = data.synthetic_batch(P, T, SEED + 31, lengths=[48, 40, 32])
    opt = torch.optim.Adam(model.parameters(), lr=lr, betas=(0.9, 0.999), weight_decay=0.0)
    model_config = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5])
    optim_config = types.SimpleNamespace(clip_norm=1.0)
    logger = logging.getLogger("golden")
    before = {k: v.detach().clone() for k, v in model.state_dict().items()}
    arrays = dict(x=batch["x_main"], y=batch["y_main"], lengths=batch["lengths"])
    meta = dict(shapes={k: list(v) for k, v in shapes.items()}, lr=lr, steps=steps)
    losses, norms = [], []
    for s in range(steps):
        d = st_draws(f"st_tiny_step{s}", P, T)
        for k, v in d.items():
            arrays[f"draw{s}::{k}"] = v
        with st_queue(d, T):
            loss, metrics = ref_st_train_step(
                logger, model, model_config, optim_config, opt, None, True, T_(batch["x_main"]),
                T_(batch["y_main"]), T_(batch["lengths"]), None, feats_criterion="l1",
                pitch_reg_dyn_ws=1.0, pitch_reg_weight=0.0, stream_wise_loss=False)
        losses.append(float(loss))
        norms.append(float(metrics["GradNorm"]))
        if s == 0:
            after = {k: v.detach().clone() for k, v in model.state_dict().items()}
            for k in after:
                if after[k].dtype == torch.float32:
                    arrays[f"delta0::{k}"] = (after[k] - before[k]).numpy()
    for k, v in model.state_dict().items():
        if v.dtype == torch.float32:
            arrays[f"final::{k}"] = v.numpy()
    meta.update(losses=losses, grad_norms=norms)
    save("st_train_step_tiny", arrays, meta)


def case_st_inference_tiny():
    """Single-track inference: pad_inference(mdn=True) around forward(y=None), whose
    lf0_model.inference pads r frames more (multistream.py:1152), T mod 4 = 0..3."""
    model, shapes = build_ref(configs.singletrack_diffusion(tiny=True))
    model.eval()
    arrays, meta = {}, {}
    for T in (28, 29, 30, 31):
        batch = data.synthetic_batch(1, T, SEED + 37 + T)
        pad = 4 - T % 4
        Tp = T + pad
        Tpp = Tp + 4
        r = rng_for(f"st_inf_tiny_{T}")
        masks = ar_masks(f"st_inf_tiny_masks_{T}", 1, Tpp // 4)
        nm = r.standard_normal((101, 1, 1, 60, Tp)).astype(np.float32)
        nb = r.standard_normal((101, 1, 1, 5, Tp)).astype(np.float32)
        DROP.queue = [T_(masks[0:1, t]) for t in range(Tpp // 4)]
        with torch.no_grad(), inject_diffusion(normals=[T_(n) for n in nm] + [T_(n) for n in nb]):
            mu, sigma = model.inference(T_(batch["x_main"]), T_(batch["lengths"]))
        assert not DROP.queue and torch.equal(mu, sigma)
        arrays[f"T{T}::x"] = batch["x_main"]
        arrays[f"T{T}::lengths"] = batch["lengths"]
        arrays[f"T{T}::masks"] = masks
        arrays[f"T{T}::noise_mgc"] = nm
        arrays[f"T{T}::noise_bap"] = nb
        arrays[f"T{T}::out"] = mu.numpy()
        meta[f"T{T}"] = dict(pad=pad, out_shape=list(mu.shape))
    meta["shapes"] = {k: list(v) for k, v in shapes.items()}
    save("st_inference_tiny", arrays, meta)


class FakeLabels:
    """Test-side stand-in for nnmnkwii's HTSLabelFile in the timing-inference golden: it only
    CARRIES data (start/end times, context strings, per-label feature rows returned by the
    patched fe.linguistic_features); every arithmetic step is the reference's own."""

    def __init__(self, start, end, contexts, feats):
        self.start_times = list(start)
        self.end_times = list(end)
        self.contexts = list(contexts)
        self.feats = np.asarray(feats, dtype=np.float32)
        self.frame_shift = 50000

    def round_(self):
        return self

    def __len__(self):
        return len(self.start_times)

    def __getitem__(self, idx):
        idx = list(idx)
        return FakeLabels([self.start_times[i] for i in idx], [self.end_times[i] for i in idx],
                          [self.contexts[i] for i in idx], self.feats[idx])


def timing_track(r, n_notes, D, grid):
    """A synthetic score track: notes on a coarse onset grid (ties with the other track),
    1-3 phonemes per note sharing the note's onset (as get_note_indices expects), a silence
    note now and then.  Times in HTS units (5 ms frame = 50 000)."""
    onsets = np.sort(r.choice(np.arange(0, grid), size=n_notes, replace=False)) * 10 * 50000
    start, end, ctx = [], [], []
    for k, o in enumerate(onsets):
        nxt = onsets[k + 1] if k + 1 < n_notes else o + 10 * 50000
        sil = r.random() < 0.15
        nph = 1 if sil else int(r.integers(1, 4))
        for _ in range(nph):
            start.append(int(o))
            end.append(int(nxt))
            ctx.append("x-sil+y@1" if sil else "x-a+y@1")
    feats = r.random((len(start), D)).astype(np.float32) * 4 - 1
    return start, end, ctx, feats


def case_timing_inference():
    """predict_timelag_multitrack (gen.py:214-416) and predict_duration_multitrack
    (gen.py:551-720) of the reference on two synthetic score tracks, with the recipe's
    MDN time-lag / duration models (seeded weights) and fitted sklearn scalers."""
    import nnsvs.gen as ref_gen
    from nnsvs.model import MultiTrackVariancePredictor as RefVP
    from sklearn.preprocessing import MinMaxScaler, StandardScaler
    ref_gen.fe = types.SimpleNamespace(
        linguistic_features=lambda labels, *a, **k: np.asarray(labels.feats))
    r = rng_for("timing_inference")
    D = 82
    arrays, meta = {}, {"cases": []}
    models = {}
    for name in ("timelag", "duration"):
        cfg = configs.multitrack_timing(name, num_speaker=3)
        cfg = {k: v for k, v in cfg.items() if k != "_target_"}
        torch.manual_seed(0)
        m = RefVP(**cfg)
        shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
        m.load_state_dict({k: torch.from_numpy(v) for k, v in
                           seeded_state_dict(shapes, SEED).items()})
        m.eval()
        models[name] = m
        fit = r.random((500, D)) * 5 - 2
        ins = MinMaxScaler().fit(fit)
        outs = StandardScaler().fit(r.standard_normal((500, 1)) * 7 + (1 if name == "timelag" else 9))
        models[name + "_sc"] = (ins, outs)
        for k in ("min_", "scale_", "data_min_", "data_max_"):
            arrays[f"{name}::in::{k}"] = getattr(ins, k)
        for k in ("mean_", "var_", "scale_"):
            arrays[f"{name}::out::{k}"] = getattr(outs, k)
    conf = types.SimpleNamespace(has_dynamic_features=[False])
    for case in range(3):
        tr = [timing_track(r, int(r.integers(6, 14)), D, 30) for _ in range(2)]
        labs = [FakeLabels(*t) for t in tr]
        spk = [int(r.integers(0, 3)) for _ in range(2)]
        spks = [torch.IntTensor([spk[0]]), torch.IntTensor([spk[1]])]
        lag, lag_eval, mask = ref_gen.predict_timelag_multitrack(
            "cpu", labs, spks, models["timelag"], conf, models["timelag_sc"][0],
            models["timelag_sc"][1], {}, {}, pitch_indices=[], log_f0_conditioning=False,
            force_clip_input_features=True)
        labs = [FakeLabels(*t) for t in tr]
        mu, sig = ref_gen.predict_duration_multitrack(
            "cpu", labs, spks, models["duration"], conf, models["duration_sc"][0],
            models["duration_sc"][1], {}, {}, pitch_indices=[], log_f0_conditioning=False,
            force_clip_input_features=True)
        p = f"c{case}::"
        for t in range(2):
            arrays[p + f"start{t}"] = np.asarray(tr[t][0], dtype=np.int64)
            arrays[p + f"end{t}"] = np.asarray(tr[t][1], dtype=np.int64)
            arrays[p + f"sil{t}"] = np.asarray(["sil" in c for c in tr[t][2]])
            arrays[p + f"feats{t}"] = tr[t][3]
        arrays[p + "spk"] = np.asarray(spk)
        arrays[p + "lag"] = np.asarray(lag)
        arrays[p + "lag_eval"] = np.asarray(lag_eval)
        arrays[p + "mask"] = np.asarray(mask)
        arrays[p + "dur_mu"] = np.asarray(mu)
        arrays[p + "dur_sigma_sq"] = np.asarray(sig)
        meta["cases"].append(case)
    meta["shapes"] = {n: {k: list(v.shape) for k, v in models[n].state_dict().items()}
                      for n in ("timelag", "duration")}
    save("timing_inference", arrays, meta)


def case_data_path():
    """Integer/byte fixtures: pairing, collation, masks (bit-exact)."""
    r = rng_for("data_path")
    arrays, meta = {}, {}
    with tempfile.TemporaryDirectory() as d:
        names = []
        for spk in ("Vo1", "S1", "ritsu", "A2"):
            for seg in ("seg01", "seg02", "songB_003"):
                if spk == "A2" and seg == "seg02":
                    continue
                n = int(r.integers(20, 60))
                np.save(os.path.join(d, f"{spk}_{seg}-feats.npy"), np.zeros((n, 3), np.float32))
                names.append(f"{spk}_{seg}")
        pairs, plens = ref_train_util.get_filtered_files_multitrack(d, None)
        meta["pairs"] = [[os.path.basename(a), os.path.basename(b)] for a, b in pairs]
        meta["pair_lengths"] = [[int(a), int(b)] for a, b in plens]
        files = sorted(os.path.join(d, f) for f in os.listdir(d))
        meta["files"] = [os.path.basename(f) for f in files]
        meta["file_lengths"] = [int(len(np.load(f))) for f in files]
    batch = []
    for i in range(5):
        n0, n1 = int(r.integers(17, 40)), int(r.integers(17, 40))
        x0 = r.standard_normal((n0, 6)).astype(np.float32)
        y0 = r.standard_normal((n0, 4)).astype(np.float32)
        x1 = r.standard_normal((n1, 6)).astype(np.float32)
        y1 = r.standard_normal((n1, 4)).astype(np.float32)
        batch.append((x0, y0, int(r.integers(0, 3)), np.zeros(3), x1, y1, int(r.integers(0, 3)),
                      np.zeros(3)))
        for k, v in dict(x0=x0, y0=y0, x1=x1, y1=y1).items():
            arrays[f"in{i}::{k}"] = v
        arrays[f"in{i}::spk"] = np.array([batch[-1][2], batch[-1][6]])
    out = ref_train_util.collate_fn_syncmultitrack_acoustic(batch, reduction_factor=4)
    for i, o in enumerate(out):
        arrays[f"collate{i}"] = o.numpy()
    lengths = r.integers(1, 50, size=7)
    arrays["mask_lengths"] = lengths
    arrays["non_pad_mask"] = ref_make_non_pad_mask(torch.from_numpy(lengths)).numpy()
    # pad_inference_multitrack frame arithmetic (util.py:157-158)
    meta["pad_inference"] = {str(T): int(4 - T % 4) for T in range(24, 33)}
    save("data_path", arrays, meta)


class _AttrDict(dict):
    """Stand-in for the OmegaConf vocoder config: attribute access + `in`."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k)


def case_usfgan():
    """uSFGAN generator forward and USFGANWrapper.inference (usfgan/__init__.py:13-65) at
    40 frames (9 600 samples: > the 512 dilation of the filter network), weight norm on."""
    from nnsvs.usfgan import USFGANWrapper as RefWrapper
    cfg = configs.to_reference_targets(configs.usfgan_generator())
    torch.manual_seed(0)
    gen = configs.instantiate(cfg)
    shapes = {k: tuple(v.shape) for k, v in gen.state_dict().items()}
    sd = seeded_state_dict(shapes, SEED)
    gen.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    gen.eval()
    r = rng_for("usfgan")
    T = 40
    f0 = np.repeat(r.uniform(110.0, 880.0, size=T // 5), 5).astype(np.float32)
    f0[12:17] = 0.0  # unvoiced frames: d = 1, vuv = 0
    f0 = f0.reshape(T, 1)
    aux = r.standard_normal((T, 65)).astype(np.float32)
    L = T * configs.USFGAN_DATA["hop_size"]
    sine_noise = r.standard_normal((1, 1, L)).astype(np.float32)
    noise = r.standard_normal((1, 1, L)).astype(np.float32)
    cap = {}
    orig = gen.forward

    def capture(x, c, d):
        out = orig(x, c, d)
        cap.update(x=x, c=c, d=d, out=out)
        return out
    gen.forward = capture
    wcfg = _AttrDict(data=_AttrDict(configs.USFGAN_DATA),
                     generator=_AttrDict(aux_context_window=2))
    wrapper = RefWrapper(wcfg, gen)
    with torch.no_grad(), inject_diffusion(normals=[T_(sine_noise), T_(noise)]):
        y = wrapper.inference(f0.copy(), T_(aux))
    x_out, s, h, n, a = cap["out"]
    assert torch.equal(y, x_out)
    # the reference loads vocoders with remove_weight_norm() (nnsvs/util.py:412-414)
    gen.forward = orig
    gen.remove_weight_norm()
    with torch.no_grad():
        y_rwn = gen(cap["x"], cap["c"], cap["d"])[0]
    save("usfgan", dict(f0=f0, aux=aux, sine_noise=sine_noise, noise=noise,
                        x=cap["x"].numpy(), c=cap["c"].numpy(), d=cap["d"].numpy(),
                        y=y.numpy(), s=s.numpy(), h=h.numpy(), n=n.numpy(),
                        a4=a[:, :4].numpy(), y_rwn=y_rwn.numpy()),
         dict(shapes={k: list(v) for k, v in shapes.items()}))


def case_pd_index():
    """Bit-exact pitch-dependent indexing (usfgan/utils/index.py:12-54) and dilated factors
    (features.py:56-75) over 10 s at 48 kHz: source sample per (dilation, sample)."""
    from nnsvs.usfgan.utils import dilated_factor as ref_df, index_initial, pd_indexing
    r = rng_for("pd_index")
    T, hop = 2000, configs.USFGAN_DATA["hop_size"]
    L = T * hop
    f0 = r.uniform(70.0, 1100.0, size=T).astype(np.float32)
    f0[r.random(T) < 0.2] = 0.0
    df = ref_df(f0.copy(), 48000, 4).repeat(hop, axis=0)
    d = torch.FloatTensor(df).view(1, 1, -1)
    x = torch.arange(1, L + 1, dtype=torch.float32).view(1, 1, L)  # value = sample + 1
    bi, ci = index_initial(1, 1)
    arrays = dict(f0=f0, d=d.numpy().reshape(-1))
    n1 = np.arange(1, L + 1, dtype=np.int64)
    for dil in (1, 2, 4, 8, 16):
        xP, xF = pd_indexing(x, d, dil, bi, ci)
        # stored as offsets from the sample itself (runs of equal values compress)
        arrays[f"offP{dil}"] = (n1 - xP.numpy().reshape(-1).astype(np.int64)).astype(np.int32)
        arrays[f"offF{dil}"] = (xF.numpy().reshape(-1).astype(np.int64) - n1).astype(np.int32)
    save("usfgan_pd_index", arrays, dict(T=T, hop=hop))


def case_mdn():
    """nnsvs/mdn.py on a (G, D, dim_wise) grid (loss without reduction, its input gradients,
    most-probable selection) and nnsvs.model.MDN with the reference's own fixture weights
    tests/data/mdn_test.pth (mdn_test.yaml: in 331, hidden 4, out 1, G 1; BASELINE config 1)."""
    from nnsvs import mdn as ref_mdn
    from nnsvs.model import MDN as RefMDN
    r = rng_for("mdn")
    arrays, meta = {}, {"grid": []}
    B, T = 2, 23
    for G, D, dw in ((1, 1, False), (4, 1, False), (4, 3, False), (4, 3, True), (30, 1, False)):
        key = f"G{G}D{D}{'w' if dw else ''}"
        raw = r.standard_normal((B, T, G, D) if dw else (B, T, G)).astype(np.float32) * 3
        lp = TF.log_softmax(T_(raw), dim=2)
        ls = T_(r.uniform(-8.0, 1.0, (B, T, G, D)).astype(np.float32))  # hits the -7 clamp
        mu = T_(r.standard_normal((B, T, G, D)).astype(np.float32))
        tgt = r.standard_normal((B, T, D)).astype(np.float32)
        tgt[:, ::5] *= 40.0  # far targets: the +-5 sigma clip
        lp_, ls_, mu_ = (t.clone().requires_grad_() for t in (lp, ls, mu))
        loss = ref_mdn.mdn_loss(lp_, ls_, mu_, T_(tgt), reduce=False)
        R = r.standard_normal(tuple(loss.shape)).astype(np.float32)
        (loss * T_(R)).sum().backward()
        sig, m = ref_mdn.mdn_get_most_probable_sigma_and_mu(lp, ls, mu)
        red = ref_mdn.mdn_loss(lp, ls, mu, T_(tgt), reduce=True)
        for k, v in dict(lp=lp, ls=ls, mu=mu, tgt=tgt, R=R, loss=loss, d_lp=lp_.grad,
                         d_ls=ls_.grad, d_mu=mu_.grad, sigma=sig, mu_best=m, loss_red=red).items():
            arrays[f"{key}::{k}"] = v.detach().numpy() if torch.is_tensor(v) else v
        meta["grid"].append([key, G, D, dw])
    # BASELINE config 1: the reference's MDN fixture weights
    ck = torch.load("/root/reference/tests/data/mdn_test.pth", map_location="cpu",
                    weights_only=True)
    model = RefMDN(in_dim=331, hidden_dim=4, out_dim=1, num_layers=1, num_gaussians=1)
    model.load_state_dict(ck["state_dict"])
    x = r.random((2, 50, 331)).astype(np.float32)
    y = r.standard_normal((2, 50, 1)).astype(np.float32)
    lp, ls, mu = model(T_(x))
    loss = ref_mdn.mdn_loss(lp, ls, mu, T_(y)).mean()
    loss.backward()
    for k, v in model.state_dict().items():
        arrays["mdn_test::" + k] = v.numpy()
    for k, p in model.named_parameters():
        arrays["mdn_test::grad::" + k] = p.grad.numpy()
    with torch.no_grad():
        mu_i, sig_i = model.inference(T_(x))
    arrays.update({"mdn_test::x": x, "mdn_test::y": y, "mdn_test::lp": lp.detach().numpy(),
                   "mdn_test::ls": ls.detach().numpy(), "mdn_test::mu": mu.detach().numpy(),
                   "mdn_test::loss": loss.detach().numpy(), "mdn_test::inf_mu": mu_i.numpy(),
                   "mdn_test::inf_sigma": sig_i.numpy()})
    save("mdn", arrays, meta)


def case_vp():
    """MultiTrackVariancePredictor, the recipe's duration and time-lag models
    (conf/train/{duration,timelag}/model/multitrack_*_vp_mdn.yaml): eval forward, and a
    training forward with the nn.Dropout keep masks injected + masked MDN loss + backward."""
    from nnsvs import mdn as ref_mdn
    from nnsvs.model import MultiTrackVariancePredictor as RefVP
    arrays, meta = {}, {}
    for name, hid, nl, k in (("duration", 256, 5, 5), ("timelag", 32, 3, 3)):
        cfg = dict(in_dim=82, out_dim=1, hidden_dim=hid, num_layers=nl, kernel_size=k,
                   dropout=0.5, use_mdn=True, num_gaussians=4, init_type="kaiming_normal",
                   num_speaker=3, spk_embed_dim=16)
        torch.manual_seed(0)
        model = RefVP(**cfg)
        shapes = {kk: tuple(v.shape) for kk, v in model.state_dict().items()}
        model.load_state_dict({kk: torch.from_numpy(v) for kk, v in
                               seeded_state_dict(shapes, SEED).items()})
        r = rng_for("vp_" + name)
        B, T = 2, 37
        x = r.random((B, T, 164)).astype(np.float32)
        s0 = r.integers(0, 3, size=(B, 1)).astype(np.int64)
        s1 = r.integers(0, 3, size=(B, 1)).astype(np.int64)
        y = r.standard_normal((B, T, 1)).astype(np.float32)
        lengths = np.array([37, 30], dtype=np.int64)
        model.eval()
        with torch.no_grad():
            ev = model(T_(x), (T_(s0), T_(s1)))
            inf_mu, inf_sig = model.inference(T_(x), (T_(s0), T_(s1)))
        model.train()
        masks = [(r.random((B, hid, T)) > 0.5).astype(np.float32) * 2.0 for _ in range(nl)]
        for i, blk in enumerate(model.conv):
            blk[3].forward = (lambda m: (lambda t: t * m))(T_(masks[i]))
        lp, ls, mu = model(T_(x), (T_(s0), T_(s1)))
        mask = torch.arange(T)[None, :] < T_(lengths)[:, None]
        loss = ref_mdn.mdn_loss(lp, ls, mu, T_(y), reduce=False).masked_select(mask).mean()
        model.zero_grad()
        loss.backward()
        p = name + "::"
        arrays.update({p + "x": x, p + "s0": s0, p + "s1": s1, p + "y": y, p + "lengths": lengths,
                       p + "eval_lp": ev[0].numpy(), p + "eval_ls": ev[1].numpy(),
                       p + "eval_mu": ev[2].numpy(), p + "inf_mu": inf_mu.numpy(),
                       p + "inf_sigma": inf_sig.numpy(), p + "loss": loss.detach().numpy()})
        for i, m in enumerate(masks):
            arrays[p + f"mask{i}"] = m
        for kk, prm in model.named_parameters():
            if prm.numel() <= 20000:  # large conv weights: summary only (fixture size)
                arrays[p + "grad::" + kk] = prm.grad.numpy()
        meta[name] = dict(cfg=cfg, shapes={kk: list(v) for kk, v in shapes.items()},
                          grad_summary=grad_summary(model))
    save("variance_predictor", arrays, meta)


TRANSFORMER_CASES = (
    # name, constructor kwargs, B, T, lengths
    ("base", dict(in_dim=20, out_dim=5, hidden_dim=16, attention_dim=24, num_heads=2,
                  num_layers=2, kernel_size=3, dropout=0.0), 2, 37, [37, 30]),
    ("embed", dict(in_dim=20, out_dim=3, hidden_dim=16, attention_dim=12, num_heads=4,
                   num_layers=1, kernel_size=1, dropout=0.0, embed_dim=8, in_ph_start_idx=2,
                   in_ph_end_idx=12), 3, 29, [29, 17, 5]),
    ("rf4_stride", dict(in_dim=12, out_dim=4, hidden_dim=32, attention_dim=40, num_heads=2,
                        num_layers=2, kernel_size=4, dropout=0.0, reduction_factor=4), 2, 70,
     [70, 45]),
    ("rf2_conv", dict(in_dim=12, out_dim=4, hidden_dim=16, attention_dim=16, num_heads=1,
                      num_layers=1, kernel_size=3, dropout=0.0, reduction_factor=2,
                      downsample_by_conv=True), 2, 41, [41, 20]),
    ("short", dict(in_dim=6, out_dim=2, hidden_dim=8, attention_dim=8, num_heads=2,
                   num_layers=1, kernel_size=3, dropout=0.0), 2, 3, [3, 2]),
)


def case_transformer():
    """nnsvs.model.TransformerEncoder (model.py:1540-1671; transformer/encoder.py,
    attentions.py) on ragged batches: phoneme embedding, reduction factor (stride and conv
    downsampling), even FFN kernel (asymmetric "same" padding), T below the relative window.
    Training-mode forward (dropout 0) + backward of sum(out * R): output, input grad and every
    parameter grad."""
    from nnsvs.model import TransformerEncoder as RefTE
    arrays, meta = {}, {}
    for name, cfg, B, T, lengths in TRANSFORMER_CASES:
        torch.manual_seed(0)
        model = RefTE(**cfg)
        shapes = {k: tuple(v.shape) for k, v in model.state_dict().items()}
        model.load_state_dict({k: torch.from_numpy(v) for k, v in
                               seeded_state_dict(shapes, SEED).items()})
        r = rng_for("transformer_" + name)
        x = r.standard_normal((B, T, cfg["in_dim"])).astype(np.float32)
        if cfg.get("embed_dim"):
            p0, p1 = cfg["in_ph_start_idx"], cfg["in_ph_end_idx"]
            x[:, :, p0:p1] = 0.0
            ids = r.integers(0, p1 - p0, size=(B, T))
            for b in range(B):
                x[b, np.arange(T), p0 + ids[b]] = 1.0
        model.train()
        xt = T_(x).requires_grad_()
        out = model(xt, T_(np.array(lengths, dtype=np.int64)))
        R = r.standard_normal(tuple(out.shape)).astype(np.float32)
        (out * T_(R)).sum().backward()
        p = name + "::"
        arrays.update({p + "x": x, p + "R": R, p + "out": out.detach().numpy(),
                       p + "dx": xt.grad.numpy(), p + "lengths": np.array(lengths)})
        for k, prm in model.named_parameters():
            arrays[p + "grad::" + k] = prm.grad.numpy()
        model.eval()
        with torch.no_grad():
            arrays[p + "eval_out"] = model(T_(x), T_(np.array(lengths, dtype=np.int64))).numpy()
        meta[name] = dict(cfg=cfg, B=B, T=T, shapes={k: list(v) for k, v in shapes.items()})
    save("transformer", arrays, meta)


POSTPROCESS_CASES = (
    # name, T, note fraction, voiced fraction
    ("song", 1500, 0.8, 0.7),
    ("short", 15, 1.0, 0.6),      # below lowpass_filter's length guard (18)
    ("edge", 19, 0.5, 0.5),       # just above it
    ("unvoiced", 300, 0.6, 0.0),  # no voiced frame: interp1d returns its input
    ("nonote", 240, 0.0, 0.8),    # no note frame: variance_scaling returns its input
)


def case_postprocess():
    """postprocess_acoustic (gen.py:1314-1530) with the recipe's synthesis settings
    (conf/synthesis/synthesis/world_gv_usfgan.yaml: gv post-filter, trajectory smoothing
    50 / 20 Hz, vuv_threshold 0.3, relative_f0 false).  Absent dependencies patched in:
    the frame-level linguistic features are given (fe.linguistic_features returns them;
    only the score-pitch column is read) and nnmnkwii's interp1d is the oracle's restatement
    (parity of that piece unpinned)."""
    import re
    import nnsvs.gen as ref_gen
    from oracle import postprocess_oracle as PO
    arrays, meta = {}, {"cases": []}
    cfg = types.SimpleNamespace(stream_sizes=[60, 1, 1, 5],
                                has_dynamic_features=[False, False, False, False],
                                num_windows=1)
    r = rng_for("postprocess")
    gv = (0.02 + r.random(67)) ** 2
    scaler = types.SimpleNamespace(var_=gv)
    numeric_dict = {0: ("e1", re.compile(r"/E:(\d+)"))}
    saved = (ref_gen.fe, ref_gen.interp1d)
    try:
        ref_gen.interp1d = PO.interp1d
        for name, T, note_frac, voiced_frac in POSTPROCESS_CASES:
            runs = lambda frac: np.repeat(r.random(T // 10 + 1) < frac, 10)[:T]  # noqa: E731
            score = np.where(runs(note_frac), r.integers(55, 80, size=T), 0).astype(np.float32)
            x = np.empty((T, 67), dtype=np.float32)
            x[:, :60] = (r.standard_normal((T, 60)) * np.linspace(2.0, 0.1, 60)).astype(
                np.float32) + np.cumsum(r.standard_normal((T, 1)), 0).astype(np.float32) * .05
            x[:, 60] = (5.5 + 0.3 * np.sin(np.arange(T) / 17.0) + 0.05 * r.standard_normal(T))
            x[:, 61] = np.where(runs(voiced_frac), 0.5 + 0.5 * r.random(T), 0.3 * r.random(T))
            x[:, 62:] = (-25.0 + 30.0 * r.standard_normal((T, 5))).astype(np.float32)
            ling = score[:, None].copy()
            ref_gen.fe = types.SimpleNamespace(linguistic_features=lambda *a, **k: ling)
            out = ref_gen.postprocess_acoustic(
                "cpu", x.copy(), None, {}, numeric_dict, cfg, scaler, sample_rate=48000,
                frame_period=5, relative_f0=False, feature_type="world", post_filter_type="gv",
                trajectory_smoothing=True, trajectory_smoothing_cutoff=50,
                trajectory_smoothing_cutoff_f0=20, vuv_threshold=0.3, f0_shift_in_cent=0,
                vibrato_scale=1.0, force_fix_vuv=False)
            p = name + "::"
            arrays.update({p + "x": x, p + "score": score})
            for k, v in zip(("mgc", "lf0", "vuv", "bap"), out):
                arrays[p + k] = np.asarray(v)
            meta["cases"].append(name)
    finally:
        ref_gen.fe, ref_gen.interp1d = saved
    arrays["gv"] = gv
    save("postprocess", arrays, meta)


def case_onset_merge():
    """Timing-path onset merge (collate_fn_syncmultitrack, train_util.py:776-934): two
    tracks' note rows aligned by onset time, with ties, empty overlaps and ragged ends
    (bit-exact)."""
    r = rng_for("onset_merge")
    arrays, meta = {}, {"cases": []}
    for rf in (1, 4):
        batch = []
        for i in range(4):
            n0, n1 = int(r.integers(5, 30)), int(r.integers(5, 30))
            # onsets on a coarse grid so that ties are frequent; sorted, distinct per track
            a = np.sort(r.choice(np.arange(0, 80), size=n0, replace=False)) * 50000
            b = np.sort(r.choice(np.arange(0, 80), size=n1, replace=False)) * 50000
            x0 = r.standard_normal((n0, 7)).astype(np.float32)
            y0 = r.standard_normal((n0, 2)).astype(np.float32)
            x1 = r.standard_normal((n1, 7)).astype(np.float32)
            y1 = r.standard_normal((n1, 2)).astype(np.float32)
            s0, s1 = int(r.integers(0, 3)), int(r.integers(0, 3))
            batch.append((x0, y0, s0, a, x1, y1, s1, b))
            key = f"rf{rf}_in{i}"
            for k, v in dict(x0=x0, y0=y0, a=a, x1=x1, y1=y1, b=b).items():
                arrays[f"{key}::{k}"] = v
            arrays[f"{key}::spk"] = np.array([s0, s1])
        out = ref_train_util.collate_fn_syncmultitrack(
            [tuple(x) for x in batch], reduction_factor=rf)
        for j, o in enumerate(out):
            arrays[f"rf{rf}::out{j}"] = o.numpy()
        meta["cases"].append(rf)
    save("onset_merge", arrays, meta)



def case_loader():
    from golden_util import loader_tree
    """On-disk pair dataset (train_util.py:103-246, 439-520): file discovery and pairing,
    SyncMultiTrackDataset items, shuffled ordered_indices, batch_by_size at several
    world sizes and max_tokens, and the collate of a loaded batch (bit-exact)."""
    r = rng_for("loader")
    arrays, meta = {}, {}
    spk_list = ["S1", "A2", "Vo1", "ritsu"]
    for spk in spk_list:
        for seg in ("songA_001", "songA_002", "songB_010", "x_y"):
            if (spk, seg) in (("A2", "songA_002"), ("ritsu", "x_y")):
                continue
            utt = f"{spk}_{seg}"
            n = int(r.integers(30, 220))
            arrays[f"file::in::{utt}"] = r.standard_normal((n, 6)).astype(np.float32)
            arrays[f"file::out::{utt}"] = r.standard_normal((n, 4)).astype(np.float32)
            arrays[f"file::times::{utt}"] = np.sort(r.integers(0, 10**7, size=int(r.integers(3, 12))))
    meta["spk_list"] = spk_list
    with tempfile.TemporaryDirectory() as d:
        dirs = loader_tree(d, arrays)
        in_files, lengths = ref_train_util.get_filtered_files_multitrack(dirs["in"], None)
        out_files, _ = ref_train_util.get_filtered_files_multitrack(dirs["out"], None)
        rel_ = lambda p: os.path.relpath(p, d)  # noqa: E731
        meta["in_pairs"] = [[rel_(a), rel_(b)] for a, b in in_files]
        meta["out_pairs"] = [[rel_(a), rel_(b)] for a, b in out_files]
        meta["lengths"] = [[int(a), int(b)] for a, b in lengths]
        ds = ref_train_util.SyncMultiTrackDataset(in_files, out_files, lengths, spk_list,
                                                  shuffle=True, allow_cache=False)
        meta["items"] = []
        for i in range(len(in_files)):
            it = ds[i]
            meta["items"].append([int(it[2]), int(it[6]), len(it[3]), len(it[7])])
            arrays[f"item{i}::times0"] = np.asarray(it[3])
            arrays[f"item{i}::times1"] = np.asarray(it[7])
        meta["orders"], meta["batches"] = {}, {}
        for seed in (0, 7):
            np.random.seed(seed)
            idx = ds.ordered_indices()
            meta["orders"][str(seed)] = [int(i) for i in idx]
            for mt in (250, 700, 2000):
                for w in (1, 2, 3):
                    b = ref_train_util.batch_by_size(idx, ds.num_tokens, max_tokens=mt,
                                                     required_batch_size_multiple=w)
                    meta["batches"][f"{seed}/{mt}/{w}"] = [[int(i) for i in x] for x in b]
        big = meta["batches"]["7/700/1"][0]
        out = ref_train_util.collate_fn_syncmultitrack_acoustic([ds[i] for i in big],
                                                                reduction_factor=4)
        meta["collate_batch"] = [int(i) for i in big]
        for j, o in enumerate(out):
            arrays[f"collate{j}"] = o.numpy()
    save("loader", arrays, meta)


def main():
    which = sys.argv[1:] or ["all"]
    run = lambda n: "all" in which or n in which  # noqa: E731
    full = lambda: build_ref(configs.multitrack_diffusion(num_speakers=4))[0]  # noqa: E731
    # every case starts from freshly seeded parameters (BatchNorm running stats!)
    if run("model"):
        case_model_forward_full()
    if run("diffnet"):
        case_diffnet(full(), "mgc", 2, 64, ["input_projection.weight",
                                            "residual_layers.19.output_projection.weight",
                                            "residual_layers.3.conditioner_projection.weight"])
        case_diffnet(full(), "bap", 2, 257, ["residual_layers.0.dilated_conv.weight",
                                             "skip_projection.weight", "mlp.0.weight"])
    if run("ffconvlstm"):
        for w in ("mgc", "bap", "vuv"):
            case_ffconvlstm(full(), w, 3, 64, [64, 52, 40])
    if run("lf0"):
        case_lf0(full(), 2, 64, [64, 56])
    if run("inference"):
        case_inference_bap(full())
    if run("tiny"):
        case_train_step_tiny()
    if run("tiny_il"):
        case_train_step_tiny(logf0_diff_weight=0.5, name="train_step_tiny_il")
    if run("full_train"):
        case_train_step_full()
    if run("prod_train"):
        case_train_step_full(P=2, T=1024, lengths=(1024, 900), name="train_step_prod")
    if run("inference_tiny"):
        case_model_inference_tiny()
    if run("st"):
        case_st_forward_full()
        case_st_train_tiny()
        case_st_inference_tiny()
    if run("timing_inf"):
        case_timing_inference()
    if run("data"):
        case_data_path()
    if run("usfgan"):
        case_usfgan()
    if run("pd_index"):
        case_pd_index()
    if run("mdn"):
        case_mdn()
    if run("vp"):
        case_vp()
    if run("transformer"):
        case_transformer()
    if run("postprocess"):
        case_postprocess()
    if run("onset"):
        case_onset_merge()
    if run("loader"):
        case_loader()
    if run("sf0"):
        case_sf0_forward(True, 3, 40, [40, 33, 21], "sf0_forward_tiny")
        case_sf0_forward(False, 2, 32, [32, 28], "sf0_forward_full")
        case_sf0_train_tiny()
        case_sf0_inference_tiny()
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(dict(seed=SEED, torch=torch.__version__, numpy=np.__version__,
                       reference="sarulab-speech/ensemble_svs_with_interactions @ 2025-03-21",
                       files=sorted(x for x in os.listdir(HERE) if x.endswith(".npz"))),
                  f, indent=1)


if __name__ == "__main__":
    main()
