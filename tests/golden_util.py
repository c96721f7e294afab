"""Loading helpers for the reference-generated fixtures in tests/golden/."""
import json
import os

import numpy as np
import torch

from oracle import ensvs_oracle as O
from oracle.weights import seeded_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
SEED = 20250321


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    arrays = {k: z[k] for k in z.files if k != "meta_json"}
    meta = json.loads(bytes(z["meta_json"]).decode())
    return arrays, meta


def full_shapes():
    return load_case("model_forward_full")[1]["shapes"]


def tiny_shapes():
    return load_case("train_step_tiny")[1]["shapes"]


def params_from_shapes(shapes, seed=SEED, requires_grad=False):
    """Seeded parameters + diffusion schedule buffers, as torch tensors."""
    sd = seeded_state_dict(shapes, seed)
    P = {k: torch.from_numpy(v.copy()) for k, v in sd.items()}
    for prefix in ("mgc_model.", "bap_model."):
        for k, v in O.diffusion_schedule().items():
            if prefix + k in shapes:
                P[prefix + k] = v
    if requires_grad:
        for k, v in P.items():
            if "running" not in k and v.dtype == torch.float32 and not _is_buffer(k):
                v.requires_grad_()
    return P


def _is_buffer(k):
    from oracle.weights import SCHEDULE_BUFFERS
    return k.rsplit(".", 1)[-1] in SCHEDULE_BUFFERS


def rel(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    return ((a - b).abs().max() / (b.abs().max() + 1e-30)).item()


def check_grad_summary(grads, summary, prefix, rtol=1e-4, atol=1e-7):
    """grads: {full_key: tensor}; summary: {module_key: [sum, abs, l2]} from the golden."""
    bad = []
    for k, (s, a, l2) in summary.items():
        if _pre_bn_bias(k):
            # Conv bias feeding a training-mode BatchNorm: analytically zero
            # gradient, the stored values are float cancellation noise.
            g = grads.get(prefix + k)
            w = summary[k.replace(".bias", ".weight")][2]
            if g is not None and g.double().norm().item() > 1e-5 * w + 1e-6:
                bad.append((k, "pre-BN bias grad not ~0"))
            continue
        g = grads.get(prefix + k)
        if g is None:
            gs = [0.0, 0.0, 0.0]
        else:
            g = g.double()
            gs = [g.sum().item(), g.abs().sum().item(), g.norm().item()]
        ref = [s, a, l2]
        scale = max(abs(a), atol)
        for x, y in zip(gs, ref):
            if abs(x - y) > rtol * scale + atol:
                bad.append((k, gs, ref))
                break
    return bad


def _pre_bn_bias(k):
    parts = k.split(".")
    return len(parts) >= 3 and parts[-3] == "conv" and parts[-1] == "bias" and \
        parts[-2] in ("1", "5", "9")


def rel_l2(g, ref):
    g = torch.as_tensor(g).double()
    ref = torch.as_tensor(ref).double()
    return ((g - ref).norm() / (ref.norm() + 1e-30)).item()


def sampled_grad_errors(grads, a, meta):
    """Per-parameter errors of full-width gradients against a fixture that keeps a seeded
    element sample of every reference gradient (train_step_full): {key: (sampled rel-L2,
    relative error of the exact L2 norm)}.  grads: {key: tensor} (any device)."""
    out = {}
    for k, (s, ab, l2) in meta["grad_summary"].items():
        g = grads[k].detach().reshape(-1).double().cpu()
        idx = torch.from_numpy(a["gidx::" + k].astype(np.int64))
        ref = torch.from_numpy(a["gval::" + k])
        out[k] = (rel_l2(g[idx], ref), abs(g.norm().item() - l2) / (l2 + 1e-30))
    return out


def record_errors(case, values):
    """Merge measured errors of one test case into $ENSVS_RECORD_DIR/<case>.json (nothing
    when the variable is unset): the numbers DESIGN.md section 4 quotes."""
    d = os.environ.get("ENSVS_RECORD_DIR")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, case + ".json")
    old = {}
    if os.path.exists(path):
        with open(path) as f:
            old = json.load(f)
    old.update(values)
    with open(path, "w") as f:
        json.dump(old, f, indent=1, sort_keys=True)


def grad_close(g, ref, rtol, name=None):
    """Relative L2 error of a gradient tensor (robust to isolated ReLU-kink flips); with a
    name, the measured error is recorded (record_errors("end_to_end_grads", ...))."""
    e = rel_l2(g, ref)
    if name is not None:
        record_errors("end_to_end_grads", {name: e})
    return e <= rtol

def loader_tree(root, arrays):
    """Write the on-disk dataset held in `arrays` (loader fixture) under root:
    dump/norm/{in,out}_acoustic/<utt>-feats.npy and dump/org/in_acoustic/<utt>-times.npy.
    Shared with tests/test_loader.py so both sides read byte-identical files."""
    dirs = {k: os.path.join(root, "dump", a, b) for k, a, b in
            (("in", "norm", "in_acoustic"), ("out", "norm", "out_acoustic"),
             ("times", "org", "in_acoustic"))}
    for d in dirs.values():
        os.makedirs(d, exist_ok=True)
    for key, v in arrays.items():
        if key.startswith("file::"):
            _, kind, utt = key.split("::")
            suffix = "-times.npy" if kind == "times" else "-feats.npy"
            np.save(os.path.join(dirs[kind], utt + suffix), v)
    return dirs
