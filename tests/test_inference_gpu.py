"""Acoustic-model inference on MI355X vs the reference goldens.

* inference_bap.npz: GaussianDiffusion.inference of the bap stream (100-step reverse
  process, diffusion.py:302-336) with the reference's 101 N(0, 1) draws replayed.
* model_inference_tiny.npz: MultiTrackNPSSMDN...inference (pad_inference_multitrack,
  acoustic_models/util.py:154-188) at T = 28..31 (every T mod 4), AR-decoder dropout masks
  and diffusion draws replayed.
The HIP-graph replay of the reverse process must equal the eager launches bit for bit.
Tolerance: fp32 GEMMs, rel 1e-3 (max-abs relative) after 100 chained denoising steps.
"""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import configs, engine
from golden_util import load_case, full_shapes, rel
from gpu_util import build

pytestmark = pytest.mark.gpu


def _draws(nz, B, T):
    """(K+1, B, 1, M, T) reference draws -> (K+1, B*T, M) frame rows."""
    n = torch.from_numpy(np.ascontiguousarray(nz))[:, :, 0]
    return n.transpose(2, 3).contiguous().view(n.shape[0], B * T, -1).cuda()


def test_inference_bap_matches_reference_and_graph_is_bitwise_eager():
    engine.set_gemm_precision("fp32")
    a, _ = load_case("inference_bap")
    cfg = configs.multitrack_diffusion(num_speakers=4)["bap_model"]
    gd = build(cfg, full_shapes(), "bap_model.").eval()
    B, T, D = a["cond_in"].shape
    cond = torch.from_numpy(a["cond_in"]).cuda()
    spk = torch.from_numpy(a["spk"]).cuda().view(B, -1).contiguous()
    lens = torch.tensor(a["lengths"].tolist(), device="cuda")
    nz = _draws(a["noises"], B, T)
    src = [(cond, D, 0, D)]
    eager = gd._inference(src, B, T, lens, spk, spk.shape[1], noises=nz, graph=False)
    graph = gd._inference(src, B, T, lens, spk, spk.shape[1], noises=nz, graph=True)
    graph2 = gd._inference(src, B, T, lens, spk, spk.shape[1], noises=nz, graph=True)
    torch.cuda.synchronize()
    assert rel(eager.cpu().view(B, T, -1), a["out"]) < 1e-3
    assert torch.equal(eager, graph) and torch.equal(graph, graph2)


@pytest.mark.parametrize("T", [28, 29, 30, 31])
def test_model_inference_tiny_matches_reference(T):
    engine.set_gemm_precision("fp32")
    a, meta = load_case("model_inference_tiny")
    model = build(configs.multitrack_diffusion(num_speakers=4, tiny=True), meta["shapes"])
    model.eval()
    g = lambda k: torch.from_numpy(a[f"T{T}::{k}"]).cuda().contiguous()  # noqa: E731
    Tp = T + meta[f"T{T}"]["pad"]
    masks = torch.from_numpy(a[f"T{T}::masks"][0]).cuda().view(-1).contiguous()
    draws = dict(noises={"mgc": _draws(a[f"T{T}::noise_mgc"], 1, Tp),
                         "bap": _draws(a[f"T{T}::noise_bap"], 1, Tp)}, masks=masks)
    out = model.inference(g("x_main"), g("x_sub"), spks=(g("spk_main"), g("spk_sub")),
                          lengths=a[f"T{T}::lengths"].tolist(), draws=draws)
    torch.cuda.synchronize()
    ref = a[f"T{T}::out"]
    assert tuple(out.shape) == tuple(meta[f"T{T}"]["out_shape"])
    assert rel(out.cpu(), ref) < 1e-3
