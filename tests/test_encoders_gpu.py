"""FFConvLSTM encoders on MI355X vs the reference (fp32 MFMA path).

Forward: max-abs relative error vs the reference goldens.
Backward: (1) tight, against the CPU oracle evaluated with the SAME ReLU
decisions as the device (mask-matched: fp32 rounding can put a pre-activation
on the other side of 0, which flips that element's gradient in any two fp32
implementations); (2) end-to-end against the reference goldens, bounded by the
measured effect of the device's ReLU decisions (oracle with vs without them).
"""
import pytest
import torch

from oracle import ensvs_oracle as O
from ensemble_svs_with_interactions_amd import configs, engine
from golden_util import load_case, full_shapes, rel, rel_l2, record_errors
from gpu_util import build

pytestmark = pytest.mark.gpu
CFG = configs.multitrack_diffusion(num_speakers=4)


def _cfg(which):
    return {"mgc": CFG["mgc_model"]["encoder"], "bap": CFG["bap_model"]["encoder"],
            "vuv": CFG["vuv_model"]}[which]


def relu_masks_from(st, B, T):
    """Device ReLU decisions of an FFConvLSTM forward (post-ReLU outputs > 0)."""
    m = {}
    for n, i in enumerate((0, 2, 4)):
        m[f"ff{i}"] = (st["hs"][n] > 0).float().cpu().view(B, T, -1)
    for li, bi in enumerate((2, 6, 10)):
        m[f"bn{bi}"] = (st["csv"][li]["out"] > 0).float().cpu().view(B, T, -1)
    return m


@pytest.mark.parametrize("which", ["mgc", "bap", "vuv"])
def test_ffconvlstm_matches_reference(which):
    engine.set_gemm_precision("fp32")
    a, meta = load_case(f"ffconvlstm_{which}")
    cfg, pre = _cfg(which), meta["prefix"]
    mod = build(cfg, full_shapes(), pre)
    mod.train()
    if which == "vuv":
        mod.lstm.dropout = 0.0  # golden captured without inter-layer dropout
    P0 = {k: v.detach().cpu().clone() for k, v in mod.state_dict().items()}
    x = torch.from_numpy(a["x"]).cuda()
    B, T = x.shape[:2]
    spk = torch.from_numpy(a["spk"]).cuda().expand(B, T, -1)
    lens = torch.tensor(a["lengths"].tolist(), device="cuda")
    out, st = mod._fwd([(x, x.shape[2], 0, x.shape[2])], B, T, lens, spk, spk.stride(0))
    R = torch.from_numpy(a["R"]).cuda().reshape(B * T, -1).contiguous()
    dX0, dspk = mod._bwd(st, R, want_spk=True)
    torch.cuda.synchronize()
    # forward vs reference
    assert rel(out.cpu().view(B, T, -1), a["out"]) < 1e-4
    sd = mod.state_dict()
    for k in a:
        if k.startswith("bn::"):
            assert rel(sd[k[4:]].cpu(), a[k]) < 1e-4, k
    # backward vs mask-matched oracle (tight)
    Pg = {k: (v.clone() if "running" in k else v.clone().requires_grad_())
          for k, v in P0.items() if v.dtype == torch.float32}
    spk_c = torch.from_numpy(a["spk"]).requires_grad_()
    oc = O.ffconvlstm(Pg, "", cfg, torch.from_numpy(a["x"]), a["lengths"],
                      spk_c.expand(B, T, -1), training=True,
                      relu_masks=relu_masks_from(st, B, T))
    (oc * torch.from_numpy(a["R"])).sum().backward()
    assert rel(dspk.cpu(), spk_c.grad.view(B, -1)) < 1e-4
    for k, p in mod.named_parameters():
        if k.endswith("bias") and k.startswith("conv.") and k.split(".")[1] in ("1", "5", "9"):
            continue  # analytically zero (conv bias before training-mode BatchNorm)
        assert rel(p.grad.cpu(), Pg[k].grad) < 2e-4, k
    # backward vs reference goldens (end-to-end).  Measured: <= 2.3e-6
    # rel-L2, except the mgc encoder's d_spk at 2.0e-2: there the device takes a different
    # ReLU decision than the reference on some element (fp32 rounding at the kink).  The
    # bound is therefore the effect of the device's decisions themselves: the oracle
    # without masks (the reference's decisions) matches the golden tightly, and the device
    # may differ from the golden by no more than the two oracle runs differ plus 2e-5.
    golden = torch.from_numpy(a["d_spk"]).view(B, -1)
    Pu = {k: (v.clone() if "running" in k else v.clone().requires_grad_())
          for k, v in P0.items() if v.dtype == torch.float32}
    spk_u = torch.from_numpy(a["spk"]).requires_grad_()
    ou = O.ffconvlstm(Pu, "", cfg, torch.from_numpy(a["x"]), a["lengths"],
                      spk_u.expand(B, T, -1), training=True)
    (ou * torch.from_numpy(a["R"])).sum().backward()
    e_oracle = rel_l2(spk_u.grad.view(B, -1), golden)
    e_decisions = rel_l2(spk_c.grad.view(B, -1), spk_u.grad.view(B, -1))
    e2e = rel_l2(dspk.cpu(), golden)
    record_errors("end_to_end_grads", {f"ffconvlstm_{which}.d_spk": e2e,
                                       f"ffconvlstm_{which}.d_spk.relu_decisions": e_decisions})
    assert e_oracle < 1e-5
    assert e2e <= e_decisions + 2e-5, (e2e, e_decisions)
