"""DiffNet (DiffSinger denoiser) on MI355X vs the reference goldens and the oracle."""
import pytest
import torch

from oracle import ensvs_oracle as O
from ensemble_svs_with_interactions_amd import configs, engine
from golden_util import load_case, full_shapes, rel, grad_close, rel_l2
from gpu_util import build

pytestmark = pytest.mark.gpu
CFG = configs.multitrack_diffusion(num_speakers=4)


def _run(which, precision):
    engine.set_gemm_precision(precision)
    a, meta = load_case(f"diffnet_{which}")
    cfg = CFG[f"{which}_model"]["denoise_fn"]
    mod = build(cfg, full_shapes(), meta["prefix"])
    P0 = {k: v.detach().cpu().clone() for k, v in mod.state_dict().items()}
    B, _, Mc, T = a["spec"].shape
    E = a["cond"].shape[1]
    xin = torch.from_numpy(a["spec"])[:, 0].transpose(1, 2).contiguous().view(B * T, Mc).cuda()
    cnd = torch.from_numpy(a["cond"]).transpose(1, 2).contiguous().view(B * T, E).cuda()
    t = torch.from_numpy(a["t"]).cuda()
    out, st = mod._fwd(xin, Mc, t, cnd, E, B, T)
    R = torch.from_numpy(a["R"])[:, 0].transpose(1, 2).contiguous().view(B * T, Mc).cuda()
    dcond = mod._bwd(st, R)
    torch.cuda.synchronize()
    out_ref = torch.from_numpy(a["out"])[:, 0].transpose(1, 2)
    return a, meta, cfg, mod, P0, st, out.cpu().view(B, T, Mc), out_ref, dcond.cpu().view(B, T, E)


@pytest.mark.parametrize("which", ["mgc", "bap"])
def test_diffnet_fp32(which):
    a, meta, cfg, mod, P0, st, out, out_ref, dcond = _run(which, "fp32")
    B, T = out.shape[:2]
    assert rel(out, out_ref) < 1e-4
    # mask-matched oracle backward (tight)
    C = cfg["residual_channels"]
    masks = {"in": (st["X"][0] > 0).float().cpu().view(B, T, C).transpose(1, 2),
             "skip": (st["p1"] > 0).float().cpu().view(B, T, C).transpose(1, 2)}
    Pg = {k: v.clone().requires_grad_() for k, v in P0.items() if v.dtype == torch.float32}
    cond = torch.from_numpy(a["cond"]).requires_grad_()
    oc = O.diffnet(Pg, "", cfg, torch.from_numpy(a["spec"]), torch.from_numpy(a["t"]), cond,
                   relu_masks=masks)
    (oc * torch.from_numpy(a["R"])).sum().backward()
    assert rel(dcond.transpose(1, 2), cond.grad) < 2e-4
    for k, p in mod.named_parameters():
        assert rel(p.grad.cpu(), Pg[k].grad) < 5e-4, k
    # end-to-end vs the reference (measured 0.6e-6 .. 2.0e-6 rel-L2)
    assert grad_close(dcond.transpose(1, 2), torch.from_numpy(a["d_cond"]), 2e-5,
                      name=f"diffnet_{which}.d_cond")
    for k in a:
        if k.startswith("grad::"):
            assert grad_close(dict(mod.named_parameters())[k[6:]].grad.cpu(),
                              torch.from_numpy(a[k]), 2e-5, name=f"diffnet_{which}.{k[6:]}"), k


@pytest.mark.parametrize("which", ["mgc", "bap"])
def test_diffnet_bf16(which):
    a, meta, cfg, mod, P0, st, out, out_ref, dcond = _run(which, "bf16")
    engine.set_gemm_precision("fp32")
    # bf16 MFMA operands, fp32 accumulation (the production precision; parity is the
    # fp32 test above).  Measured relative-L2 errors are printed for the record.
    e_out = rel_l2(out, out_ref)
    e_cond = rel_l2(dcond.transpose(1, 2), torch.from_numpy(a["d_cond"]))
    print(f"bf16 {which}: out rel-L2 {e_out:.3e}, d_cond rel-L2 {e_cond:.3e}")
    assert e_out < 3e-2 and e_cond < 1.5e-1
