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


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_skip_gemm_matches_blockwise_skip(precision):
    """Training forward: the skip sum of all blocks as one K = L*C GEMM after the blocks and
    residual-only block projections (diffsinger.SKIP_GEMM) against the skip half in every
    block's RESSKIP epilogue (the inference form).  fp32: the same skip sum, outputs and
    gradients to 1e-5 (max-abs relative).  bf16: the residual weights are rounded after their
    1/sqrt2 pre-scale, and the backward through 20 bf16 blocks amplifies that as it does any
    rounding (d_cond is 5.6 % rel-L2 from the fp32 reference; the two forms measured S 0.3 %,
    out 0.4 %, d_cond 5.4 % apart): rel-L2 bounds at the bf16 test's level."""
    from ensemble_svs_with_interactions_amd import diffsinger
    res = []
    for on in (True, False):
        diffsinger.SKIP_GEMM["on"] = on
        try:
            _, _, _, mod, _, st, out, _, dcond = _run("mgc", precision)
        finally:
            diffsinger.SKIP_GEMM["on"] = True
        res.append((st["S"].cpu(), out, dcond,
                    {k: p.grad.cpu().clone() for k, p in mod.named_parameters()}))
    engine.set_gemm_precision("fp32")
    if precision == "fp32":
        for i, name in enumerate(("S", "out", "dcond")):
            assert rel(res[0][i], res[1][i]) < 1e-5, name
        for k, g in res[0][3].items():
            assert rel(g, res[1][3][k]) < 1e-4, k
        return
    errs = {name: rel_l2(res[0][i], res[1][i]) for i, name in enumerate(("S", "out", "dcond"))}
    print("bf16 skip GEMM vs blockwise skip, rel-L2:", errs)
    assert errs["S"] < 1e-2 and errs["out"] < 1e-2 and errs["dcond"] < 1.5e-1, errs
    gerr = {k: rel_l2(g, res[1][3][k]) for k, g in res[0][3].items()}
    print("parameter gradients, largest rel-L2:", max(gerr.items(), key=lambda kv: kv[1]))
    for k, e in gerr.items():
        assert e < 1.5e-1, (k, e)
