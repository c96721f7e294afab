"""uSFGAN vocoder on MI355X vs the reference goldens.

Goldens: tests/golden/usfgan.npz (generator forward + USFGANWrapper.inference of the
reference, 40 frames = 9 600 samples, weight norm on; remove_weight_norm output) and
usfgan_pd_index.npz (reference pd_indexing / dilated_factor over 10 s at 48 kHz).
Tolerances: index and dilation-factor arithmetic bit-exact; fp32 GEMM path rel 1e-4
(max-abs relative) against the reference outputs.
"""
import numpy as np
import pytest
import torch

from ensemble_svs_with_interactions_amd import _lib, configs, engine
from ensemble_svs_with_interactions_amd import kernels as K
from ensemble_svs_with_interactions_amd import usfgan
from ensemble_svs_with_interactions_amd.usfgan import USFGANWrapper
from golden_util import load_case, params_from_shapes, rel, rel_l2

pytestmark = pytest.mark.gpu


def _gen(meta, weight_norm=True):
    gen = configs.instantiate(configs.usfgan_generator())
    gen.load_state_dict(params_from_shapes(meta["shapes"]))
    return gen.cuda()


def _wrapper(gen):
    return USFGANWrapper({"data": dict(configs.USFGAN_DATA),
                          "generator": {"aux_context_window": 2}}, gen)


def test_dilated_factor_bitexact():
    a, meta = load_case("usfgan_pd_index")
    T, hop = meta["T"], meta["hop"]
    f0 = torch.from_numpy(a["f0"]).cuda()
    d = torch.empty(T * hop, device="cuda")
    _lib.call("ensvs_usf_dfactor", f0.data_ptr(), 1, T, hop, 48000.0, 4.0, d.data_ptr(),
              torch.cuda.current_stream().cuda_stream)
    assert torch.equal(d.cpu(), torch.from_numpy(a["d"]))


def test_pd_gather_bitexact():
    """The GEMM engine's pitch-dependent segment gathers exactly the reference's past /
    current / future samples (identity weights, exact fp32 MFMA, x = sample index + 1)."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("usfgan_pd_index")
    L = meta["T"] * meta["hop"]
    d = torch.from_numpy(a["d"]).cuda()
    x = torch.zeros(L, 4, device="cuda")
    x[:, 0] = torch.arange(1, L + 1, dtype=torch.float32, device="cuda")
    w = torch.zeros(3, 4, 3, device="cuda")  # output n = tap n of channel 0
    for n in range(3):
        w[n, 0, n] = 1.0
    pb = K.PackedBuffer(_lib.DT_F32)
    ref = pb.add(w, 3, 4, 3, 12, 3, 1)
    pb.finalize("cuda")
    pb.repack()
    n1 = np.arange(1, L + 1, dtype=np.int64)
    for dil in (1, 2, 4, 8, 16):
        y = torch.full((L, 3), -1.0, device="cuda")
        K.gemm([K.Seg(x, 4, 4, ref, L, taps=3, pd=d, pd_dil=dil)], 1, L, 3, pb, y, 3)
        y = y.cpu().numpy().astype(np.int64)
        assert np.array_equal(n1 - y[:, 0], a[f"offP{dil}"]), dil
        assert np.array_equal(y[:, 1], n1)
        assert np.array_equal(y[:, 2] - n1, a[f"offF{dil}"]), dil


def test_generator_forward_matches_reference():
    engine.set_gemm_precision("fp32")
    a, meta = load_case("usfgan")
    gen = _gen(meta)
    g = lambda k: torch.from_numpy(a[k]).cuda()  # noqa: E731
    y, s, h, n, av = gen(g("x"), g("c"), g("d"))
    torch.cuda.synchronize()
    for k, v in dict(y=y, s=s, h=h, n=n).items():
        assert rel(v.cpu(), a[k]) < 1e-4, k
    assert rel(av[:, :4].cpu(), a["a4"]) < 1e-5


def test_wrapper_inference_matches_reference():
    """USFGANWrapper.inference: dilated factors, sine/noise source (fp64 phase scan) and the
    generator, replaying the reference's two N(0, 1) draws."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("usfgan")
    gen = _gen(meta)
    wr = _wrapper(gen)
    noises = (torch.from_numpy(a["sine_noise"]).cuda(), torch.from_numpy(a["noise"]).cuda())
    xsrc, d, L = wr._sources(torch.from_numpy(a["f0"]).cuda().view(-1), 1, a["f0"].shape[0],
                             noises)
    torch.cuda.synchronize()
    assert torch.equal(d.cpu(), torch.from_numpy(a["d"]).view(-1))
    ref_x = torch.from_numpy(a["x"])[0].t()
    assert (xsrc.cpu() - ref_x).abs().max().item() < 1e-5
    y = wr.inference(a["f0"], torch.from_numpy(a["aux"]), noises=noises)
    torch.cuda.synchronize()
    assert tuple(y.shape) == a["y"].shape
    assert rel(y.cpu(), a["y"]) < 1e-4


def test_remove_weight_norm_matches_reference():
    engine.set_gemm_precision("fp32")
    a, meta = load_case("usfgan")
    gen = _gen(meta)
    gen.remove_weight_norm()
    keys = list(gen.state_dict())
    assert not any(k.endswith("weight_g") or k.endswith("weight_v") for k in keys)
    g = lambda k: torch.from_numpy(a[k]).cuda()  # noqa: E731
    y = gen(g("x"), g("c"), g("d"))[0]
    assert rel(y.cpu(), a["y_rwn"]) < 1e-4


def test_batched_synthesis_equals_single():
    """inference_batch over B tracks = B single-track inferences (same draws)."""
    engine.set_gemm_precision("fp32")
    a, meta = load_case("usfgan")
    gen = _gen(meta)
    wr = _wrapper(gen)
    f0 = torch.from_numpy(a["f0"]).cuda().view(1, -1)
    f0b = torch.cat([f0, f0 * 1.25], 0)
    aux = torch.from_numpy(a["aux"]).cuda()
    auxb = torch.stack([aux, aux.flip(0)])
    L = f0.shape[1] * 240
    g = torch.Generator(device="cuda").manual_seed(3)
    nz = [torch.randn(2, L, device="cuda", generator=g) for _ in range(2)]
    yb = wr.inference_batch(f0b, auxb, noises=nz)
    for b in range(2):
        yi = wr.inference(f0b[b].cpu().numpy(), auxb[b], noises=(nz[0][b], nz[1][b]))
        assert rel(yb[b].cpu(), yi[0].cpu()) < 1e-5


def test_bf16_generator():
    """Production precision (bf16 MFMA operands, fp32 accumulate): error recorded."""
    engine.set_gemm_precision("bf16")
    try:
        a, meta = load_case("usfgan")
        gen = _gen(meta)
        g = lambda k: torch.from_numpy(a[k]).cuda()  # noqa: E731
        y = gen(g("x"), g("c"), g("d"))[0]
        e = rel_l2(y.cpu(), a["y"])
        print(f"bf16 uSFGAN waveform rel-L2 {e:.3e}")
        assert e < 5e-2
    finally:
        engine.set_gemm_precision("fp32")


def test_bf16_operand_copies_bitwise():
    """Inference on bf16 operand copies (the residual streams' copies from the output-GEMM
    epilogues, the zero-padded auxiliary features rounded once, z in bf16 only, the
    pitch-dependent gather on the bf16 copy), with two GEMMs per block and with the fused
    one-launch block, = the register-staged kernels that round the fp32 operands while
    staging: identical waveform bits, full-size generator (bench config), two tracks."""
    engine.set_gemm_precision("bf16")
    saved = dict(K.BF16_ACT)
    try:
        torch.manual_seed(9)
        gen = configs.instantiate(configs.usfgan_generator()).cuda()
        gen.remove_weight_norm()
        wr = USFGANWrapper({"data": dict(configs.USFGAN_DATA),
                            "generator": {"aux_context_window": 2}}, gen)
        T = 60
        f0 = 150.0 + 100.0 * torch.rand(2, T, device="cuda")
        f0[:, 10:14] = 0.0  # unvoiced frames
        aux = torch.randn(2, T, gen.aux_channels, device="cuda")
        L = T * 240
        g = torch.Generator(device="cuda").manual_seed(4)
        nz = [torch.randn(2, L, device="cuda", generator=g) for _ in range(2)]
        outs = []
        for on, fused in ((False, False), (True, False), (True, True)):
            K.BF16_ACT.update(on=on)
            usfgan.FUSED_BLOCK["on"] = fused
            outs.append(wr.inference_batch(f0, aux, noises=nz))
            torch.cuda.synchronize()
        assert torch.isfinite(outs[2]).all()
        assert torch.equal(outs[0], outs[1])  # bf16 operand copies, two GEMMs per block
        assert torch.equal(outs[0], outs[2])  # one launch per block (ensvs_usf_block)
    finally:
        K.BF16_ACT.clear()
        K.BF16_ACT.update(saved)
        usfgan.FUSED_BLOCK["on"] = True
        engine.set_gemm_precision("fp32")
