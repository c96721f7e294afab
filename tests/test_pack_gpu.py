"""Weight repack: the tiled kernel (ensvs_pack_weights_tiled, one workgroup per 64 x 64 tile
through LDS) against the element-per-thread kernel (ensvs_pack_weights) -- the same bits in
every packed operand of the production model (linear / conv / flipped transposed conv /
16-interleaved DiffNet gates with a second bias source / row- and column-concatenations with
their own row strides) and in synthetic descriptors with ragged sizes, odd strides, fp32
destinations and scale factors.  Both are pure data movement (source, + second source, x
scale, one rounding), so the bar is bitwise."""
import pytest
import torch

from ensemble_svs_with_interactions_amd import _lib, configs, kernels as K

pytestmark = pytest.mark.gpu


def _both(pb):
    """(element-per-thread, tiled) packed buffers of one PackedBuffer."""
    out = []
    for tiled in (False, True):
        pb.buf.fill_(float("nan"))
        K.PACK_TILED["on"] = tiled
        try:
            pb.repack()
        finally:
            K.PACK_TILED["on"] = True
        torch.cuda.synchronize()
        out.append(pb.buf.clone())
    return out


def _bits(t):
    return t.view(torch.int16) if t.dtype == torch.bfloat16 else t.view(torch.int32)


def test_tiled_pack_matches_on_the_production_model():
    torch.manual_seed(3)
    dev = torch.device("cuda")
    model = configs.instantiate(configs.multitrack_diffusion(num_speakers=4)).to(dev)
    with torch.no_grad():
        for p in model.parameters():
            p.normal_(0.0, 0.05)
    checked = 0
    for name, m in model.named_modules():
        if not (hasattr(m, "_packs") and hasattr(m, "_register")):
            continue
        pk = m._packs.ensure(m, m._register)
        for tag in ("fwd", "bwd", "bias"):
            pb = getattr(pk, tag)
            if not pb._n:
                continue
            a, b = _both(pb)
            assert torch.equal(_bits(a), _bits(b)), f"{name}.{tag}"
            checked += 1
    assert checked >= 15


@pytest.mark.parametrize("dtype", [_lib.DT_BF16, _lib.DT_F32])
def test_tiled_pack_matches_on_ragged_descriptors(dtype):
    g = torch.Generator(device="cuda").manual_seed(11)
    dev = torch.device("cuda")
    pb = K.PackedBuffer(dtype)
    w1 = torch.randn(77, 45, 5, device=dev, generator=g)          # conv (N, K, taps)
    w2 = torch.randn(130, 200, device=dev, generator=g)           # linear
    w3 = torch.randn(96, 40, 3, device=dev, generator=g)          # interleaved gate conv
    b3 = torch.randn(96, 40, 3, device=dev, generator=g)
    w4 = [torch.randn(33, 70, device=dev, generator=g) for _ in range(3)]
    pb.add(w1, 77, 45, 5, 45 * 5, 5, 1)
    pb.add(w1, 77, 45, 5, 45 * 5, 5, 1, flip=True, transpose=True, scale=0.5)
    pb.add(w2, 130, 200, 1, 200, 1, 1, npad_to=1, kpad_to=1)
    pb.add(w2, 130, 200, 1, 200, 1, 1, transpose=True, scale=1.25)
    pb.add(w3, 96, 40, 3, 120, 3, 1, perm_c=48, src2=b3)
    pb.add(w2[:, 7:], 130, 193, 1, 200, 1, 1)                     # a column range (odd base)
    pb.add_rowcat(w4, 33, 70)
    pb.add_rowcat(w4, 33, 70, transpose_blocks=True)
    pb.add_colcat(w4, 33, 70, scale=0.75)
    pb.finalize(dev)
    a, b = _both(pb)
    assert torch.equal(_bits(a), _bits(b))
