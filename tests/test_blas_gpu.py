"""ensvs_blas_gemm (hipBLASLt plain bf16 GEMM, csrc/blas.hip) against the implicit-GEMM engine
on the same bf16 operands and packed weights: the recurrences' input projection (bias
epilogue) and the two-segment input gradient (second call accumulating), at the SeparateF0
encoder's shapes and a ragged one.  Both accumulate the same bf16 products in fp32, so they
agree to summation order (1e-5 relative of the output scale); repeated calls and a captured
graph replay give the same bits (one plan, one algorithm per shape, on data-parallel grids:
TENSILE_STREAMK_DATA_PARALLEL=1, set by the library, csrc/blas.hip)."""
import pytest
import torch

from ensemble_svs_with_interactions_amd import _lib, kernels as K

pytestmark = pytest.mark.gpu


def _pack(N, Kc, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    w = torch.randn(N, Kc, device="cuda", generator=g) * 0.03
    pb = K.PackedBuffer(_lib.DT_BF16)
    ref = pb.add(w, N, Kc, 1, Kc, 1, 1)
    pb.finalize(torch.device("cuda"))
    pb.repack()
    return pb, ref


def _close(a, b, tol=1e-5):
    return ((a.double() - b.double()).abs().max() / b.double().abs().max()).item() <= tol


@pytest.mark.parametrize("M,N,Kc,T", [(30720, 4096, 1024, 1024), (30720, 4096, 512, 1024),
                                      (8000, 1024, 520, 1000)])
def test_blas_projection_matches_engine(M, N, Kc, T):
    pb, ref = _pack(N, Kc, N + Kc)
    g = torch.Generator(device="cuda").manual_seed(M)
    x = torch.randn(M, Kc, device="cuda", generator=g).to(torch.bfloat16)
    bias = torch.randn(N, device="cuda", generator=g)
    want = torch.empty(M, N, device="cuda")
    K.gemm([K.Seg(x, Kc, Kc, ref, T)], M // T, T, N, pb, want, N, bias=bias)
    got = torch.full((M, N), float("nan"), device="cuda")
    assert K.blas_gemm(x, Kc, ref, pb, M, N, Kc, got, N, bias=bias)
    again = torch.full((M, N), float("nan"), device="cuda")
    assert K.blas_gemm(x, Kc, ref, pb, M, N, Kc, again, N, bias=bias)
    torch.cuda.synchronize()
    assert _close(got, want)
    assert torch.equal(got.view(torch.int32), again.view(torch.int32))


def test_blas_two_segment_input_gradient_and_graph():
    """nd = g[:, :4H] W0^T + g[:, 4H:] W1^T as two calls (the second with beta = 1), against the
    engine's two-segment GEMM; the same calls captured in a HIP graph replay the same bits."""
    M, H, Kc, T = 30720, 512, 1024, 1024
    pb = K.PackedBuffer(_lib.DT_BF16)
    g = torch.Generator(device="cuda").manual_seed(7)
    ws = [torch.randn(4 * H, Kc, device="cuda", generator=g) * 0.03 for _ in range(2)]
    refs = [pb.add(w, 4 * H, Kc, 1, Kc, 1, 1, transpose=True) for w in ws]
    pb.finalize(torch.device("cuda"))
    pb.repack()
    gd = torch.randn(M, 8 * H, device="cuda", generator=g).to(torch.bfloat16)
    want = torch.empty(M, Kc, device="cuda")
    K.gemm([K.Seg(gd, 8 * H, 4 * H, refs[0], T), K.Seg(gd, 8 * H, 4 * H, refs[1], T, xoff=4 * H)],
           M // T, T, Kc, pb, want, Kc)

    def run(out):
        assert K.blas_gemm(gd, 8 * H, refs[0], pb, M, Kc, 4 * H, out, Kc)
        assert K.blas_gemm(gd, 8 * H, refs[1], pb, M, Kc, 4 * H, out, Kc, accum=True, xoff=4 * H)
    got = torch.full((M, Kc), float("nan"), device="cuda")
    run(got)
    torch.cuda.synchronize()
    assert _close(got, want)
    cap = torch.full((M, Kc), float("nan"), device="cuda")
    graph = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            run(cap)
    torch.cuda.current_stream().wait_stream(s)
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(cap.view(torch.int32), got.view(torch.int32))

