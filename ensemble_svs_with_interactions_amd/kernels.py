"""Thin launch layer over libensvs.so: packed-weight management and GEMM calls.

Everything here only moves pointers and sizes; all arithmetic happens in the
HIP kernels of ``csrc/``.  Tensors are fp32, channels-last frame rows.
"""
import contextlib
import ctypes
from dataclasses import dataclass
from typing import List, Optional

import torch

from . import _lib
from ._lib import ConvSeg, PackDesc, call, ptr

BM = 128
BK = 32


def _roundup(x, m):
    return (x + m - 1) // m * m


def stream():
    return torch.cuda.current_stream().cuda_stream


# weight repacks as one workgroup per 64 x 64 tile (ensvs_pack_weights_tiled: coalesced
# reads and writes through LDS, exactly the tiles) or the element-per-thread pack_kernel;
# same bits
PACK_TILED = {"on": True}
PACK_TILE = 64  # gemm.hip PACK_T


@dataclass
class PackedRef:
    """Where one packed GEMM operand lives inside a PackedBuffer."""
    offset: int  # elements
    N: int
    K: int
    taps: int
    Npad: int
    Kp: int


class PackedBuffer:
    """A set of weights repacked to the GEMM layout [tap][Npad][Kp] by ONE launch.

    Sources are views into the model's flat fp32 parameter buffer; the packed
    copy is refreshed with :meth:`repack` after every optimizer step.
    """

    def __init__(self, dtype: int):
        self.dtype = dtype
        self.specs = []
        self.size = 0
        self.buf = None
        self._dev_descs = None
        self._max = 0

    def add(self, src: torch.Tensor, N: int, K: int, taps: int, sn: int, sk: int, sj: int,
            perm_c: int = 0, flip: bool = False, transpose: bool = False, scale: float = 1.0,
            src2: Optional[torch.Tensor] = None, npad_to: int = BM, kpad_to: int = BK) -> PackedRef:
        gn, gk = (K, N) if transpose else (N, K)  # GEMM (rows of packed, reduction)
        Npad = _roundup(gn, npad_to)
        Kp = _roundup(gk, kpad_to)
        ref = PackedRef(self.size, gn, gk, taps, Npad, Kp)
        self.specs.append(dict(src=src, src2=src2, sn=sn, sk=sk, sj=sj, N=N, K=K, taps=taps,
                               Npad=Npad, Kp=Kp, perm_c=perm_c, flip=int(flip),
                               transpose=int(transpose), scale=float(scale), ref=ref))
        n = taps * Npad * Kp
        self.size += _roundup(n, 64)
        self._max = max(self._max, n)
        return ref

    def add_rowcat(self, srcs, N, K, transpose_blocks=False, scale=1.0, kpad_to=BK):
        """One GEMM operand made of several Linear weights.

        transpose_blocks=False: rows concatenated  -> packed (len*N) x K   (stacked outputs)
        transpose_blocks=True:  W_l^T side by side  -> packed K x (len*N)  (summed inputs)
        """
        L = len(srcs)
        if not transpose_blocks:
            Npad, Kp = _roundup(L * N, BM), _roundup(K, kpad_to)
            ref = PackedRef(self.size, L * N, K, 1, Npad, Kp)
            for l, w in enumerate(srcs):
                sub = PackedRef(self.size + l * N * Kp, N, K, 1, N, Kp)
                self.specs.append(dict(src=w, src2=None, sn=K, sk=1, sj=1, N=N, K=K, taps=1,
                                       Npad=N, Kp=Kp, perm_c=0, flip=0, transpose=0,
                                       scale=float(scale), ref=sub, ldk=0))
        else:
            Npad, Kp = _roundup(K, BM), _roundup(L * N, BK)
            ref = PackedRef(self.size, K, L * N, 1, Npad, Kp)
            for l, w in enumerate(srcs):
                sub = PackedRef(self.size + l * N, K, N, 1, Npad, N)
                self.specs.append(dict(src=w, src2=None, sn=K, sk=1, sj=1, N=N, K=K, taps=1,
                                       Npad=Npad, Kp=N, perm_c=0, flip=0, transpose=1,
                                       scale=float(scale), ref=sub, ldk=Kp))
        n = Npad * Kp
        self.size += _roundup(n, 64)
        self._max = max(self._max, n)
        return ref

    def add_colcat(self, srcs, N, K, scale=1.0):
        """Several (N, K) weights (row stride K) side by side along the reduction: packed
        N x (len*K) -- one output summed over the inputs of every block (the DiffNet skip
        halves)."""
        L = len(srcs)
        Npad, Kp = _roundup(N, BM), _roundup(L * K, BK)
        ref = PackedRef(self.size, N, L * K, 1, Npad, Kp)
        for l, w in enumerate(srcs):
            sub = PackedRef(self.size + l * K, N, K, 1, Npad, K)
            self.specs.append(dict(src=w, src2=None, sn=K, sk=1, sj=1, N=N, K=K, taps=1,
                                   Npad=Npad, Kp=K, perm_c=0, flip=0, transpose=0,
                                   scale=float(scale), ref=sub, ldk=Kp))
        n = Npad * Kp
        self.size += _roundup(n, 64)
        self._max = max(self._max, n)
        return ref

    def finalize(self, device):
        tdtype = torch.bfloat16 if self.dtype == _lib.DT_BF16 else torch.float32
        self.buf = torch.zeros(max(self.size, 64), dtype=tdtype, device=device)
        n = len(self.specs)
        arr = (PackDesc * max(n, 1))()
        esz = self.buf.element_size()
        tiles = 0
        for i, s in enumerate(self.specs):
            d = arr[i]
            d.src = s["src"].data_ptr()
            d.src2 = None if s["src2"] is None else s["src2"].data_ptr()
            d.dst = self.buf.data_ptr() + s["ref"].offset * esz
            d.sn, d.sk, d.sj = s["sn"], s["sk"], s["sj"]
            d.N, d.K, d.taps, d.Npad, d.Kp = s["N"], s["K"], s["taps"], s["Npad"], s["Kp"]
            d.perm_c, d.flip, d.transpose = s["perm_c"], s["flip"], s["transpose"]
            d.dtype, d.scale = self.dtype, s["scale"]
            d.ldk = s.get("ldk", 0)
            d.tile0 = tiles
            tiles += s["taps"] * -(-s["Npad"] // PACK_TILE) * -(-s["Kp"] // PACK_TILE)
        self._tiles = tiles
        raw = bytes(arr)
        host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
        self._dev_descs = host.to(device)
        self._n = n

    def repack(self):
        if not self._n:
            return
        if PACK_TILED["on"]:
            call("ensvs_pack_weights_tiled", self._dev_descs.data_ptr(), self._n, self._tiles,
                 stream())
        else:
            call("ensvs_pack_weights", self._dev_descs.data_ptr(), self._n, self._max, stream())


@dataclass
class Seg:
    """One K-segment of a GEMM's activation operand."""
    x: torch.Tensor         # any tensor whose data_ptr is the segment's first channel of frame 0
    ld: int                 # row stride (floats)
    K: int                  # channels
    ref: PackedRef          # packed weights of this segment
    Tin: int
    taps: int = 1
    dil: int = 1
    shift0: int = 0
    pad: int = _lib.PAD_ZERO
    radd: Optional[torch.Tensor] = None
    radd_ld: int = 0
    xoff: int = 0           # element offset added to x.data_ptr()
    pd: Optional[torch.Tensor] = None  # per-row pitch-dependent dilation factor (uSFGAN)
    pd_dil: int = 0


# bf16-operand GEMMs: activations rounded to bf16 in HBM by one cast pass (radd fused),
# then both operands staged by global_load_lds (ensvs_conv_gemm_bf16a).  Same bits as the
# register-staged kernel; pays where the A tile is re-read (several N tiles or taps) --
# at every row count: at M = 2 000 (one pair of 10 s in the reverse diffusion) a
# register-staged DiffNet GEMM launch averaged 33 us against ~10 us here (pair inference
# 185 -> 102 ms), so there is no row threshold (min_rows 0).  Single-reuse GEMMs (one tap,
# one N tile) too (min_reuse 1): round 5, with the plain ones on hipBLASLt, 13.46-13.53 vs
# 13.51-13.56 ms/step, SeparateF0 and synth RTF unchanged (profiles/r5_min_reuse_ab.txt;
# round 2 measured 22.0 vs 21.9 ms/step and ensemble RTF 0.0305 vs 0.0294 and kept 2).  Two
# LDS stages (three: 22.3 vs 20.1 ms/step).  Tests switch the entries to compare the paths
# bitwise.
BF16_ACT = {"on": True, "stages": 2, "stages_small": 2, "min_reuse": 1, "min_rows": 0}


# Small-M bf16-operand GEMMs split their K-steps over up to max_split workgroups per output
# tile (ensvs_conv_gemm_bf16a: part / part_floats) when the launch has fewer than max_tiles
# tiles.  Off: the 64 x 64-tile kernel fills the chip at small M instead (its accumulation
# order is the register-staged kernel's); the sum-order tests switch it on.
SPLITK = {"on": False, "max_split": 8, "max_tiles": 128}


def _castable(s):
    """ensvs_cast_bf16's operand contract (gemm.hip): K % 8, ld % 4, 16-B aligned rows and
    radd; an fp32 segment that misses it stays on the register-staged kernel."""
    ok = s.pd is None and s.K % 8 == 0 and s.ld % 4 == 0 and \
        (s.x.data_ptr() + 4 * s.xoff) % 16 == 0
    if s.radd is not None:
        ok = ok and s.radd_ld % 4 == 0 and s.radd.data_ptr() % 16 == 0
    return ok


def _bf16_act_ok(segs, W, Npad, M):
    if any(s.x.dtype == torch.bfloat16 for s in segs):  # operands already rounded
        # (a pitch-dependent segment: segment 0, already bf16 -- the 128 x 128 kernel gathers it)
        assert W.dtype == _lib.DT_BF16 and all(s.pd is None or (i == 0 and s.x.dtype ==
                                                                torch.bfloat16)
                                               for i, s in enumerate(segs))
        assert all(s.radd is None for s in segs if s.x.dtype == torch.bfloat16)
        for s in segs:  # ensvs_conv_gemm_bf16a's contract: a caller-side layout error
            if s.x.dtype == torch.bfloat16 and (s.ld % 8 or (s.x.data_ptr() + 2 * s.xoff) % 16
                                                or s.ld < -(-s.K // 8) * 8):
                raise ValueError("bf16 GEMM operand needs ld % 8 == 0 and 16-B aligned rows "
                                 "(K % 8 != 0: zero-padded to a multiple of 8 within ld)")
            if s.x.dtype != torch.bfloat16 and not _castable(s):
                raise ValueError("fp32 segment beside bf16 operands is not castable")
        return True
    if not BF16_ACT["on"] or W.dtype != _lib.DT_BF16 or M < BF16_ACT["min_rows"]:
        return False
    if not all(_castable(s) for s in segs):
        return False
    return max(s.taps for s in segs) * (Npad // 128) >= BF16_ACT["min_reuse"]


def set_big_tile(mode, stages=0):
    """Route large-M bf16-operand GEMMs to a 256 x 256-tile kernel (mode 2: 64-deep
    two-stage, the default; 1: 32-deep LDS ring of `stages` stages) or keep them on the
    128 x 128 kernel (0 / False); all give identical bits."""
    _lib.call("ensvs_set_big_tile", int(mode), int(stages))


def set_small(on):
    """Small-M bf16-operand launches (< 128 tiles of 128 x 128) on the 64 x 64-tile kernel
    (default; the one-group kernel's bits) or on the dual / split-K / one-group kernels."""
    _lib.call("ensvs_set_small", int(bool(on)))


def set_dual_small(on):
    """Small-M bf16-operand launches (< 128 tiles) that the 64 x 64 kernel does not take on
    the two-K-group kernel, or on the one-group kernel (default: the register-staged
    kernel's bits)."""
    _lib.call("ensvs_set_dual_small", int(bool(on)))


def gemm_dtype_is_bf16(W):
    return W.dtype == _lib.DT_BF16


def cast_bf16(x, ld, K, rows, xoff=0, radd=None, radd_ld=0, T=1, out=None, out_ld=0, out_off=0):
    """bf16 copy [rows, K] of x (row stride ld floats, + radd[row // T] when given); into
    `out` (row stride out_ld, element offset out_off) when given."""
    if out is None:
        out, out_ld, out_off = torch.empty(rows, K, dtype=torch.bfloat16, device=x.device), K, 0
    call("ensvs_cast_bf16", x.data_ptr() + 4 * xoff, ld, ptr(radd), radd_ld, T, rows, K,
         out.data_ptr() + 2 * out_off, out_ld, stream())
    return out


def gemm(segs: List[Seg], B: int, Tout: int, N: int, W: PackedBuffer, Y, ldy: int,
         bias=None, epi=_lib.EPI_PLAIN, relu=False, accum=False, aux0=None, ld0=0, aux1=None,
         ld1=0, alpha=0.0, C=0, yoff=0, bias_off=0, ybf=None, ybf_ld=0, ybf_radd=None,
         ybf_radd_ld=0, csum=None, csum_ld=0, csum_off=0, keep_y=True):
    """One implicit-GEMM launch (bf16-operand kernel when the A panels are bf16 or worth a
    cast pass, register-staged kernel otherwise).  ybf (bf16 tensor): also receives
    bf16(y + ybf_radd[row // Tout]) of the Y values written (PLAIN / GATE / RESSKIP /
    ADDSCALE: the Y columns; GATE_BWD: both halves) -- from the epilogue when it can, else
    by a cast.  csum (fp32, B*Tout % 128 == 0, no bias / accum / relu): per 128-row tile
    column sums of the accumulator into csum[tile * csum_ld + csum_off + n] -- from the
    epilogue when it can, else by ensvs_tile_colsum (the same bits); GATE_BWD: of both
    outputs.  keep_y=False (GATE with ybf, GATE_BWD with ybf / csum): the fp32 Y is not
    needed by the caller and the fused epilogue skips it (Y stays allocated for the
    fallback paths, which still write it)."""
    arr = (ConvSeg * len(segs))()
    Npad = segs[0].ref.Npad
    # C-ABI epilogue flags: a bf16 gate/filter save (DiffNet production path)
    ep = epi
    if aux0 is not None and aux0.dtype == torch.bfloat16:
        ep |= _lib.EPI_AUX0_BF16
    if aux1 is not None and aux1.dtype == torch.bfloat16:
        ep |= _lib.EPI_AUX1_BF16
    M = B * Tout
    a16 = _bf16_act_ok(segs, W, Npad, M)
    if csum is not None:
        assert (M % BM == 0 and bias is None and not accum and not relu and
                epi in (_lib.EPI_PLAIN, _lib.EPI_ADDSCALE, _lib.EPI_GATE_BWD) and
                ybf_radd is None)
        yp = Y.data_ptr() + 4 * yoff
        vec = (yp % 16 == 0 and ldy % 4 == 0 and N % 4 == 0 and C % 4 == 0 and
               (aux1 is None or (aux1.data_ptr() % 16 == 0 and ld1 % 4 == 0)) and
               (ybf is None or (ybf.data_ptr() % 8 == 0 and ybf_ld % 4 == 0)))
        if not (a16 and vec) and epi == _lib.EPI_GATE_BWD:
            gemm(segs, B, Tout, N, W, Y, ldy, epi=epi, aux1=aux1, ld1=ld1, C=C, yoff=yoff,
                 ybf=ybf, ybf_ld=ybf_ld)
            call("ensvs_tile_colsum", yp, ldy, M, 2 * C, csum.data_ptr() + 4 * csum_off,
                 csum_ld, stream())
            return
        if not (a16 and vec):
            # the accumulator through a plain Y, its tile sums, then the epilogue as a pass
            flat = ldy == N and yoff == 0 and (aux1 is None or ld1 == N)
            assert flat, "csum fallback needs contiguous Y / aux1"
            acc = Y if epi == _lib.EPI_PLAIN else torch.empty(M, N, device=Y.device)
            gemm(segs, B, Tout, N, W, acc, N)
            call("ensvs_tile_colsum", acc.data_ptr(), N, M, N, csum.data_ptr() + 4 * csum_off,
                 csum_ld, stream())
            if epi == _lib.EPI_ADDSCALE:
                if ybf is not None and ybf_ld == N:
                    call("ensvs_axpby_to_bf16", Y.data_ptr(), ybf.data_ptr(), aux1.data_ptr(),
                         float(alpha), acc.data_ptr(), 1.0, M * N, stream())
                    return
                call("ensvs_axpby_to", Y.data_ptr(), aux1.data_ptr(), float(alpha),
                     acc.data_ptr(), 1.0, M * N, stream())
            if ybf is not None:
                cast_bf16(Y, N, N, M, out=ybf, out_ld=ybf_ld)
            return
    if ybf is not None and csum is None:
        assert ybf.dtype == torch.bfloat16 and epi in (_lib.EPI_PLAIN, _lib.EPI_GATE,
                                                       _lib.EPI_RESSKIP, _lib.EPI_GATE_BWD,
                                                       _lib.EPI_GATE_TS, _lib.EPI_ADDSCALE,
                                                       _lib.EPI_RELU_MASK)
        yp = Y.data_ptr() + 4 * yoff
        vec = (yp % 16 == 0 and ldy % 4 == 0 and N % 4 == 0 and C % 4 == 0 and
               all(t is None or (t.data_ptr() % 16 == 0 and ld % 4 == 0)
                   for t, ld in ((aux0, ld0), (aux1, ld1))) and ybf.data_ptr() % 8 == 0 and
               ybf_ld % 4 == 0 and (ybf_radd is None or (ybf_radd.data_ptr() % 16 == 0 and
                                                         ybf_radd_ld % 4 == 0)))
        if not (a16 and vec):
            gemm(segs, B, Tout, N, W, Y, ldy, bias=bias, epi=epi, relu=relu, accum=accum,
                 aux0=aux0, ld0=ld0, aux1=aux1, ld1=ld1, alpha=alpha, C=C, yoff=yoff,
                 bias_off=bias_off)
            # the same rounding by a cast pass over what was written
            width = 2 * C if epi == _lib.EPI_GATE_BWD else (
                C if epi in (_lib.EPI_GATE, _lib.EPI_RESSKIP, _lib.EPI_GATE_TS) else N)
            cast_bf16(Y, ldy, width, B * Tout, xoff=yoff, radd=ybf_radd, radd_ld=ybf_radd_ld,
                      T=Tout, out=ybf, out_ld=ybf_ld)
            return
    keep = []
    for i, s in enumerate(segs):
        assert s.ref.Npad == Npad and s.ref.taps == s.taps and s.ref.Kp >= s.K
        d = arr[i]
        if a16 and s.x.dtype == torch.bfloat16:
            d.x, d.ld, d.radd, d.radd_ld = s.x.data_ptr() + 2 * s.xoff, s.ld, None, 0
        elif a16:
            xb = cast_bf16(s.x, s.ld, s.K, B * s.Tin, s.xoff, s.radd, s.radd_ld, s.Tin)
            keep.append(xb)
            d.x, d.ld, d.radd, d.radd_ld = xb.data_ptr(), s.K, None, 0
        else:
            d.x = s.x.data_ptr() + 4 * s.xoff
            d.radd = None if s.radd is None else s.radd.data_ptr()
            d.ld, d.radd_ld = s.ld, s.radd_ld
        d.pd = None if s.pd is None else s.pd.data_ptr()
        d.pd_dil = s.pd_dil
        d.wofs = s.ref.offset
        d.K, d.taps, d.dil, d.shift0 = s.K, s.taps, s.dil, s.shift0
        d.pad, d.Tin, d.Kp = s.pad, s.Tin, s.ref.Kp
    bptr = None if bias is None else bias.data_ptr() + 4 * bias_off
    yptr = Y.data_ptr() + 4 * yoff
    if not keep_y and ((epi in (_lib.EPI_GATE, _lib.EPI_GATE_TS) and ybf is not None) or
                       (epi == _lib.EPI_GATE_BWD and (ybf is not None or csum is not None))):
        yptr = None  # only reached on the fused-epilogue path
    # split-K workspace for small-M launches (fewer than 128 output tiles of 128 x 128)
    part, part_n = None, 0
    small = -(-M // BM) * (Npad // BM) < SPLITK["max_tiles"]
    stages = BF16_ACT["stages_small"] if small else BF16_ACT["stages"]
    if a16 and csum is None and SPLITK["on"] and small:
        part_n = SPLITK["max_split"] * M * Npad
        part = scratch(part_n, segs[0].x.device, key="splitk")
    if ybf is not None or csum is not None:
        call("ensvs_conv_gemm_bf16a_out", ctypes.addressof(arr), len(segs), B, Tout, N,
             Npad, W.buf.data_ptr(), bptr, yptr, ldy, ep, int(relu), int(accum), ptr(aux0),
             ld0, ptr(aux1), ld1, float(alpha), C, ptr(ybf), ybf_ld, ptr(ybf_radd),
             ybf_radd_ld, None if csum is None else csum.data_ptr() + 4 * csum_off, csum_ld,
             stages, ptr(part), part_n, stream())
        return
    if a16:
        call("ensvs_conv_gemm_bf16a", ctypes.addressof(arr), len(segs), B, Tout, N, Npad,
             W.buf.data_ptr(), bptr, yptr, ldy, ep, int(relu), int(accum),
             ptr(aux0), ld0, ptr(aux1), ld1, float(alpha), C, stages, ptr(part),
             part_n, stream())
    else:
        call("ensvs_conv_gemm", ctypes.addressof(arr), len(segs), B, Tout, N, Npad,
             W.buf.data_ptr(), W.dtype, bptr, yptr, ldy, ep, int(relu),
             int(accum), ptr(aux0), ld0, ptr(aux1), ld1, float(alpha), C, stream())


def usf_block(segs: List[Seg], B, Tout, W: PackedBuffer, C, ref2, x, ldx, alpha, relu=False,
              xb=None, bias=None, bias_off=0, bias2=None, bias2_off=0):
    """One uSFGAN residual block in one launch (ensvs_usf_block): the gate GEMM over the
    bf16 segments segs (packed 2C = 128 gate/filter columns), z on chip, the output conv
    ref2 and x = alpha * x + out + bias2 in place (+ its bf16 copy xb).  The same bits as
    gemm(.., EPI_GATE_TS, ybf=z copy) followed by gemm(.., EPI_ADDSCALE) on that copy."""
    arr = (ConvSeg * len(segs))()
    for d, sg in zip(arr, segs):
        assert sg.x.dtype == torch.bfloat16 and sg.radd is None and sg.ref.taps == sg.taps
        d.x = sg.x.data_ptr() + 2 * sg.xoff
        d.ld, d.radd, d.radd_ld = sg.ld, None, 0
        d.pd = None if sg.pd is None else sg.pd.data_ptr()
        d.pd_dil = sg.pd_dil
        d.wofs = sg.ref.offset
        d.K, d.taps, d.dil, d.shift0 = sg.K, sg.taps, sg.dil, sg.shift0
        d.pad, d.Tin, d.Kp = sg.pad, sg.Tin, sg.ref.Kp
    call("ensvs_usf_block", ctypes.addressof(arr), len(segs), B, Tout, W.buf.data_ptr(),
         None if bias is None else bias.data_ptr() + 4 * bias_off, C, ref2.offset, ref2.Kp,
         None if bias2 is None else bias2.data_ptr() + 4 * bias2_off, x.data_ptr(), ldx,
         float(alpha), int(bool(relu)), ptr(xb), 0 if xb is None else xb.shape[1], stream())


def bf16_operands(W, M):
    """Whether GEMMs on these packed weights with M rows take pre-rounded bf16 operands
    (callers then round an operand shared by several GEMMs once, instead of per GEMM)."""
    return BF16_ACT["on"] and W.dtype == _lib.DT_BF16 and M >= BF16_ACT["min_rows"]


_part_cache = {}


def scratch(nfloats, device, key="part"):
    """Reusable split-reduction workspace, one per (key, device, stream): launches on
    one stream are ordered, launches on concurrent branch streams get their own."""
    ck = (key, device, torch.cuda.current_stream(device).cuda_stream)
    t = _part_cache.get(ck)
    if t is None or t.numel() < nfloats:
        if t is not None:  # a captured graph may hold the old one (engine.retire)
            from .engine import retire
            retire(t)
        grow = 2 * t.numel() if t is not None else 0
        t = torch.empty(max(nfloats, grow, 1 << 20), dtype=torch.float32, device=device)
        _part_cache[ck] = t
    return t


# fp32-operand weight gradients whose channel count the vector kernels cannot stage (K % 4)
# run on bf16 copies through the LDS-DMA kernel (wgrad above); off: the register kernel
WGRAD_CAST = {"on": True}
# weight gradients split the frame reduction until about this many workgroups (tile x split)
WGRAD_TARGET = 512  # workgroups a weight gradient aims for (256: 20.7, 1024: 20.5 vs 20.1 ms/step)
# bf16 weight gradients with >= 16 output tiles of 256 x 256: the 256 x 256-tile kernel (its
# switch is ensvs_set_wgrad_big, the shape rule gemm.hip wgrad_big_shape; splits are chosen
# here for one workgroup per CU)
WGRAD_BIG = {"on": True, "target": 256}


def set_wgrad_big(on: bool):
    """The 256 x 256 weight-gradient kernel on / off, in the library (ensvs_set_wgrad_big) and
    in the split-count rule below together, so the splits always match the kernel that runs."""
    call("ensvs_set_wgrad_big", int(bool(on)))
    WGRAD_BIG["on"] = bool(on)


class WredDesc(ctypes.Structure):  # include/ensvs.h ensvs_wred_desc
    _fields_ = [("part", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("sn", ctypes.c_longlong),
                ("sk", ctypes.c_longlong), ("sj", ctypes.c_longlong), ("splits", ctypes.c_int),
                ("taps", ctypes.c_int), ("N", ctypes.c_int), ("K", ctypes.c_int),
                ("accum", ctypes.c_int), ("scale", ctypes.c_float)]


# Deferred split reductions of the weight gradients of one training step: inside
# deferred_wgrad(), a parameter gradient split over row splits (wgrad_into) writes its
# partials into a buffer of its own and the reduction is queued per stream; flush_wgrad()
# issues every queued reduction of the current stream as ONE launch
# (ensvs_wgrad_reduce_batch: the same per-element sums, the same bits).  Branch ends
# (engine.Branches) and the data-parallel bucket launches flush, so no reader sees a gradient
# before its reduction.  ~140 reduce launches per training step become a handful.
# stream handle -> [(desc fields, part or source, (lo, hi))]: weight-gradient reductions and
# bias-gradient column sums
_DEFER = {"depth": 0, "pending": {}, "colsum": {}}


@contextlib.contextmanager
def deferred_wgrad():
    _DEFER["depth"] += 1
    try:
        yield
    except BaseException:
        # the branch that raised left its queue unflushed: drop the queues and let the
        # original error (a CoopError, an OOM, ...) propagate unchanged
        _DEFER["depth"] -= 1
        if _DEFER["depth"] == 0:
            _DEFER["pending"].clear()
            _DEFER["colsum"].clear()
        raise
    else:
        _DEFER["depth"] -= 1
        flush_wgrad()
        if _DEFER["depth"] == 0 and (_DEFER["pending"] or _DEFER["colsum"]):
            left = {k: len(v) for k, v in list(_DEFER["pending"].items()) +
                    list(_DEFER["colsum"].items())}
            _DEFER["pending"].clear()
            _DEFER["colsum"].clear()
            raise RuntimeError(f"weight-gradient reductions queued on streams {left} were "
                               "never flushed (a wgrad outside an engine.Branches region)")


def flush_wgrad():
    """Issue the current stream's queued weight-gradient reductions (one launch per 48) and
    column sums (two launches per 48)."""
    if not _DEFER["pending"] and not _DEFER["colsum"]:
        return
    key = stream()
    cols = _DEFER["colsum"].pop(key, None)
    if cols:
        carr = (ColsumDesc * len(cols))()
        for i, (f, _, _) in enumerate(cols):
            carr[i] = ColsumDesc(*f)
        nf = _lib.query("ensvs_colsum_batch_part_floats", ctypes.addressof(carr), len(cols))
        part = scratch(nf, cols[0][1].device, key="colsum_batch")
        call("ensvs_colsum_batch", ctypes.addressof(carr), len(cols), part.data_ptr(), nf, key)
    items = _DEFER["pending"].pop(key, None)
    if not items:
        return
    arr = (WredDesc * len(items))()
    for i, (f, _, _) in enumerate(items):
        arr[i] = WredDesc(*f)
    call("ensvs_wgrad_reduce_batch", ctypes.addressof(arr), len(items), key)
    # the partial buffers go back to the caching allocator here: stream-ordered, so a later
    # allocation on this stream reuses them only after the reduction has read them


def wgrad(dy, ldy, x, ldx, B, Tout, Tin, N, K, taps, dil, shift0, pad, dst, sn, sk, sj,
          accum=False, dtype=_lib.DT_BF16, radd=None, radd_ld=0, dyoff=0, xoff=0, splits=None,
          scale=1.0, dstoff=0, defer=False):
    """dst (+)= scale * dy^T x (conv/linear weight gradient).  dy and x may both be bf16
    tensors already rounded (radd then folded into x): the glds-staged kernel, same bits.
    defer: inside deferred_wgrad(), queue the split reduction (see flush_wgrad)."""
    M = B * Tout
    if (splits is None and dtype == _lib.DT_BF16 and WGRAD_BIG["on"] and N >= 256 and
            K >= 256 and -(-N // 256) * -(-K // 256) * taps >= 16):
        # the 256 x 256-tile kernel (gemm.hip wgrad_b16_big_kernel) for bf16 operands, one
        # workgroup per CU; fp32 sources rounded in staging (production precision) take the
        # same split count, so they give the same bits.  Exact-fp32 parity mode (DT_F32)
        # keeps the 128 x 128 kernel's split rule.
        tiles = -(-N // 256) * -(-K // 256) * taps
        splits = max(1, min(64, WGRAD_BIG["target"] // max(tiles, 1), -(-M // 512)))
    if splits is None:
        tiles = -(-N // 128) * -(-K // 128) * taps
        splits = max(1, min(64, WGRAD_TARGET // max(tiles, 1), -(-M // 256)))
        # a multiple of 8 lets each split's workgroups share one XCD's L2 (gemm.hip
        # wgrad_tile) -- when that still fits one wave of WGRAD_TARGET workgroups: rounding
        # the DiffNet dilated conv's 21 splits up to 24 (576 workgroups) cost 51 -> 68 us
        up = -(-splits // 8) * 8
        if splits >= 8 and up * tiles <= WGRAD_TARGET:
            splits = up
    def castable(t, ld, C, off):  # ensvs_cast_bf16: the padded copy, or 16-B rows
        return C % 8 or (ld % 4 == 0 and (t.data_ptr() + 4 * off) % 16 == 0)
    if (WGRAD_CAST["on"] and dtype == _lib.DT_BF16 and radd is None and (K % 4 or N % 4)
            and dy.dtype == x.dtype == torch.float32 and castable(x, ldx, K, xoff) and
            castable(dy, ldy, N, dyoff)):
        # fp32 operands with an odd channel count (the input-feature embeddings, K = 39 / 130;
        # the 1-channel k7 conv; K = 5; the 1 / 4 / 5-wide output projections) stage one
        # element per lane on the register kernel: bf16 copies (zero-padded to 8 channels, the
        # rounding the kernel applies while staging) and the LDS-DMA kernel instead, same split
        # count
        def b16(t, ld, C, rows, off):
            C8 = -(-C // 8) * 8
            out = torch.empty(rows, C8, dtype=torch.bfloat16, device=t.device)
            call("ensvs_cast_bf16", t.data_ptr() + 4 * off, ld, None, 0, 1, rows, C,
                 out.data_ptr(), C8, stream())
            return out, C8
        x, ldx = b16(x, ldx, K, B * Tin, xoff)
        dy, ldy = b16(dy, ldy, N, M, dyoff)
        dyoff = xoff = 0
    flag = int(accum)
    dptr = dst.data_ptr() + 4 * dstoff
    queue = None
    if defer and DEFER_WGRAD["on"] and splits > 1 and _DEFER["depth"] > 0:
        lo = dptr
        hi = dptr + 4 * ((N - 1) * sn + (K - 1) * sk + (taps - 1) * sj + 1)
        key = stream()
        if any(a < hi and lo < b for _, _, (a, b) in _DEFER["pending"].get(key, ())):
            flush_wgrad()  # one launch's destinations must not overlap
        part = torch.empty(splits * taps * N * K, dtype=torch.float32, device=dy.device)
        queue = ((part.data_ptr(), dptr, sn, sk, sj, splits, taps, N, K, int(accum),
                  float(scale)), part, (lo, hi))
        flag |= 2  # ENSVS_WGRAD_DEFER
    else:
        part = scratch(splits * taps * N * K, dy.device)
    if dy.dtype == torch.bfloat16 or x.dtype == torch.bfloat16:
        assert dy.dtype == x.dtype == torch.bfloat16 and radd is None and dtype == _lib.DT_BF16
        call("ensvs_conv_wgrad_bf16", dy.data_ptr() + 2 * dyoff, ldy, x.data_ptr() + 2 * xoff,
             ldx, B, Tout, Tin, N, K, taps, dil, shift0, pad, splits, part.data_ptr(),
             dptr, sn, sk, sj, flag, float(scale), stream())
    else:
        call("ensvs_conv_wgrad", dy.data_ptr() + 4 * dyoff, ldy, x.data_ptr() + 4 * xoff, ldx,
             ptr(radd), radd_ld, B, Tout, Tin, N, K, taps, dil, shift0, pad, splits,
             part.data_ptr(), dptr, sn, sk, sj, flag, float(scale), dtype, stream())
    if queue is not None:
        _DEFER["pending"].setdefault(stream(), []).append(queue)


_cnt_cache = {}
# column sums in one launch (ensvs_colsum_once, the last block of each column block reducing
# the split partials) or two (partial + final kernels); same bits.  Off: the one-launch form
# measured slower in the step, 14.27 / 14.31 vs 13.98 / 14.04 ms (write-through form;
# 15.48 ms with release / acquire fences), profiles/r5_reduction_ab.txt
COLSUM_ONCE = {"on": False}
# queue the split reductions of parameter gradients inside deferred_wgrad() (one batched launch
# per branch, ~140 -> ~10 reduce launches per step) or reduce each weight gradient right after
# it (same bits either way): 13.91 / 13.92 vs 13.98 / 14.04 ms, profiles/r5_reduction_ab.txt
DEFER_WGRAD = {"on": True}
# queue the bias-gradient column sums (layers.colsum_into) the same way: one ensvs_colsum_batch
# (two launches) per flush instead of two launches per bias
DEFER_COLSUM = {"on": True}


def counters(n, device):
    """Zero-initialised ticket counters of the single-launch reductions (ensvs_colsum_once),
    one buffer per (device, stream): every launch leaves them zero, launches on one stream
    are ordered, concurrent streams get their own."""
    ck = (device, torch.cuda.current_stream(device).cuda_stream)
    t = _cnt_cache.get(ck)
    if t is None or t.numel() < n:
        if t is not None:  # a captured graph may hold the old one (engine.retire)
            from .engine import retire
            retire(t)
        t = torch.zeros(max(n, 1 << 14), dtype=torch.int32, device=device)
        _cnt_cache[ck] = t
    return t


class ColsumDesc(ctypes.Structure):  # include/ensvs.h ensvs_colsum_desc
    _fields_ = [("y", ctypes.c_void_p), ("out", ctypes.c_void_p), ("ld", ctypes.c_int),
                ("M", ctypes.c_int), ("N", ctypes.c_int), ("max_splits", ctypes.c_int),
                ("scale", ctypes.c_float), ("accum", ctypes.c_int)]


def colsum(y, ld, M, N, out, groups=1, mean=None, scale=1.0, accum=False, yoff=0, ldo=0,
           outoff=0, defer=False):
    """out[g*ldo + n] (+)= scale * sum over the M rows of group g (ldo 0 -> N): partial and
    final launches (ensvs_colsum; COLSUM_ONCE: ensvs_colsum_once).  defer (a parameter
    gradient: groups 1, no mean): inside deferred_wgrad(), queued and issued with the stream's
    other deferred column sums by flush_wgrad (ensvs_colsum_batch, the same bits)."""
    # row splits: what ensvs_colsum picks (>= 2048 blocks, >= 128 rows per split)
    max_splits = max(1, min(256, M // 128, -(-2048 // (-(-N // 64) * groups))))
    if (defer and DEFER_COLSUM["on"] and _DEFER["depth"] > 0 and groups == 1 and mean is None
            and ldo == 0):
        lo = out.data_ptr() + 4 * outoff
        hi = lo + 4 * N
        key = stream()
        if any(a < hi and lo < b for _, _, (a, b) in _DEFER["colsum"].get(key, ())):
            flush_wgrad()  # one launch's outputs must not overlap
        _DEFER["colsum"].setdefault(key, []).append(
            ((y.data_ptr() + 4 * yoff, lo, ld, M, N, max_splits, float(scale), int(accum)), y,
             (lo, hi)))
        return
    part = scratch(groups * max_splits * N, y.device, key="colsum")
    if not COLSUM_ONCE["on"]:
        call("ensvs_colsum", y.data_ptr() + 4 * yoff, ld, M, groups, N, ptr(mean),
             float(scale), part.data_ptr(), max_splits, out.data_ptr() + 4 * outoff, ldo,
             int(accum), stream())
        return
    cnt = counters(-(-N // 64) * groups, y.device)
    call("ensvs_colsum_once", y.data_ptr() + 4 * yoff, ld, M, groups, N, ptr(mean),
         float(scale), part.data_ptr(), max_splits, cnt.data_ptr(),
         out.data_ptr() + 4 * outoff, ldo, int(accum), stream())
