"""The C-ABI library loads and exports every symbol include/ensvs.h declares (CPU only)."""
import ctypes
import os
import re

from ensemble_svs_with_interactions_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "ensvs.h")).read()
    return sorted(set(re.findall(r"^(?:int|long long|unsigned\*) (ensvs_\w+)\(", src, flags=re.M)))


def test_header_symbols_exported():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    names = declared()
    assert len(names) >= 25
    for n in names:
        assert hasattr(lib, n), n


def test_binding_covers_header():
    assert set(declared()) == set(_lib.SIGNATURES)


def test_loader_has_no_fallback(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(_lib, "_lib", None)
    try:
        _lib.load()
    except RuntimeError as e:
        assert "no CPU fallback" in str(e)
    else:
        raise AssertionError("load() must raise when the library is missing")


def test_struct_layouts_match_header():
    import subprocess, tempfile
    src = ('#include "ensvs.h"\n#include <stdio.h>\nint main(){printf("%zu %zu %zu %zu\\n", '
           'sizeof(ensvs_conv_seg), sizeof(ensvs_pack_desc), sizeof(ensvs_wred_desc), '
           'sizeof(ensvs_colsum_desc));}\n')
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "t.c"), "w") as f:
            f.write(src)
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), os.path.join(d, "t.c"),
                               "-o", os.path.join(d, "t")])
        out = subprocess.check_output([os.path.join(d, "t")]).decode().split()
    assert int(out[0]) == ctypes.sizeof(_lib.ConvSeg)
    assert int(out[1]) == ctypes.sizeof(_lib.PackDesc)
    from ensemble_svs_with_interactions_amd.kernels import ColsumDesc, WredDesc
    assert int(out[2]) == ctypes.sizeof(WredDesc)
    assert int(out[3]) == ctypes.sizeof(ColsumDesc)


def test_library_newer_than_sources():
    import glob
    lib_t = os.path.getmtime(_lib.LIB_PATH)
    for s in glob.glob(os.path.join(ROOT, "ensemble_svs_with_interactions_amd", "csrc", "*")):
        assert os.path.getmtime(s) <= lib_t, f"stale libensvs.so: {s} is newer (run make)"


def test_workspace_query():
    # 1000 frames -> 4 chunks of 256 frames, each a V x C partial table
    assert _lib.query("ensvs_embed_bwd_workspace", 1000, 256, 47) == 4 * 47 * 256


def test_gemm_rejects_inconsistent_epilogue_shapes():
    """Argument validation runs before any launch (no GPU needed): epilogue widths that
    would index past the caller's rows come back as E_SHAPE / E_ARG, not as a fault."""
    lib = ctypes.CDLL(_lib.LIB_PATH)
    seg = (_lib.ConvSeg * 1)()
    seg[0].x = 16
    seg[0].ld, seg[0].K, seg[0].taps, seg[0].Tin, seg[0].Kp = 256, 256, 1, 64, 256
    f = lib.ensvs_conv_gemm
    f.restype = ctypes.c_int
    P = ctypes.c_void_p
    # GATE_BWD expands C channels of dz into 2C outputs: N must equal C
    rc = f(seg, 1, 1, 64, 512, 512, P(16), 1, None, P(16), 512, _lib.EPI_GATE_BWD, 0, 0, None,
           0, P(16), 512, ctypes.c_float(0.0), 256, None)
    assert rc == 1
    # GATE: N = 2C interleaved gate/filter pairs
    rc = f(seg, 1, 1, 64, 256, 256, P(16), 1, None, P(16), 256, _lib.EPI_GATE, 0, 0, P(16),
           512, None, 0, ctypes.c_float(0.0), 256, None)
    assert rc == 1
    # RESSKIP needs its residual and skip operands
    rc = f(seg, 1, 1, 64, 512, 512, P(16), 1, None, P(16), 256, _lib.EPI_RESSKIP, 0, 0, None,
           0, None, 0, ctypes.c_float(0.0), 256, None)
    assert rc == 4


def test_coop_error_word_per_device():
    """The cooperative kernels' persistent error word is registered per device ordinal
    (ADVICE r4): registering device 1 does not move device 0's word, NULL unregisters, and
    out-of-range ordinals or misaligned words are rejected.  Host bookkeeping only."""
    g = _lib.query
    try:
        _lib.call("ensvs_coop_set_error_word_dev", 0, 0x1000)
        _lib.call("ensvs_coop_set_error_word_dev", 1, 0x2000)
        assert g("ensvs_coop_error_word", 0) == 0x1000
        assert g("ensvs_coop_error_word", 1) == 0x2000
        assert not g("ensvs_coop_error_word", 2)
        _lib.call("ensvs_coop_set_error_word_dev", 1, None)
        assert not g("ensvs_coop_error_word", 1)
        assert g("ensvs_coop_error_word", 0) == 0x1000
        lib = _lib.load()
        assert lib.ensvs_coop_set_error_word_dev(64, 0x1000) == 4
        assert lib.ensvs_coop_set_error_word_dev(-1, 0x1000) == 4
        assert lib.ensvs_coop_set_error_word_dev(0, 0x1002) == 4
        assert not g("ensvs_coop_error_word", 64)
    finally:
        _lib.call("ensvs_coop_set_error_word_dev", 0, None)
        _lib.call("ensvs_coop_set_error_word_dev", 1, None)


def test_pack_tile_numbering():
    """PackedBuffer's descriptors carry the tile numbering ensvs_pack_weights_tiled expects:
    tile0 = the prefix sum of taps * cdiv(Npad, 64) * cdiv(Kp, 64) in descriptor order, the
    launch's tile count their total (host logic only; the kernels are in test_pack_gpu.py)."""
    import torch
    from ensemble_svs_with_interactions_amd import kernels as K
    pb = K.PackedBuffer(_lib.DT_BF16)
    w = torch.zeros(77, 45, 5)
    pb.add(w, 77, 45, 5, 45 * 5, 5, 1)
    pb.add(w, 77, 45, 5, 45 * 5, 5, 1, flip=True, transpose=True)
    pb.add(torch.zeros(130, 200), 130, 200, 1, 200, 1, 1, npad_to=1, kpad_to=1)
    pb.add_rowcat([torch.zeros(33, 70) for _ in range(3)], 33, 70, transpose_blocks=True)
    pb.finalize(torch.device("cpu"))
    descs = (_lib.PackDesc * pb._n).from_buffer_copy(pb._dev_descs.numpy().tobytes())
    t = 0
    for d in descs:
        assert d.tile0 == t
        t += d.taps * -(-d.Npad // 64) * -(-d.Kp // 64)
    assert pb._tiles == t and pb._n == 6
    assert K.PACK_TILE == 64
