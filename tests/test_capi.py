"""The C-ABI library loads and exports every symbol include/ensvs.h declares (CPU only)."""
import ctypes
import os
import re

from ensemble_svs_with_interactions_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "ensvs.h")).read()
    return sorted(set(re.findall(r"^(?:int|long long) (ensvs_\w+)\(", src, flags=re.M)))


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
    src = '#include "ensvs.h"\n#include <stdio.h>\nint main(){printf("%zu %zu\\n", sizeof(ensvs_conv_seg), sizeof(ensvs_pack_desc));}\n'
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "t.c"), "w") as f:
            f.write(src)
        subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), os.path.join(d, "t.c"),
                               "-o", os.path.join(d, "t")])
        out = subprocess.check_output([os.path.join(d, "t")]).decode().split()
    assert int(out[0]) == ctypes.sizeof(_lib.ConvSeg)
    assert int(out[1]) == ctypes.sizeof(_lib.PackDesc)


def test_library_newer_than_sources():
    import glob
    lib_t = os.path.getmtime(_lib.LIB_PATH)
    for s in glob.glob(os.path.join(ROOT, "ensemble_svs_with_interactions_amd", "csrc", "*")):
        assert os.path.getmtime(s) <= lib_t, f"stale libensvs.so: {s} is newer (run make)"


def test_workspace_query():
    # 1000 frames -> 4 chunks of 256 frames, each a V x C partial table
    assert _lib.query("ensvs_embed_bwd_workspace", 1000, 256, 47) == 4 * 47 * 256
