"""CPU tests of the C-ABI library: it loads, exports every symbol include/gsplat.h declares,
and its error paths fail loudly (no GPU needed; no compute calls)."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gsplat.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gs_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import openglgaussiansplattingrenderer_amd as g
    from openglgaussiansplattingrenderer_amd import _native
    L = ctypes.CDLL(g.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 30
    for s in syms:
        assert hasattr(L, s), s
        assert s in _native.SIGNATURES, f"{s} missing from the ctypes binding"
    # and the binding declares nothing the header does not
    assert set(_native.SIGNATURES) <= set(syms)


def test_library_is_gfx950_code_object():
    """the shipped .so carries a gfx950 code object (hand-written HIP, not a CPU build)"""
    import openglgaussiansplattingrenderer_amd as g
    data = open(g.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"k_draw" in data and b"k_downsweep" in data and b"k_preprocess" in data


def test_error_paths_without_device():
    import openglgaussiansplattingrenderer_amd as g
    L = g.lib()
    h = ctypes.c_void_p()
    assert L.gs_ctx_create(0, None) == -1
    n = ctypes.c_int()
    L.gs_device_count(ctypes.byref(n))
    if n.value == 0:  # CPU container: creating a context must fail loudly, not fall back
        rc = L.gs_ctx_create(0, ctypes.byref(h))
        assert rc == -2
        assert b"no HIP device" in L.gs_last_error(None)
        with pytest.raises(g.GsError):
            g.Context(0)
    assert L.gs_sort(None) == -1
    assert L.gs_render(None, None, None, 0, None, 0, None) == -1
    assert L.gs_ply_count(b"/nonexistent.ply", ctypes.byref(n)) == -3


def test_oracle_is_not_imported_by_product():
    """the product package never references oracle/"""
    pkg = os.path.join(ROOT, "openglgaussiansplattingrenderer_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".hpp", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"#\s*include\s*[<\"].*gs_oracle|^\s*(from|import)\s+oracle|libgsoracle", txt,
                                     re.M), f


def _read_png(path):
    """minimal PNG reader (8-bit RGBA, filter 0 rows) for the writer's output"""
    import struct
    import zlib
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat = 8, b""
    W = H = 0
    while pos < len(data):
        (n,) = struct.unpack(">I", data[pos:pos + 4])
        typ, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0]
        assert zlib.crc32(typ + body) == crc, typ
        if typ == b"IHDR":
            W, H = struct.unpack(">II", body[:8])
            assert body[8:13] == bytes([8, 6, 0, 0, 0])
        elif typ == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, np.uint8).reshape(H, 1 + 4 * W)
    assert np.all(rows[:, 0] == 0)
    return rows[:, 1:].reshape(H, W, 4)


@pytest.mark.parametrize("flip", [False, True])
def test_save_png_roundtrip(tmp_path, flip):
    """gs_save_png (saveImage, src/Splats.cpp:516-540): row 0 first unless flipped; > 64 KiB
    of rows spans several stored deflate blocks"""
    import openglgaussiansplattingrenderer_amd as g
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (130, 170, 4), dtype=np.uint8)
    p = str(tmp_path / "x.png")
    g.save_png(p, img, flip)
    back = _read_png(p)
    assert np.array_equal(back, img[::-1] if flip else img)


def test_raw_ply_loads_as_from_raw(tmp_path):
    """scenes.write_raw_ply (bench.py's C++ facade scene): the loader's activations of the raw
    fields equal gs_activate's of the same fields (Splats(path) == Splats.from_raw) bit for bit"""
    import openglgaussiansplattingrenderer_amd as g
    from openglgaussiansplattingrenderer_amd.scenes import bicycle_standin_raw, write_raw_ply
    means, f_dc, logit, log_sc, rot = bicycle_standin_raw(5000, seed=9)
    p = str(tmp_path / "raw.ply")
    write_raw_ply(p, means, f_dc, logit, log_sc, rot)
    m4, cols, op, sc, r4 = g.load_ply(p)
    cols2, op2, sc2, r42 = g.activate(f_dc, logit, log_sc, rot)
    assert np.array_equal(m4[:, :3], means) and np.array_equal(cols, cols2) and np.array_equal(op, op2)
    assert np.array_equal(sc, sc2) and np.array_equal(r4, r42)
