"""CPU: the C-ABI library builds, loads, exports exactly what include/segamd.h
declares, and the ctypes prototypes match the header's parameter types."""
import ctypes
import os
import re

import pytest

from seg_amd import _lib
from seg_amd.build import LIB_PATH, build

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "segamd.h")

CTYPE = {"const float*": ctypes.c_void_p, "float*": ctypes.c_void_p, "const long long*": ctypes.c_void_p,
         "long long*": ctypes.c_void_p, "int*": ctypes.c_void_p, "const void*": ctypes.c_void_p, "const seg_bf16*": ctypes.c_void_p, "seg_bf16*": ctypes.c_void_p, "const unsigned char*": ctypes.c_void_p, "unsigned char*": ctypes.c_void_p, "hipStream_t": ctypes.c_void_p, "const SegAdamTensor*": ctypes.c_void_p, "const long*": ctypes.c_void_p, "long": ctypes.c_long, "void*": ctypes.c_void_p, "void**": ctypes.c_void_p, "const int*": ctypes.c_void_p, "unsigned*": ctypes.c_void_p,
         "const char*": ctypes.c_char_p, "char*": ctypes.c_char_p, "long*": ctypes.c_void_p,
         "int": ctypes.c_int, "float": ctypes.c_float}


def header_decls():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    decls = {}
    for m in re.finditer(r"\b(int|long)\s+(seg_\w+)\s*\(([^)]*)\)\s*;", text):
        ret, name, params = m.group(1), m.group(2), m.group(3)
        types = []
        for prm in ([] if params.strip() in ("", "void") else params.split(",")):
            prm = " ".join(prm.split())
            t = re.sub(r"\s*\b\w+$", "", prm).replace(" *", "*")
            types.append(t)
        decls[name] = (ret, types)
    return decls


@pytest.fixture(scope="module")
def lib():
    build()
    return _lib.lib()


def test_header_matches_prototypes():
    decls = header_decls()
    assert set(decls) == set(_lib.PROTOTYPES), set(decls) ^ set(_lib.PROTOTYPES)
    for name, (ret, types) in decls.items():
        res, args = _lib.PROTOTYPES[name]
        assert res == (ctypes.c_int if ret == "int" else ctypes.c_long), name
        assert [CTYPE[t] for t in types] == args, name


def test_library_exports_every_symbol(lib):
    assert os.path.exists(LIB_PATH)
    for name in header_decls():
        assert hasattr(lib, name), name


def test_host_side_queries(lib):
    # pure host functions: callable without a GPU
    s = _lib.query("seg_conv_wgrad_splits", 32 * 16 * 32, 256, 1344, 3)
    assert 1 <= s <= 256
    assert _lib.query("seg_conv_wgrad_splits", 10, 32, 32, 3) == 1
    assert _lib.query("seg_chan_workspace_floats", 1 << 20, 96) >= 2 * 96
    assert _lib.query("seg_dw_wgrad_blocks", 32, 128, 256, 32) >= 1
    assert _lib.query("seg_ce_workspace_floats", 4 * 256 * 512) >= 2
    # split-K only when the output tiles cannot fill the chip
    assert _lib.query("seg_conv_igemm_splits", 32 * 128 * 256, 32, 80, 3) == 1
    assert _lib.query("seg_conv_igemm_splits", 8 * 16, 256, 1344, 3) > 1
    # the all-points Winograd weight gradient: every dense 3x3 decoder shape >= 32 channels, every split non-empty
    for N, H, W, Cin, Cout in ((32, 128, 256, 32, 32), (32, 128, 256, 80, 32), (32, 16, 32, 1344, 256),
                               (8, 512, 1024, 64, 64), (8, 64, 128, 512, 512), (2, 4, 4, 32, 32)):
        assert _lib.query("seg_conv_wino_wgrad_pick", N, H, W, Cin, Cout) == 2
        sp = _lib.query("seg_conv_wino_wgrad16_splits", N, H, W, Cin, Cout)
        T = N * (H // 2) * (W // 2)
        chunk = -(-(-(-T // sp)) // 16) * 16
        assert 1 <= sp <= 1024 and -(-T // chunk) == sp, (N, H, W, Cin, Cout, sp)
    assert _lib.query("seg_conv_wino_wgrad_pick", 8, 512, 1024, 4, 64) == 0  # UNet inc.0 (3 -> 64): direct
    import ctypes
    plan = (ctypes.c_int * 3)()
    for args, want in (((32 * 128 * 256, 32, 80, 3), (1, -1)), ((8 * 16, 256, 1344, 3), (32, 12)),
                       ((64 * 128, 32, 32, 3), (1, 3)), ((4 * 8, 1280, 320, 1), (1, 3))):
        assert _lib.query("seg_conv_igemm_plan_b1", *args, ctypes.addressof(plan)) == 0
        assert tuple(plan[:2]) == want, (args, list(plan))


def test_argument_validation_without_gpu(lib):
    # invalid arguments are rejected before any launch (hipErrorInvalidValue == 1)
    rc = lib.seg_conv_igemm(None, 3, 1, 4, 4, 3, None, 4, None, None, 4, 4, 4, 8, 3, 1, 1, None, 0, None, None)
    assert rc == 1  # Cin % 4 != 0
    rc = lib.seg_nchw_to_nhwc(None, 1, 3, 4, 4, None, 2, None)
    assert rc == 1  # ld < C
    rc = lib.seg_conv_wgrad_reduce(None, 1, None, 4, 4, 3, 2, 0, None)
    assert rc == 1  # unknown mode
    rc = lib.seg_conv_igemm_act(None, 4, 1, 4, 4, 4, None, 36, None, None, 4, 4, 4, 8, 3, 1, 1, None, 0, None, 3, None, 1,
                                None)
    assert rc == 1  # unknown activation
    rc = lib.seg_preprocess_bgr(None, 1, 720, 1280, 1280, None, 4, 128, 256, 0, 0, 0, 1, 1, 1, None)
    assert rc == 1  # row_bytes < 3 * Wf
    rc = lib.seg_argmax_nearest(None, 10, 1, 64, 128, 10, 128, 256, None, 720, 1280, None)
    assert rc == 1  # ld not a multiple of 4


def test_build_hash_decides_staleness(lib):
    """The library carries the source hash it was built from; build() relinks exactly when
    the tree's hash differs (not by file times) and the binding refuses a mismatch."""
    from seg_amd import build as b
    buf = ctypes.create_string_buffer(80)
    assert lib.seg_build_hash(buf, 80) == 64
    assert buf.value.decode() == b.source_hash() == b.library_hash()
    os.utime(LIB_PATH, (1, 1))  # an old mtime alone must not trigger a rebuild
    before = open(LIB_PATH, "rb").read()
    build()
    assert open(LIB_PATH, "rb").read() == before
