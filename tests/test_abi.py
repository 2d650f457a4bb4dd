"""CPU-side checks of the C ABI: the library loads, exports every symbol the header
declares, and its host-only entry points (sizes, argument validation, error
strings) behave — no kernel is launched here."""
import ctypes
import os
import re

import pytest
import torch  # noqa: F401  (load order: torch's HIP runtime first)

from monodepth2_amd import _lib
from monodepth2_amd.build import INCLUDE, LIB_PATH, build
from monodepth2_amd.hotpath import HotPathConfig


@pytest.fixture(scope="module")
def L():
    build()
    return _lib.lib()


def header_symbols():
    src = open(os.path.join(INCLUDE, "md2hot.h")).read()
    return sorted(set(re.findall(r"\b(md2_[a-z0-9_]+)\s*\(", src)))


def test_exports_match_header(L):
    syms = header_symbols()
    assert set(syms) == set(_lib.EXPORTS)
    for s in syms:
        assert hasattr(L, s), s


def test_abi_version(L):
    assert L.md2_abi_version() == _lib.ABI_VERSION


def test_build_id_matches_tree(L):
    """the in-tree library is the build of these sources (a stale prebuilt .so of the
    same ABI would be refused by _lib.lib())"""
    from monodepth2_amd.build import source_hash
    assert L.md2_build_id().decode() == source_hash()


def test_struct_sizes():
    assert ctypes.sizeof(_lib.Desc) == 48
    # disp[4], color[4][4], K[4], inv_K[4], T, noise, seed_ptr, mask, src8 (ABI 20)
    assert ctypes.sizeof(_lib.Tensors) == 8 * (4 + 16 + 4 + 4 + 5)
    # weight, planes_fwd, planes_dgrad, 4 x int32, planes_col (ABI 19)
    assert ctypes.sizeof(_lib.WsplitEntry) == 48 and _lib.WsplitEntry.planes_col.offset == 40


@pytest.mark.parametrize("B,H,W,S", [(12, 192, 640, 2), (8, 320, 1024, 2), (12, 192, 640, 3), (1, 32, 32, 1)])
def test_workspace_sizes(L, B, H, W, S):
    cfg = HotPathConfig(batch=B, height=H, width=W, num_src=S)
    d = cfg.desc()
    ws = L.md2_workspace_bytes(ctypes.byref(d))
    assert ws > 0 and ws % 256 == 0
    # the per-scale full-resolution gradient buffers dominate: 4 * B*H*W floats
    assert ws >= 4 * B * H * W * 4
    assert L.md2_select_bytes(ctypes.byref(d)) == 4 * B * H * W


def test_v1_select_bytes(L):
    cfg = HotPathConfig(batch=2, height=64, width=128, num_src=2, v1_multiscale=True)
    d = cfg.desc()
    assert L.md2_select_bytes(ctypes.byref(d)) == sum(2 * (64 >> s) * (128 >> s) for s in range(4))


@pytest.mark.parametrize("kw,msg", [
    (dict(batch=0, height=64, width=64, num_src=2), "batch"),
    (dict(batch=1, height=60, width=64, num_src=2), "divisible"),
    (dict(batch=1, height=64, width=64, num_src=4), "num_src"),
    (dict(batch=1, height=64, width=64, num_src=2, num_scales=5), "num_scales"),
    (dict(batch=1, height=16, width=16, num_src=2), "coarsest"),
])
def test_invalid_desc(L, kw, msg):
    d = HotPathConfig(**kw).desc()
    assert L.md2_workspace_bytes(ctypes.byref(d)) == 0
    assert msg in L.md2_last_error().decode()


def test_fwd_rejects_null_operands(L):
    d = HotPathConfig(batch=1, height=64, width=64, num_src=2).desc()
    t = _lib.Tensors()
    rc = L.md2_photometric_fwd(ctypes.byref(d), ctypes.byref(t), None, None, None, None)
    assert rc == -1
    assert "NULL" in L.md2_last_error().decode()


def test_product_path_has_no_cpu_fallback():
    from monodepth2_amd.hotpath import photometric_loss
    cfg = HotPathConfig(batch=1, height=32, width=32, num_src=1)
    T = torch.eye(4).view(1, 1, 4, 4)
    with pytest.raises(RuntimeError, match="GPU only"):
        photometric_loss(cfg, [torch.rand(1, 1, 32 >> s, 32 >> s) for s in range(4)], None, None, None, T)


def test_src8_contract_check():
    """hotpath.check_src8 (MD2_CHECK_SRC8=1): 8-bit copies that no longer match the
    fp32 colours are refused (colours edited after packing)."""
    import torch
    from monodepth2_amd.data import pack_rgbx
    from monodepth2_amd.hotpath import check_src8
    g = torch.Generator().manual_seed(0)
    cols = [torch.randint(0, 256, (2, 3, 4, 6), generator=g).float() / 255.0 for _ in range(2)]
    s8 = pack_rgbx(cols)
    check_src8(s8, cols)
    edited = [c.clone() for c in cols]
    edited[1][0, 2, 3, 5] = (edited[1][0, 2, 3, 5] * 255 + 1) % 256 / 255.0
    with pytest.raises(ValueError, match="frame 1"):
        check_src8(s8, edited)
