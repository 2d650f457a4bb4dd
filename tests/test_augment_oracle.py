"""Pins oracle/augment_oracle.py (the CPU restatement of the reference's PIL input
pipeline, datasets/mono_dataset.py:90-200) bit-exactly to the installed Pillow, and
checks the host-side draw logic of monodepth2_amd/augment.py (no GPU needed).

Pillow is the library the reference's transforms call (torchvision 0.2.1 is not
installed here; its PIL code paths are written out in augment_oracle.pil_jitter)."""
import ctypes
import random

import numpy as np
import pytest

from oracle import augment_oracle as A

PIL = pytest.importorskip("PIL.Image")


def _all_colours():
    g = np.arange(256, dtype=np.uint8)
    return np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(4096, 4096, 3)


def test_gray_hsv_exhaustive():
    img = _all_colours()
    pim = PIL.fromarray(img)
    np.testing.assert_array_equal(A.to_gray(img), np.asarray(pim.convert("L")))
    np.testing.assert_array_equal(A.rgb_to_hsv(img), np.asarray(pim.convert("HSV")))
    np.testing.assert_array_equal(A.hsv_to_rgb(img), np.asarray(PIL.fromarray(img, "HSV").convert("RGB")))


def _texture(rng, h, w):
    x = rng.random((h // 4 + 2, w // 4 + 2, 3)) * 255
    img = np.asarray(PIL.fromarray(x.astype(np.uint8)).resize((w, h), PIL.Resampling.BICUBIC))
    return np.clip(img.astype(np.int32) + rng.integers(-20, 21, img.shape), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("src,dst", [((375, 1242), (192, 640)), ((192, 640), (96, 320)), ((24, 80), (12, 40)),
                                     ((100, 300), (128, 416)), ((37, 53), (37, 53)), ((64, 64), (17, 91)),
                                     ((5, 7), (3, 2))])
def test_lanczos_resize_matches_pillow(src, dst):
    img = _texture(np.random.default_rng(sum(src) + sum(dst)), *src)
    np.testing.assert_array_equal(A.resize_lanczos(img, *dst), A.pil_resize(img, *dst))


def test_hue_shift_wraps_like_numpy1():
    assert [A.hue_shift_u8(v) for v in (-0.1, -0.05, 0.05, 0.1, 0.0)] == [231, 244, 12, 25, 0]


def test_color_jitter_matches_pillow():
    rng = np.random.default_rng(7)
    img = _texture(rng, 48, 160)
    for trial in range(40):
        order = list(rng.permutation(4))
        b, c, s = rng.uniform(0.8, 1.2, 3)
        h = rng.uniform(-0.1, 0.1)
        np.testing.assert_array_equal(A.color_jitter(img, order, b, c, s, h), A.pil_jitter(img, order, b, c, s, h),
                                      err_msg=f"order={order} b={b} c={c} s={s} h={h}")


def test_blend_edges_match_pillow():
    img = _all_colours()[::16, ::16].copy()
    for f in (0.0, 1.0, 0.5, 1.2, 0.8, 1.0000001, 2.5):
        np.testing.assert_array_equal(A.brightness(img, f), A.pil_jitter(img, [0], f, 1, 1, 0))
        np.testing.assert_array_equal(A.saturation(img, f), A.pil_jitter(img, [2], 1, 1, f, 0))
        np.testing.assert_array_equal(A.contrast(img, f), A.pil_jitter(img, [1], 1, f, 1, 0))


def test_preprocess_matches_pillow_pipeline():
    """Flip (kitti_dataset.py:58-63) -> cascaded resize -> to_tensor / jitter."""
    rng = np.random.default_rng(3)
    native = _texture(rng, 375, 1242)
    jit = ([2, 0, 3, 1], 1.13, 0.86, 1.05, -0.07)
    color, aug = A.preprocess(native, 192, 640, 4, flip=True, jitter=jit)
    img = PIL.fromarray(native).transpose(PIL.Transpose.FLIP_LEFT_RIGHT)
    for s in range(4):
        img = img.resize((640 >> s, 192 >> s), PIL.Resampling.LANCZOS)
        arr = np.asarray(img)
        np.testing.assert_array_equal(color[s], arr.transpose(2, 0, 1).astype(np.float32) / np.float32(255))
        np.testing.assert_array_equal(aug[s], A.pil_jitter(arr, *jit).transpose(2, 0, 1).astype(np.float32)
                                      / np.float32(255))


def test_draw_order_follows_reference():
    """do_color_aug, do_flip, then b, c, s, h uniforms and one shuffle of 4."""
    from monodepth2_amd.augment import draw_item, hue_shift
    r1, r2 = random.Random(11), random.Random(11)
    for _ in range(50):
        d = draw_item(r1)
        aug = r2.random() > 0.5
        flip = r2.random() > 0.5
        assert (d.do_color_aug, d.do_flip) == (aug, flip)
        if aug:
            vals = [r2.uniform(0.8, 1.2) for _ in range(3)] + [r2.uniform(-0.1, 0.1)]
            order = [0, 1, 2, 3]
            r2.shuffle(order)
            assert [d.brightness, d.contrast, d.saturation, d.hue] == vals and d.order == order
            assert hue_shift(d.hue) == A.hue_shift_u8(d.hue)
    assert not draw_item(random.Random(0), is_train=False).do_flip


def test_item_struct_layout():
    from monodepth2_amd import _lib
    from monodepth2_amd.augment import ItemDraw, pack_items
    assert ctypes.sizeof(_lib.AugItem) == 20 and ctypes.sizeof(_lib.AugDesc) == 32
    t = pack_items([ItemDraw(True, True, 1.1, 0.9, 1.0, -0.1, [3, 2, 1, 0])])
    raw = bytes(t)
    assert raw[:8] == bytes([1, 1, 231, 0, 3, 2, 1, 0])
    assert np.frombuffer(raw[8:], np.float32).tolist() == [np.float32(1.1), np.float32(0.9), 1.0]
