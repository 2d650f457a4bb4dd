"""ctypes binding of the C ABI in include/md2hot.h (libmd2hot.so).

There is deliberately no fallback: if the library is missing or fails to load,
`lib()` raises.  The library must be loaded after `import torch` so that its
libamdhip64.so.7 dependency resolves to the HIP runtime torch already loaded.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

from .build import LIB_PATH as _BUILT_LIB
from .build import source_hash

# MD2_LIB overrides the library path (A/B runs of alternative builds: their build id
# is not checked against the tree)
LIB_PATH = os.environ.get("MD2_LIB", _BUILT_LIB)

MAX_SCALES = 4
MAX_SRC = 3
ABI_VERSION = 23

NO_SSIM = 1 << 0
AVG_REPROJECTION = 1 << 1
NO_AUTOMASK = 1 << 2
V1_MULTISCALE = 1 << 3
T_PER_SCALE = 1 << 4
PREDICTIVE_MASK = 1 << 5

_vp = ctypes.c_void_p


class Desc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
                ("num_src", ctypes.c_int32), ("num_scales", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("min_depth", ctypes.c_float), ("max_depth", ctypes.c_float),
                ("disparity_smoothness", ctypes.c_float), ("disp_dtype", ctypes.c_uint32),
                ("seed", ctypes.c_uint64)]


class Tensors(ctypes.Structure):
    _fields_ = [("disp", _vp * MAX_SCALES),
                ("color", (_vp * (1 + MAX_SRC)) * MAX_SCALES),
                ("K", _vp * MAX_SCALES),
                ("inv_K", _vp * MAX_SCALES),
                ("T", _vp),
                ("noise", _vp),
                ("seed_ptr", _vp),
                ("mask", _vp),
                ("src8", _vp)]


_lock = threading.Lock()
_lib = None

EXPORTS = ["md2_abi_version", "md2_last_error", "md2_workspace_bytes", "md2_select_bytes",
           "md2_photometric_fwd", "md2_photometric_bwd", "md2_generate_images", "md2_tiebreak_noise",
           "md2_timing_begin", "md2_timing_end", "md2_timing_calls", "md2_decoder_pad_fwd", "md2_decoder_pad_bwd",
           "md2_decoder_pad_workspace_bytes", "md2_adam_step", "md2_adam_step_dev", "md2_adam_hyper", "md2_adam_apply_dev", "md2_encoder_input",
           "md2_pose_fwd", "md2_pose_bwd", "md2_aug_plan_create", "md2_aug_plan_destroy", "md2_aug_run",
           "md2_bn_workspace_bytes", "md2_bn_fwd", "md2_bn_bwd", "md2_maxpool3s2_fwd", "md2_maxpool3s2_bwd",
           "md2_disp_head_workspace_bytes", "md2_disp_head_fwd", "md2_disp_head_bwd",
           "md2_stem_wgrad_workspace_bytes", "md2_stem_wgrad", "md2_stem_fwd", "md2_conv_col2im", "md2_bias_act_fwd", "md2_bias_act_bwd",
           "md2_bias_act_workspace_bytes", "md2_maxpool3s2_bwd_add", "md2_bn_bwd_multi",
           "md2_conv_fwd", "md2_conv_workspace_bytes", "md2_conv_split_weights",
           "md2_conv_dgrad", "md2_conv_wgrad", "md2_conv_direct", "md2_conv_wgrad_direct",
           "md2_conv_wgrad_direct_workspace_bytes", "md2_conv_split_weights_multi", "md2_bn_fwd_mask",
           "md2_bn_bwd_mask", "md2_build_id", "md2_maxpool3s2_bwd_multi", "md2_decoder_pad_bwd2", "md2_aug_run2",
           "md2_conv_bf16_weights", "md2_conv_bf16_weights_multi"]

DTYPE_F32 = 0    # md2_desc.disp_dtype
DTYPE_BF16 = 1
PAD_ELU = 1 << 0
PAD_UPSAMPLE = 1 << 1
PAD_NHWC = 1 << 2
PAD_BF16 = 1 << 3


class PadDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("channels", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("skip_channels", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class AugDesc(ctypes.Structure):
    _fields_ = [("items", ctypes.c_int32), ("frames", ctypes.c_int32), ("in_height", ctypes.c_int32),
                ("in_width", ctypes.c_int32), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
                ("num_scales", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class AugItem(ctypes.Structure):
    _fields_ = [("flip", ctypes.c_uint8), ("color_aug", ctypes.c_uint8), ("hue_shift", ctypes.c_uint8),
                ("reserved", ctypes.c_uint8), ("order", ctypes.c_uint8 * 4), ("brightness", ctypes.c_float),
                ("contrast", ctypes.c_float), ("saturation", ctypes.c_float)]


BN_RELU = 1 << 0
BN_RESIDUAL = 1 << 1
BN_BF16 = 1 << 2


class BnDesc(ctypes.Structure):
    _fields_ = [("pixels", ctypes.c_int64), ("channels", ctypes.c_int32), ("flags", ctypes.c_uint32),
                ("eps", ctypes.c_float), ("momentum", ctypes.c_float), ("groups", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


POOL_BF16 = 1 << 0


CONV_NO_SPLIT = 1 << 1
CONV_TILE_N32 = 1 << 2
CONV_TILE_N64 = 1 << 3
CONV_TILE_N128 = 1 << 4
CONV_X6 = 1 << 5
CONV_BM256 = 1 << 6
CONV_PRESPLIT = 1 << 7
CONV_PATCH = 1 << 8
CONV_S2_ONE = 1 << 9
CONV_WS = 1 << 10
CONV_BF16 = 1 << 11   # ABI 22: bf16 operands (autocast convolutions, config C5)


class ConvDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("height", ctypes.c_int32), ("width", ctypes.c_int32),
                ("in_channels", ctypes.c_int32), ("out_channels", ctypes.c_int32), ("kernel_h", ctypes.c_int32),
                ("kernel_w", ctypes.c_int32), ("stride", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("flags", ctypes.c_uint32)]


class WsplitEntry(ctypes.Structure):
    """include/md2hot.h md2_wsplit_entry (one weight of md2_conv_split_weights_multi)."""
    _fields_ = [("weight", _vp), ("planes_fwd", _vp), ("planes_dgrad", _vp), ("co", ctypes.c_int32),
                ("kt", ctypes.c_int32), ("ci", ctypes.c_int32), ("block0", ctypes.c_int32), ("planes_col", _vp)]


class PoolDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("channels", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("flags", ctypes.c_uint32), ("reserved", ctypes.c_int32)]


HEAD_WEIGHT_CL = 1 << 0
HEAD_BF16 = 1 << 1   # ABI 23: bf16 padded input / its gradient


class HeadDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("channels", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("flags", ctypes.c_uint32)]


STEM_WEIGHT_CL = 1 << 0
STEM_BF16 = 1 << 1   # ABI 23: md2_stem_wgrad on bf16 x / grad_y


class StemDesc(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int32), ("channels", ctypes.c_int32), ("height", ctypes.c_int32),
                ("width", ctypes.c_int32), ("flags", ctypes.c_uint32)]


BIAS_ACT_RELU = 1 << 0


class BiasActDesc(ctypes.Structure):
    _fields_ = [("pixels", ctypes.c_int64), ("channels", ctypes.c_int32), ("flags", ctypes.c_uint32)]


def _declare(L):
    L.md2_bias_act_fwd.restype = ctypes.c_int
    L.md2_bias_act_fwd.argtypes = [ctypes.POINTER(BiasActDesc)] + [_vp] * 4
    L.md2_bias_act_bwd.restype = ctypes.c_int
    L.md2_bias_act_bwd.argtypes = [ctypes.POINTER(BiasActDesc)] + [_vp] * 6
    L.md2_bias_act_workspace_bytes.restype = ctypes.c_size_t
    L.md2_bias_act_workspace_bytes.argtypes = [ctypes.POINTER(BiasActDesc)]
    L.md2_conv_fwd.restype = ctypes.c_int
    L.md2_conv_fwd.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 5
    L.md2_conv_dgrad.restype = ctypes.c_int
    L.md2_conv_dgrad.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 5
    L.md2_conv_wgrad.restype = ctypes.c_int
    L.md2_conv_wgrad.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 5
    L.md2_conv_split_weights.restype = ctypes.c_int
    L.md2_conv_direct.restype = ctypes.c_int
    L.md2_conv_direct.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 4
    L.md2_conv_wgrad_direct.restype = ctypes.c_int
    L.md2_conv_wgrad_direct.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 5
    L.md2_conv_wgrad_direct_workspace_bytes.restype = ctypes.c_size_t
    L.md2_conv_wgrad_direct_workspace_bytes.argtypes = [ctypes.POINTER(ConvDesc)]
    L.md2_conv_split_weights.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 4
    L.md2_conv_split_weights_multi.restype = ctypes.c_int
    L.md2_conv_split_weights_multi.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
    L.md2_conv_bf16_weights.restype = ctypes.c_int
    L.md2_conv_bf16_weights.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 4
    L.md2_conv_bf16_weights_multi.restype = ctypes.c_int
    L.md2_conv_bf16_weights_multi.argtypes = [_vp, ctypes.c_int, ctypes.c_int, _vp]
    L.md2_conv_workspace_bytes.restype = ctypes.c_size_t
    L.md2_conv_workspace_bytes.argtypes = [ctypes.POINTER(ConvDesc)]
    L.md2_stem_wgrad_workspace_bytes.restype = ctypes.c_size_t
    L.md2_stem_wgrad_workspace_bytes.argtypes = [ctypes.POINTER(StemDesc)]
    L.md2_stem_wgrad.restype = ctypes.c_int
    L.md2_stem_wgrad.argtypes = [ctypes.POINTER(StemDesc)] + [_vp] * 5
    L.md2_stem_fwd.restype = ctypes.c_int
    L.md2_conv_col2im.restype = ctypes.c_int
    L.md2_conv_col2im.argtypes = [ctypes.POINTER(ConvDesc)] + [_vp] * 3
    L.md2_stem_fwd.argtypes = [ctypes.POINTER(StemDesc)] + [_vp] * 4
    L.md2_disp_head_workspace_bytes.restype = ctypes.c_size_t
    L.md2_disp_head_workspace_bytes.argtypes = [ctypes.POINTER(HeadDesc)]
    L.md2_disp_head_fwd.restype = ctypes.c_int
    L.md2_disp_head_fwd.argtypes = [ctypes.POINTER(HeadDesc)] + [_vp] * 5
    L.md2_disp_head_bwd.restype = ctypes.c_int
    L.md2_disp_head_bwd.argtypes = [ctypes.POINTER(HeadDesc)] + [_vp] * 9
    L.md2_abi_version.restype = ctypes.c_int
    L.md2_abi_version.argtypes = []
    L.md2_build_id.restype = ctypes.c_char_p
    L.md2_build_id.argtypes = []
    L.md2_last_error.restype = ctypes.c_char_p
    L.md2_last_error.argtypes = []
    L.md2_workspace_bytes.restype = ctypes.c_size_t
    L.md2_workspace_bytes.argtypes = [ctypes.POINTER(Desc)]
    L.md2_select_bytes.restype = ctypes.c_size_t
    L.md2_select_bytes.argtypes = [ctypes.POINTER(Desc)]
    L.md2_photometric_fwd.restype = ctypes.c_int
    L.md2_photometric_fwd.argtypes = [ctypes.POINTER(Desc), ctypes.POINTER(Tensors), _vp, _vp, _vp, _vp]
    L.md2_photometric_bwd.restype = ctypes.c_int
    L.md2_photometric_bwd.argtypes = [ctypes.POINTER(Desc), ctypes.POINTER(Tensors), _vp, _vp,
                                      ctypes.POINTER(_vp), _vp, _vp, _vp, _vp]
    L.md2_generate_images.restype = ctypes.c_int
    L.md2_generate_images.argtypes = [ctypes.POINTER(Desc), ctypes.POINTER(Tensors),
                                      ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp]
    L.md2_tiebreak_noise.restype = ctypes.c_int
    L.md2_tiebreak_noise.argtypes = [ctypes.POINTER(Desc), _vp, ctypes.c_int, _vp, _vp]
    L.md2_decoder_pad_fwd.restype = ctypes.c_int
    L.md2_decoder_pad_fwd.argtypes = [ctypes.POINTER(PadDesc), _vp, _vp, _vp, _vp, _vp]
    L.md2_decoder_pad_bwd.restype = ctypes.c_int
    L.md2_decoder_pad_bwd.argtypes = [ctypes.POINTER(PadDesc), _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.md2_decoder_pad_bwd2.restype = ctypes.c_int
    L.md2_decoder_pad_bwd2.argtypes = [ctypes.POINTER(PadDesc)] + [_vp] * 9
    L.md2_encoder_input.restype = ctypes.c_int
    L.md2_encoder_input.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, _vp,
                                    ctypes.c_float, ctypes.c_float, _vp, _vp]
    L.md2_adam_step.restype = ctypes.c_int
    L.md2_adam_step.argtypes = [_vp, _vp, ctypes.c_int, _vp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                ctypes.c_double, ctypes.c_int, _vp]
    L.md2_adam_step_dev.restype = ctypes.c_int
    L.md2_adam_step_dev.argtypes = [_vp, _vp, ctypes.c_int, _vp, _vp, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, _vp, _vp, _vp]
    L.md2_adam_hyper.restype = ctypes.c_int
    L.md2_adam_hyper.argtypes = [_vp, ctypes.c_double, ctypes.c_double, _vp, _vp, _vp]
    L.md2_adam_apply_dev.restype = ctypes.c_int
    L.md2_adam_apply_dev.argtypes = [_vp, _vp, ctypes.c_int, ctypes.c_int, _vp, ctypes.c_double, ctypes.c_double,
                                     ctypes.c_double, _vp, _vp]
    L.md2_decoder_pad_workspace_bytes.restype = ctypes.c_size_t
    L.md2_decoder_pad_workspace_bytes.argtypes = [ctypes.POINTER(PadDesc)]
    L.md2_pose_fwd.restype = ctypes.c_int
    L.md2_pose_fwd.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _vp, _vp, _vp, _vp]
    L.md2_pose_bwd.restype = ctypes.c_int
    L.md2_pose_bwd.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _vp, _vp, _vp, _vp, _vp, _vp]
    L.md2_aug_plan_create.restype = _vp
    L.md2_aug_plan_create.argtypes = [ctypes.POINTER(AugDesc)]
    L.md2_aug_plan_destroy.restype = None
    L.md2_aug_plan_destroy.argtypes = [_vp]
    L.md2_aug_run.restype = ctypes.c_int
    L.md2_aug_run.argtypes = [_vp, _vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp]
    L.md2_aug_run2.restype = ctypes.c_int
    L.md2_aug_run2.argtypes = [_vp, _vp, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _vp, _vp]
    L.md2_bn_workspace_bytes.restype = ctypes.c_size_t
    L.md2_bn_workspace_bytes.argtypes = [ctypes.POINTER(BnDesc)]
    L.md2_bn_fwd.restype = ctypes.c_int
    L.md2_bn_fwd.argtypes = [ctypes.POINTER(BnDesc)] + [_vp] * 11
    L.md2_bn_bwd.restype = ctypes.c_int
    L.md2_bn_bwd.argtypes = [ctypes.POINTER(BnDesc)] + [_vp] * 12
    L.md2_maxpool3s2_fwd.restype = ctypes.c_int
    L.md2_maxpool3s2_fwd.argtypes = [ctypes.POINTER(PoolDesc), _vp, _vp, _vp, _vp]
    L.md2_maxpool3s2_bwd.restype = ctypes.c_int
    L.md2_maxpool3s2_bwd.argtypes = [ctypes.POINTER(PoolDesc), _vp, _vp, _vp, _vp]
    L.md2_bn_bwd_multi.restype = ctypes.c_int
    L.md2_bn_bwd_multi.argtypes = [ctypes.POINTER(BnDesc)] + [_vp] * 14
    L.md2_bn_fwd_mask.restype = ctypes.c_int
    L.md2_bn_fwd_mask.argtypes = [ctypes.POINTER(BnDesc)] + [_vp] * 12
    L.md2_bn_bwd_mask.restype = ctypes.c_int
    L.md2_bn_bwd_mask.argtypes = [ctypes.POINTER(BnDesc)] + [_vp] * 14
    L.md2_maxpool3s2_bwd_add.restype = ctypes.c_int
    L.md2_maxpool3s2_bwd_add.argtypes = [ctypes.POINTER(PoolDesc)] + [_vp] * 5
    L.md2_maxpool3s2_bwd_multi.restype = ctypes.c_int
    L.md2_maxpool3s2_bwd_multi.argtypes = [ctypes.POINTER(PoolDesc)] + [_vp] * 6
    L.md2_timing_begin.restype = ctypes.c_int
    L.md2_timing_begin.argtypes = [ctypes.c_int]
    L.md2_timing_calls.restype = ctypes.c_int
    L.md2_timing_calls.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                   ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]
    L.md2_timing_end.restype = ctypes.c_int
    L.md2_timing_end.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int),
                                 ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]


def lib():
    """The loaded library; raises RuntimeError if it is not built or not loadable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"{LIB_PATH} is not built. Build it with `python -m monodepth2_amd.build` "
                    "(hipcc --offload-arch=gfx950); there is no CPU fallback.")
            L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
            _declare(L)
            v = L.md2_abi_version()
            if v != ABI_VERSION:
                raise RuntimeError(f"libmd2hot ABI {v} != expected {ABI_VERSION}")
            if LIB_PATH == _BUILT_LIB:
                got, want = L.md2_build_id().decode(), source_hash()
                if got != want:
                    raise RuntimeError(
                        f"{LIB_PATH} was built from other sources (build id {got}, tree {want}): "
                        "rebuild it with `python -m monodepth2_amd.build`")
            _lib = L
    return _lib


def stream(device) -> int:
    """The raw hipStream_t of `device`'s current stream (what torch.cuda.current_stream(
    device).cuda_stream returns, without building a Stream object: ~10x cheaper on the
    host, and this is called for every kernel the step launches)."""
    idx = device.index if isinstance(device, torch.device) else device
    return torch._C._cuda_getCurrentRawStream(torch.cuda.current_device() if idx is None else idx)


def check(rc: int, what: str):
    if rc != 0:
        msg = lib().md2_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed ({rc}): {msg}")


class KernelTimer:
    """Context manager around md2_timing_begin/end: average photo-kernel durations."""

    def __init__(self, max_launches: int = 4096):
        self.max_launches = max_launches
        self.fwd_ms = self.bwd_ms = 0.0
        self.n_fwd = self.n_bwd = 0

    def __enter__(self):
        check(lib().md2_timing_begin(self.max_launches), "md2_timing_begin")
        return self

    def __exit__(self, *exc):
        f, b = ctypes.c_double(), ctypes.c_double()
        nf, nb = ctypes.c_int(), ctypes.c_int()
        check(lib().md2_timing_end(ctypes.byref(f), ctypes.byref(nf), ctypes.byref(b), ctypes.byref(nb)),
              "md2_timing_end")
        self.fwd_ms, self.n_fwd, self.bwd_ms, self.n_bwd = f.value, nf.value, b.value, nb.value
        check(lib().md2_timing_calls(ctypes.byref(f), ctypes.byref(nf), ctypes.byref(b), ctypes.byref(nb)),
              "md2_timing_calls")
        self.fwd_call_ms, self.n_fwd_call, self.bwd_call_ms, self.n_bwd_call = f.value, nf.value, b.value, nb.value
        return False
