"""The fused photometric hot path as a torch.autograd.Function over the C ABI.

`photometric_loss(...)` replaces, forward and backward, everything
`Trainer.generate_images_pred` (trainer.py:341-391) and `Trainer.compute_losses`
(trainer.py:407-496) compute: upsample -> depth -> back-project -> project ->
border bilinear warp -> SSIM+L1 -> per-pixel min over identity/reprojection with
tie-break noise -> mean, plus edge-aware smoothness, for every scale.

Inputs are the reference's own tensors (no repacking): disparities per scale,
colour pyramids, K / inv_K and the stacked cam_T_cam.  Gradients flow to the
disparities and to T; colours, intrinsics and noise are constants (as in the
reference, where they never require grad).

There is no eager fallback: the library must be built and the tensors must be on
a ROCm device, otherwise this raises.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import torch

from . import _lib


@dataclass(frozen=True)
class HotPathConfig:
    """POD view of the `opt.*` fields the hot path reads (md2_desc)."""
    batch: int
    height: int
    width: int
    num_src: int
    num_scales: int = 4
    min_depth: float = 0.1
    max_depth: float = 100.0
    disparity_smoothness: float = 1e-3
    no_ssim: bool = False
    avg_reprojection: bool = False
    disable_automasking: bool = False
    v1_multiscale: bool = False
    t_per_scale: bool = False
    predictive_mask: bool = False

    @property
    def flags(self) -> int:
        f = 0
        f |= _lib.NO_SSIM if self.no_ssim else 0
        f |= _lib.AVG_REPROJECTION if self.avg_reprojection else 0
        f |= _lib.NO_AUTOMASK if self.disable_automasking else 0
        f |= _lib.V1_MULTISCALE if self.v1_multiscale else 0
        f |= _lib.T_PER_SCALE if self.t_per_scale else 0
        f |= _lib.PREDICTIVE_MASK if self.predictive_mask else 0
        return f

    def desc(self, seed: int = 0, disp_dtype: torch.dtype = torch.float32) -> _lib.Desc:
        dt = _lib.DTYPE_BF16 if disp_dtype == torch.bfloat16 else _lib.DTYPE_F32
        return _lib.Desc(self.batch, self.height, self.width, self.num_src, self.num_scales, self.flags,
                         self.min_depth, self.max_depth, self.disparity_smoothness, dt, seed & (2 ** 64 - 1))

    def loss_res(self, s: int):
        if self.v1_multiscale:
            return self.height >> s, self.width >> s
        return self.height, self.width

    def noise_channels(self) -> int:
        return 1 if self.avg_reprojection else self.num_src

    def noise_shape(self, s: int):
        h, w = self.loss_res(s)
        return (self.batch, self.noise_channels(), h, w)


def _stream_ptr(device: torch.device) -> int:
    return _lib.stream(device)


def _require(t: torch.Tensor, name: str, shape, device, dtypes=(torch.float32,)):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device != device:
        raise ValueError(f"{name} is on {t.device}, expected {device}")
    if t.dtype not in dtypes:
        raise ValueError(f"{name} must be {' or '.join(str(d) for d in dtypes)} (got {t.dtype})")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} has shape {tuple(t.shape)}, expected {tuple(shape)}")


def _capturing() -> bool:
    return torch.cuda.is_available() and torch.cuda.is_current_stream_capturing()


def check_src8(src8: torch.Tensor, sources: Sequence[torch.Tensor]) -> None:
    """The 8-bit contract of `src8` (photometric_loss): every packed channel k equals
    round(255 * colour) and the colour is exactly k/255.  The kernels trust it (the
    forward then skips its own exactness flags and reads only the 8-bit copies), so a
    pipeline that edits the colours after md2_aug_run2 / pack_rgbx must drop
    color_src8 from the batch.  MD2_CHECK_SRC8=1 runs this on every call (a debug
    check: one pass over the sources and a host sync)."""
    for fi, c in enumerate(sources):
        p = src8[fi].cpu()
        k = torch.stack([(p >> (8 * ch)) & 255 for ch in range(3)], 1).double()
        # on the host in float64, as data.pack_rgbx checks (exact k/255 rounded once)
        want = (k / 255.0).float()
        got = c.float().cpu()
        if not torch.equal(want, got):
            raise ValueError(f"color_src8 frame {fi} does not match the fp32 source colours "
                             f"({int((want != got).sum())} channels differ): drop color_src8 when the colours change")


class Operands:
    """The non-differentiable operands of one call, validated and made contiguous.

    colors[s][fi]: (B,3,H>>s,W>>s) with fi=0 the target and fi=1..S the sources;
    entries the configuration never reads may be None.  K / inv_K: per scale
    (B,4,4) (only scale 0 unless v1_multiscale).
    """

    def __init__(self, cfg: HotPathConfig, colors: Sequence[Sequence[Optional[torch.Tensor]]],
                 K: Sequence[Optional[torch.Tensor]], inv_K: Sequence[Optional[torch.Tensor]],
                 noise: Optional[Dict[int, torch.Tensor]], device: torch.device,
                 seed_tensor: Optional[torch.Tensor] = None, src8: Optional[torch.Tensor] = None):
        B, H, W, S = cfg.batch, cfg.height, cfg.width, cfg.num_src
        self.cfg = cfg
        self.src8 = None
        if src8 is not None and not cfg.v1_multiscale:   # (the v1 layout samples every scale's planes)
            if (src8.device != device or src8.dtype != torch.int32 or tuple(src8.shape) != (S, B, H, W)
                    or not src8.is_contiguous()):
                raise ValueError(f"src8 must be a contiguous int32 {(S, B, H, W)} tensor on {device}, got "
                                 f"{src8.dtype} {tuple(src8.shape)} on {src8.device}")
            self.src8 = src8
        if seed_tensor is not None and (seed_tensor.device != device or seed_tensor.dtype != torch.int64
                                        or seed_tensor.numel() != 1):
            raise ValueError("seed_tensor must be a 1-element int64 tensor on " + str(device))
        self.seed_tensor = seed_tensor
        self.colors: List[List[Optional[torch.Tensor]]] = [[None] * (1 + S) for _ in range(cfg.num_scales)]
        self.K: List[Optional[torch.Tensor]] = [None] * cfg.num_scales
        self.inv_K: List[Optional[torch.Tensor]] = [None] * cfg.num_scales
        for s in range(cfg.num_scales):
            shp = (B, 3, H >> s, W >> s)
            t = colors[s][0]
            _require(t, f"color[{s}][target]", shp, device)
            self.colors[s][0] = t.contiguous()
            if cfg.v1_multiscale or s == 0:
                for fi in range(1, S + 1):
                    t = colors[s][fi]
                    _require(t, f"color[{s}][{fi}]", shp, device)
                    self.colors[s][fi] = t.contiguous()
                _require(K[s], f"K[{s}]", (B, 4, 4), device)
                _require(inv_K[s], f"inv_K[{s}]", (B, 4, 4), device)
                self.K[s] = K[s].contiguous()
                self.inv_K[s] = inv_K[s].contiguous()
        if self.src8 is not None and os.environ.get("MD2_CHECK_SRC8") == "1" and not _capturing():
            check_src8(self.src8, [self.colors[0][fi] for fi in range(1, S + 1)])
        self.noise = None
        if noise is not None:
            parts = []
            for s in range(cfg.num_scales):
                _require(noise[s], f"noise[{s}]", cfg.noise_shape(s), device)
                parts.append(noise[s].reshape(-1))
            self.noise = torch.cat(parts).contiguous()

    def struct(self, disps: Sequence[torch.Tensor], T: torch.Tensor,
               mask: Optional[torch.Tensor] = None) -> _lib.Tensors:
        st = _lib.Tensors()
        for s, d in enumerate(disps):
            st.disp[s] = d.data_ptr()
        for s in range(self.cfg.num_scales):
            for fi, c in enumerate(self.colors[s]):
                if c is not None:
                    st.color[s][fi] = c.data_ptr()
            if self.K[s] is not None:
                st.K[s] = self.K[s].data_ptr()
                st.inv_K[s] = self.inv_K[s].data_ptr()
        st.T = T.data_ptr()
        st.noise = self.noise.data_ptr() if self.noise is not None else None
        st.seed_ptr = self.seed_tensor.data_ptr() if self.seed_tensor is not None else None
        st.mask = mask.data_ptr() if mask is not None else None
        st.src8 = self.src8.data_ptr() if self.src8 is not None else None
        return st


class _PhotometricLoss(torch.autograd.Function):

    @staticmethod
    def forward(ctx, cfg: HotPathConfig, ops: Operands, seed: int, T: torch.Tensor, mask, *disps: torch.Tensor):
        L = _lib.lib()
        dev = T.device
        desc = cfg.desc(seed, disps[0].dtype)
        st = ops.struct(disps, T, mask)
        ws = torch.empty(L.md2_workspace_bytes(ctypes.byref(desc)), dtype=torch.uint8, device=dev)
        sel = torch.empty(L.md2_select_bytes(ctypes.byref(desc)), dtype=torch.uint8, device=dev)
        loss = torch.empty(cfg.num_scales + 1, dtype=torch.float32, device=dev)
        _lib.check(L.md2_photometric_fwd(ctypes.byref(desc), ctypes.byref(st), loss.data_ptr(), sel.data_ptr(),
                                         ws.data_ptr(), _stream_ptr(dev)), "md2_photometric_fwd")
        ctx.has_mask = mask is not None
        ctx.save_for_backward(T, *(([mask] if mask is not None else []) + list(disps)))
        ctx.cfg, ctx.ops, ctx.seed, ctx.ws, ctx.sel = cfg, ops, seed, ws, sel
        ctx.mark_non_differentiable(sel)
        # no zero-filled gradient for the (non-differentiable, 1 byte per pixel and scale)
        # selection map: backward gets None for it — a 5.9 MB fill at B=12 between the
        # hot path's forward and backward, where both networks wait
        ctx.set_materialize_grads(False)
        return loss, sel

    @staticmethod
    def backward(ctx, grad_loss, _grad_sel):
        L = _lib.lib()
        T, *rest = ctx.saved_tensors
        mask = rest[0] if ctx.has_mask else None
        disps = rest[1:] if ctx.has_mask else rest
        cfg = ctx.cfg
        dev = T.device
        if grad_loss is None:
            grad_loss = torch.zeros(cfg.num_scales + 1, dtype=torch.float32, device=dev)
        grad_loss = grad_loss.contiguous().float()
        desc = cfg.desc(ctx.seed, disps[0].dtype)
        st = ctx.ops.struct(disps, T, mask)
        gdisp = [torch.empty_like(d) for d in disps]   # the disparities' dtype (bf16 written by the kernel)
        gT = torch.empty_like(T)
        gmask = torch.empty_like(mask) if mask is not None else None
        arr = (ctypes.c_void_p * _lib.MAX_SCALES)(*([g.data_ptr() for g in gdisp]
                                                    + [None] * (_lib.MAX_SCALES - len(gdisp))))
        _lib.check(L.md2_photometric_bwd(ctypes.byref(desc), ctypes.byref(st), grad_loss.data_ptr(),
                                         ctx.sel.data_ptr(), arr, gT.data_ptr(),
                                         gmask.data_ptr() if gmask is not None else None, ctx.ws.data_ptr(),
                                         _stream_ptr(dev)), "md2_photometric_bwd")
        return (None, None, None, gT, gmask, *gdisp)


def photometric_loss(cfg: HotPathConfig, disps: Sequence[torch.Tensor], colors, K, inv_K, T: torch.Tensor,
                     noise: Optional[Dict[int, torch.Tensor]] = None, seed: int = 0,
                     seed_tensor: Optional[torch.Tensor] = None,
                     mask: Optional[Dict[int, torch.Tensor]] = None,
                     src8: Optional[torch.Tensor] = None):
    """Fused hot path.  Returns (loss_vec, select).

    loss_vec[s] = losses["loss/s"], loss_vec[num_scales] = losses["loss"];
    select is the packed per-scale argmin map (uint8), see `selection_maps`.
    T: (S,B,4,4) stacked cam_T_cam (or (num_scales,S,B,4,4) with t_per_scale).
    noise: optional {scale: unit-normal (B,C,h,w)}; None draws it in-kernel from seed.
    seed_tensor: optional 1-element int64 device tensor mixed into the seed at run
    time (lets a captured hipGraph draw fresh noise per replay).
    mask: with cfg.predictive_mask, {scale: (B,S,h,w)} predictive masks already
    upsampled to the loss resolution (trainer.py:449-455); differentiable.  The
    BCE weighting term (trainer.py:457-459) is the caller's.
    src8: optional (S,B,H,W) int32 8-bit RGBx copies of the source frames at scale 0
    (data.pack_rgbx / md2_aug_run2): the forward then reads them instead of packing
    them per call.  Contract (not checked unless MD2_CHECK_SRC8=1, `check_src8`): the
    same frames as the fp32 source colours, which are exactly k/255 — drop
    color_src8 from a batch whose colours were edited after it was packed.
    """
    dev = T.device
    if dev.type != "cuda":
        raise RuntimeError("photometric_loss runs on the GPU only (HIP kernels); got device " + str(dev))
    B, H, W, S = cfg.batch, cfg.height, cfg.width, cfg.num_src
    if len(disps) != cfg.num_scales:
        raise ValueError(f"expected {cfg.num_scales} disparity maps, got {len(disps)}")
    disps = [d.contiguous() for d in disps]
    for s, d in enumerate(disps):
        # fp32, or bf16 as the decoder emits them under bf16 autocast (read as is,
        # md2_desc.disp_dtype); every scale in the same dtype
        _require(d, f"disp[{s}]", (B, 1, H >> s, W >> s), dev, (torch.float32, torch.bfloat16))
        if d.dtype != disps[0].dtype:
            raise ValueError(f"disp[{s}] is {d.dtype}, disp[0] {disps[0].dtype}: one dtype for every scale")
    tshape = (cfg.num_scales, S, B, 4, 4) if cfg.t_per_scale else (S, B, 4, 4)
    _require(T, "T", tshape, dev)
    ops = Operands(cfg, colors, K, inv_K, noise, dev, seed_tensor, src8)
    packed = None
    if cfg.predictive_mask:
        if mask is None:
            raise ValueError("cfg.predictive_mask needs mask={scale: (B,S,h,w)}")
        if not cfg.disable_automasking:
            raise ValueError("predictive_mask requires disable_automasking (trainer.py:91-92)")
        for s in range(cfg.num_scales):
            h, w = cfg.loss_res(s)
            _require(mask[s], f"mask[{s}]", (B, S, h, w), dev)
        packed = torch.cat([mask[s].reshape(-1) for s in range(cfg.num_scales)]).contiguous()
    elif mask is not None:
        raise ValueError("mask given but cfg.predictive_mask is False")
    return _PhotometricLoss.apply(cfg, ops, int(seed), T.contiguous(), packed, *disps)


def predictive_mask_inputs(cfg: HotPathConfig, masks: Dict[int, torch.Tensor]):
    """trainer.py:449-459: upsample the mask decoder's outputs to the loss
    resolution (bilinear, align_corners=False) and form the BCE weighting terms
    0.2 * BCE(mask, 1).  Returns ({scale: upsampled mask}, (num_scales,) BCE)."""
    import torch.nn.functional as F
    up, bce = {}, []
    for s in range(cfg.num_scales):
        m = masks[s]
        if not cfg.v1_multiscale:
            m = F.interpolate(m, [cfg.height, cfg.width], mode="bilinear", align_corners=False)
        up[s] = m
        bce.append(0.2 * F.binary_cross_entropy(m, torch.ones_like(m)))
    return up, torch.stack(bce)


def selection_maps(cfg: HotPathConfig, select: torch.Tensor) -> Dict[int, torch.Tensor]:
    """Unpack the argmin map into per-scale (B,h,w) index tensors."""
    out, off = {}, 0
    for s in range(cfg.num_scales):
        h, w = cfg.loss_res(s)
        n = cfg.batch * h * w
        out[s] = select[off:off + n].view(cfg.batch, h, w)
        off += n
    return out


def generate_images(cfg: HotPathConfig, disps, colors, K, inv_K, T, want_depth=True, want_sample=True,
                    want_color=True):
    """Materialise generate_images_pred's outputs (no autograd): returns
    {"depth": {s: (B,1,h,w)}, "sample": {(f,s): (B,h,w,2)}, "color": {(f,s): (B,3,h,w)}}
    with f the source index 0..S-1."""
    L = _lib.lib()
    dev = T.device
    disps = [d.contiguous() for d in disps]
    ops = Operands(cfg, colors, K, inv_K, None, dev)
    st = ops.struct(disps, T.contiguous())
    desc = cfg.desc(0, disps[0].dtype)
    S = cfg.num_src
    depth, sample, color = {}, {}, {}
    dptr = (ctypes.c_void_p * _lib.MAX_SCALES)()
    sptr = (ctypes.c_void_p * (_lib.MAX_SCALES * _lib.MAX_SRC))()
    cptr = (ctypes.c_void_p * (_lib.MAX_SCALES * _lib.MAX_SRC))()
    for s in range(cfg.num_scales):
        h, w = cfg.loss_res(s)
        if want_depth:
            depth[s] = torch.empty(cfg.batch, 1, h, w, device=dev)
            dptr[s] = depth[s].data_ptr()
        for f in range(S):
            if want_sample:
                sample[(f, s)] = torch.empty(cfg.batch, h, w, 2, device=dev)
                sptr[s * S + f] = sample[(f, s)].data_ptr()
            if want_color:
                color[(f, s)] = torch.empty(cfg.batch, 3, h, w, device=dev)
                cptr[s * S + f] = color[(f, s)].data_ptr()
    _lib.check(L.md2_generate_images(ctypes.byref(desc), ctypes.byref(st), dptr, sptr, cptr, _stream_ptr(dev)),
               "md2_generate_images")
    return {"depth": depth, "sample": sample, "color": color}


def tiebreak_noise(cfg: HotPathConfig, seed: int = 0, seed_tensor: Optional[torch.Tensor] = None,
                   device="cuda") -> Dict[int, torch.Tensor]:
    """The unit-normal tie-break noise a forward with noise=None draws in-kernel
    (trainer.py:468), {scale: (B,C,h,w)} — what `photometric_loss(..., seed=seed,
    seed_tensor=seed_tensor)` adds (x 1e-5) to the identity losses."""
    L = _lib.lib()
    dev = torch.device(device)
    desc = cfg.desc(seed)
    C = 1 if cfg.avg_reprojection else cfg.num_src
    out = {}
    for s in range(cfg.num_scales):
        h, w = cfg.loss_res(s)
        out[s] = torch.empty(cfg.batch, C, h, w, device=dev)
        _lib.check(L.md2_tiebreak_noise(ctypes.byref(desc), seed_tensor.data_ptr() if seed_tensor is not None else None,
                                        s, out[s].data_ptr(), _stream_ptr(dev)), "md2_tiebreak_noise")
    return out
