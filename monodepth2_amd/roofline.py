"""Algorithmic work of the photometric hot path, pinned in code.

bench.py divides these by the measured kernel time for its `roofline` figures;
DESIGN.md §5 states them.  "Algorithmic" = what the reference's computation
(generate_images_pred + compute_losses, /root/reference/trainer.py:341-496, with the
layers.py primitives it calls) needs at minimum, counted once: no recomputation,
no intermediate planes, target-only SSIM terms shared by every candidate, the
scale-invariant identity losses formed once (trainer.py:432-439), and in the
backward only the reprojection candidates (the identity ones are functions of data).

Bytes (§8(d)), per image, forward + backward at full resolution:
read the target and the S source frames at scale 0 (3 fp32 planes each), the target
pyramid at scales 1..3 for the smoothness term (3 planes x 0.328125 N), the disparity
pyramid once (1.328125 N) and write its gradient once (1.328125 N):
    bytes = 4 N (3 (1 + S) + 3 * 0.328125 + 2 * 1.328125) = 4 N (3 S + 6.640625)
mono S=2: 50.5625 N = 6.21 MB at 640x192.

Flops: one FMA = 2, every add / mul / div / compare / abs / min / max / exp = 1.
The per-unit counts, with the reference line each follows:
"""
from __future__ import annotations

from dataclasses import dataclass

# ---- forward -----------------------------------------------------------------
# BackprojectDepth ray inv_K[:3,:3] @ [x, y, 1] (layers.py:164): 3 rows x (2 mul + 2 add),
# the same for every scale and frame of an image -> once per pixel
RAY = 12
# per (pixel, scale): bilinear upsample of disp_s (trainer.py:350-351; 4 taps:
# 6 mul + 3 add; none at s = 0, a same-size copy), disp_to_depth (layers.py:21-25:
# 1 mul + 1 add + 1 reciprocal), depth * ray (layers.py:165: 3 mul)
UPSAMPLE = 9
DEPTH = 3
CAM = 3
# per (pixel, scale, frame): Project3D (layers.py:182-192): P @ [X, Y, Z, 1] 3 x (3 mul +
# 3 add), z + eps and two divisions, normalisation (x / (W-1) - 0.5) * 2 per coordinate
PROJECT = 18 + 3 + 6
# grid_sample border, align_corners=False (trainer.py:384-387): unnormalise
# ((g + 1) W - 1) / 2 per coordinate (4), border clip (2 per coordinate), floor (2),
# fractional weights (2 sub, 2 one-minus, 4 corner products), 3 channels x (4 mul + 3 add)
WARP = 8 + 4 + 2 + 8 + 3 * 7
# per (pixel, candidate) loss, compute_reprojection_loss (trainer.py:393-405) with SSIM
# (layers.py:239-248), per channel with the target-side terms shared: x^2, xy (2);
# 3x3 means of x, x^2, xy (3 x (4 add + 1 mul)); mu_x^2, sigma_x, mu_x mu_y, sigma_xy (4);
# SSIM_n (5); SSIM_d (5); 1 - n/d, /2, clamp (5) -> 36 per channel; channel mean (3);
# L1: 3 sub, 3 abs, channel mean (3); 0.85 a + 0.15 b (3)
SSIM_CH = 2 + 15 + 4 + 5 + 5 + 5
L1 = 9
CANDIDATE_SSIM = 3 * SSIM_CH + 3 + L1 + 3
CANDIDATE_L1 = L1
# target-only SSIM terms, once per pixel: y^2, 3x3 means of y and y^2, mu_y^2, sigma_y
# (13 per channel)
TARGET_SSIM = 3 * 13
# per (pixel, scale) with automasking: identity + 1e-5 noise (2 per identity candidate,
# trainer.py:468-469), min over the candidates (trainer.py:478), the automask compare
# (481-482), the mean's add (484)
def combine(S: int, automask: bool, avg: bool) -> int:
    n_ident = (1 if avg else S) if automask else 0
    n_rep = 1 if avg else S
    return 2 * n_ident + max(n_ident + n_rep - 1, 0) + (1 if automask else 0) + 1 + (S if avg else 0)
# smoothness per native pixel of scale s (trainer.py:486-488, layers.py:202-215): the
# per-image mean's add and the normalising division (2); per direction: disparity
# difference + abs (2), colour differences + abs (6), channel mean (3), exp(-g) (2),
# product (1), the mean's add (1)
SMOOTH = 2 + 2 * (2 + 6 + 3 + 2 + 1 + 1)

# ---- backward (autograd of the above, trainer.py:208) ------------------------------
# per (pixel, reprojection candidate): SSIM adjoint per channel — clamp / selection
# routing (2), d/dn and d/dd of (1 - n/d)/2 (6), through the products A B and C D (4),
# to (mu_x, sigma_x, sigma_xy) and on to (E[x], E[x^2], E[xy]) (4 + 1 + 3 + 2), the
# transposed 3x3 means of three quantities with the reflection fold (15), dx =
# g_mu + 2 x g_x2 + y g_xy (5), L1 sign term (2) -> 44 per channel; channel-mean and
# 0.85 / 0.15 split (3)
SSIM_ADJ_CH = 2 + 6 + 4 + 10 + 15 + 5 + 2
CANDIDATE_ADJ_SSIM = 3 * SSIM_ADJ_CH + 3
CANDIDATE_ADJ_L1 = 3 * 2 + 3
# per (pixel, scale, frame): bilinear derivative w.r.t. the sample point, 3 channels x
# (2 coordinates x (2 sub + 2 mul + 1 add) + 2 mul + 2 add) (42), border mask and
# unnormalise (4); normalisation (2); perspective division (6); P^T d(cam) (15) and the
# dL/dP outer-product accumulation (24); dL/ddepth = ray . d(cam) (5)
WARP_ADJ = 42 + 4 + 2 + 6 + 15 + 24 + 5
# per (pixel, scale): sum over frames (S - 1), d(1/scaled)/d(disp) (3); upsample
# adjoint for s > 0 (4 taps x (1 mul + 1 add))
DEPTH_ADJ = 3
UPSAMPLE_ADJ = 8
# smoothness adjoint per native pixel: both differences' sign x weight into two pixels
# per direction (8), the mean-normalisation term (4), the add into the upsample
# adjoint's gradient (1)
SMOOTH_ADJ = 8 + 4 + 1


@dataclass(frozen=True)
class Census:
    fwd_flops: float
    bwd_flops: float
    bytes: float

    @property
    def flops(self) -> float:
        return self.fwd_flops + self.bwd_flops


def hot_path_census(height: int, width: int, num_src: int, num_scales: int = 4, ssim: bool = True,
                    automask: bool = True, avg_reprojection: bool = False, disp_bytes: int = 4) -> Census:
    """Per-IMAGE algorithmic flops (forward, backward) and HBM bytes of the fused hot
    path at full-resolution loss (the default, not v1_multiscale).  disp_bytes = 2
    for bf16 disparities and disparity gradients (45.25 N)."""
    N = height * width
    S = num_src
    pyr = sum(1.0 / 4 ** s for s in range(num_scales))       # 1.328125 at 4 scales
    cand = CANDIDATE_SSIM if ssim else CANDIDATE_L1
    cand_adj = CANDIDATE_ADJ_SSIM if ssim else CANDIDATE_ADJ_L1
    n_ident = (1 if avg_reprojection else S) if automask else 0
    fwd = RAY
    for s in range(num_scales):
        fwd += (UPSAMPLE if s else 0) + DEPTH + CAM
        fwd += S * (PROJECT + WARP + cand)
        fwd += combine(S, automask, avg_reprojection)
    fwd += n_ident * cand + (TARGET_SSIM if ssim else 0)
    fwd += SMOOTH * pyr
    bwd = 0.0
    for s in range(num_scales):
        bwd += S * (cand_adj + WARP_ADJ) + (S - 1) + DEPTH_ADJ + (UPSAMPLE_ADJ if s else 0)
    bwd += SMOOTH_ADJ * pyr
    nbytes = 4 * 3 * (1 + S) + 4 * 3 * (pyr - 1.0) + 2 * disp_bytes * pyr
    return Census(fwd_flops=fwd * N, bwd_flops=bwd * N, bytes=nbytes * N)
