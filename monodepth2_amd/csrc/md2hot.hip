// md2hot.hip — hand-written CDNA4 (gfx950) kernels for the monodepth2 photometric
// hot path, behind the C ABI declared in include/md2hot.h.
//
// Reference semantics (all /root/reference/...):
//   upsample disp_s to (H,W), bilinear, align_corners=False      trainer.py:350-351
//   depth = 1 / (1/max_depth + (1/min_depth - 1/max_depth) disp)  layers.py:16-25
//   cam = depth * inv_K[:3,:3] @ [x,y,1];  c = (K@T)[:3] @ [cam;1]  layers.py:163-168, 182-185
//   pix = c.xy / (c.z + 1e-7), normalised by (W-1),(H-1) to [-1,1] layers.py:187-192
//   warp = grid_sample(color_f, pix, bilinear, border, align_corners=False)  trainer.py:384-387
//   reproj = 0.85 mean_c SSIM(warp, target) + 0.15 mean_c |target - warp|  trainer.py:393-405
//   SSIM: reflection pad 1, 3x3 box means, C1=1e-4, C2=9e-4, clamp [0,1]  layers.py:218-248
//   per-pixel min over cat(identity + 1e-5 noise, reproj)  trainer.py:432-482
//   smoothness on disp/mean(disp), edge-aware, weight w/2^s       trainer.py:486-490, layers.py:202-215
//
// Execution layout: one wave = one column strip of 64 lanes
// (lane <-> image column, 1 halo lane each side in the forward, 2 in the
// backward) x ROWS image rows walked top to bottom with a 3-row sliding window.
// Horizontal 3-tap sums use cross-lane shuffles, vertical ones the register
// window, so the SSIM stencil needs no LDS and no materialised warped image.
// Every HBM-sized intermediate of the eager reference (warped images, grids,
// SSIM maps, candidate stacks) stays in registers.
//
// Determinism: no float atomics.  Per-wave partial sums go to the workspace and
// are reduced in a fixed order by single-block finalize kernels.

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <map>
#include <mutex>
#include <vector>

#include "md2hot.h"
#include "md2_bf16.h"

namespace {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr int kFwdCols = kWave - 2;  // output columns per forward strip
constexpr int kBwdCols = kWave - 4;  // output columns per backward strip
#ifndef MD2_ROWS_B
#define MD2_ROWS_B 16
#endif
// minimum resident 256-thread blocks per CU (__launch_bounds__) of the backward:
// 2 = 2 waves/SIMD (<= 256 VGPRs); it spills 164 B/lane at 3 (<= 168).
#ifndef MD2_BWD_MINB
#define MD2_BWD_MINB 2
#endif
constexpr int kRowsB = MD2_ROWS_B;   // output rows per backward work item
constexpr int kSmoothChunk = 1024;   // pixels per smoothness partial (one pixel quad per thread)
constexpr float kC1 = 0.0001f;       // 0.01 ** 2   layers.py:231
constexpr float kC2 = 0.0009f;       // 0.03 ** 2   layers.py:232
constexpr float kInv9 = 1.0f / 9.0f;

// ----------------------------------------------------------------------------
// small device helpers
// ----------------------------------------------------------------------------
__device__ __forceinline__ int reflect_clamp(int i, int n) {
    i = i < 0 ? -i : i;
    i = i >= n ? 2 * (n - 1) - i : i;
    return min(max(i, 0), n - 1);
}

// Neighbour-lane reads as DPP wave shifts (one VALU op, no LDS round trip, unlike the
// ds_bpermute that __shfl_up/down lower to).  wave_shr:1 gives lane i the value of
// lane i-1, wave_shl:1 of lane i+1 (checked on MI355X); lanes 0 / 63 receive 0,
// they are halo lanes whose results are never used.
__device__ __forceinline__ float shfl_prev(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x138, 0xf, 0xf, true));
}
__device__ __forceinline__ float shfl_next(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, true));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, dispatch
// placement; speed only, never correctness).  Give every XCD a contiguous range of
// logical blocks so its private L2 streams a contiguous slice of the images instead
// of all XCDs fetching every image.  Bijective for any n.
__device__ __forceinline__ int xcd_contiguous_block(int bid, int n) {
    const int q = n >> 3, r = n & 7;
    const int xcd = bid & 7, idx = bid >> 3;
    return xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
}

// Loads at a uniform base + a non-negative 32-bit element index: the byte offset is
// formed in 32 bits, so the compiler emits the SGPR-base + VGPR-offset form of
// global_load (no 64-bit address arithmetic per lane).  ldf2 fetches two adjacent
// floats as one global_load_dwordx2 (4-byte alignment suffices on gfx950).  The
// photo kernels are bound by vector-memory instruction throughput (profiles/r01),
// so each load instruction saved counts.
typedef float float2_a4 __attribute__((ext_vector_type(2), aligned(4)));
__device__ __forceinline__ float ldf(const float* base, int idx) {
    return *(const float*)((const char*)base + ((uint32_t)idx << 2));
}
__device__ __forceinline__ float2_a4 ldf2(const float* base, int idx) {
    return *(const float2_a4*)((const char*)base + ((uint32_t)idx << 2));
}
__device__ __forceinline__ uint8_t ldb(const uint8_t* base, int idx) { return base[(uint32_t)idx]; }

// Disparities come as fp32 or bf16 (md2_desc.disp_dtype: the depth decoder's output
// under bf16 autocast, read as is instead of cast up in a separate pass; bf16 -> fp32
// is exact, so the arithmetic is the fp32 path's).  Pointers stay `const float*`;
// element offsets are scaled by the element size here.
__device__ __forceinline__ const float* disp_off(const float* base, size_t elems, bool bf16) {
    return (const float*)((const char*)base + (elems << (bf16 ? 1 : 2)));
}
__device__ __forceinline__ float ldd(const float* base, int idx, bool bf16) {
    if (bf16) return md2::bf2f(*(const uint16_t*)((const char*)base + ((uint32_t)idx << 1)));
    return ldf(base, idx);
}

// x / 3 correctly rounded (the channel mean of trainer.py:396-397 divides by 3), in
// three VALU ops instead of the IEEE division sequence: q = x * RN(1/3), one exact
// fma residual, one fma correction (Markstein)
__device__ __forceinline__ float div3(float x) {
    const float c = 1.0f / 3.0f;
    const float q = x * c;
    return fmaf(fmaf(-3.0f, q, x), c, q);
}

// k / 255 correctly rounded for integer k in 0..255 (3 ops; the 8-bit copies' decode)
__device__ __forceinline__ float div255(float k) {
    const float c = 1.0f / 255.0f;
    const float q = k * c;
    return fmaf(fmaf(-255.0f, q, k), c, q);
}

__device__ __forceinline__ float signf(float v) { return (v > 0.f) ? 1.f : ((v < 0.f) ? -1.f : 0.f); }

// Tie-break noise of the forward (trainer.py:468 draws N(0,1) * 1e-5 per
// (image, candidate, pixel) and scale): one 32-bit counter hash per (scale, image
// pixel, candidate pair) -> two uniforms -> a Box-Muller pair, i.e. two deviates per
// hash, log and sqrt.  Deterministic in (seed, scale, pixel); the draw itself cannot
// match torch.randn, so parity tests pass the noise in explicitly.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
__device__ __forceinline__ uint32_t noise_key(uint64_t seed, int gsc) {
    return lowbias32((uint32_t)seed ^ lowbias32((uint32_t)(seed >> 32) + 0x9E3779B9u * (uint32_t)(gsc + 1)));
}
// candidates 2j and 2j+1 of pixel q (= b*HW + p) at the scale keyed by `key`
__device__ __forceinline__ float2 noise_pair(uint32_t key, uint32_t q, int j) {
    const uint32_t h1 = lowbias32(q * 0x9E3779B1u + key + (uint32_t)j * 0x85EBCA77u);
    const uint32_t h2 = lowbias32(h1 ^ 0x68E31DA4u);
    const float u1 = (float)(h1 >> 8) * (1.0f / 16777216.0f) + (0.5f / 16777216.0f);
    const float u2 = (float)(h2 >> 8) * (1.0f / 16777216.0f);
    const float r = sqrtf(-2.0f * __logf(u1));
    float sn, cs;
    __sincosf(6.28318530718f * u2, &sn, &cs);
    return make_float2(r * cs, r * sn);
}

// ----------------------------------------------------------------------------
// per-(image, frame) camera: P = (K @ T)[:3] and inv_K[:3,:3]   layers.py:164,183
// ----------------------------------------------------------------------------
__device__ __forceinline__ float uniformf(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

struct Cam {
    float iK[9];
    float P[12];
};

__device__ __forceinline__ void load_cam(Cam& cm, const float* K, const float* iK, const float* T) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
            cm.P[i * 4 + j] = K[i * 4 + 0] * T[0 * 4 + j] + K[i * 4 + 1] * T[1 * 4 + j] +
                              K[i * 4 + 2] * T[2 * 4 + j] + K[i * 4 + 3] * T[3 * 4 + j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) cm.iK[i * 3 + j] = iK[i * 4 + j];
    // wave-uniform: keep them in SGPRs (VALU operands), not in 21 VGPRs
#pragma unroll
    for (int i = 0; i < 12; ++i) cm.P[i] = uniformf(cm.P[i]);
#pragma unroll
    for (int i = 0; i < 9; ++i) cm.iK[i] = uniformf(cm.iK[i]);
}

// everything a warp of one (image, frame, scale) needs
struct WarpCtx {
    const float* disp;  // (dh, dw) disparity of this image at its native scale (fp32 or bf16)
    bool dbf16;
    int dh, dw, upsh;   // upsample factor 2^upsh to the loss resolution
    const float* src;   // (3, h, w) source colours at the loss resolution
    const uint32_t* src8;  // the same colours as 8-bit RGBx per pixel (k/255 exact), or null
    int h, w;
    float sx, sy;       // W/(W-1), H/(H-1): pixel -> grid_sample source coordinate
    float min_disp, range;
    Cam cm;
};

// bilinear upsample, align_corners=False (ATen area_pixel_compute_source_index)
__device__ __forceinline__ float disp_at(const WarpCtx& c, int y, int x) {
    if (c.upsh == 0) return ldd(c.disp, y * c.dw + x, c.dbf16);
    const float sc = 1.0f / (float)(1 << c.upsh);
    const float sy = fmaxf(((float)y + 0.5f) * sc - 0.5f, 0.f);
    const float sx = fmaxf(((float)x + 0.5f) * sc - 0.5f, 0.f);
    const int y0 = min((int)sy, c.dh - 1), x0 = min((int)sx, c.dw - 1);
    const int y1 = y0 + (y0 < c.dh - 1 ? 1 : 0);
    const bool xin = x0 < c.dw - 1;   // x1 = x0 + 1, else x1 = x0 (right border)
    const float ly1 = fminf(fmaxf(sy - (float)y0, 0.f), 1.f), lx1 = fminf(fmaxf(sx - (float)x0, 0.f), 1.f);
    const float ly0 = 1.f - ly1, lx0 = 1.f - lx1;
    // (x0, x1) as one pair load; at the right border the pair starts one column left
    const int xa = xin ? x0 : x0 - 1;
    float2_a4 t, u;
    if (c.dbf16) {
        t.x = ldd(c.disp, y0 * c.dw + xa, true), t.y = ldd(c.disp, y0 * c.dw + xa + 1, true);
        u.x = ldd(c.disp, y1 * c.dw + xa, true), u.y = ldd(c.disp, y1 * c.dw + xa + 1, true);
    } else {
        t = ldf2(c.disp, y0 * c.dw + xa), u = ldf2(c.disp, y1 * c.dw + xa);
    }
    const float t0 = xin ? t.x : t.y, u0 = xin ? u.x : u.y;
    return ly0 * (lx0 * t0 + lx1 * t.y) + ly1 * (lx0 * u0 + lx1 * u.y);
}

// one projected sample: the forward values the backward chain needs
struct Sample {
    float depth;
    float ray[3];   // inv_K[:3,:3] @ [x, y, 1]
    float pt[3];    // depth * ray
    float cam[3];   // P @ [pt; 1]
    float den;      // cam.z + eps
    float gmx, gmy; // grid-sample input gradient multipliers (size/2, 0 when clipped)
    int x0, y0;
    float tx, ty;   // fractional position inside the source cell
};

__device__ __forceinline__ void project(const WarpCtx& c, int y, int x, Sample& s) {
    const float d = disp_at(c, y, x);
    s.depth = 1.0f / (c.min_disp + c.range * d);
    const float fx = (float)x, fy = (float)y;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        s.ray[i] = c.cm.iK[i * 3 + 0] * fx + c.cm.iK[i * 3 + 1] * fy + c.cm.iK[i * 3 + 2];
        s.pt[i] = s.depth * s.ray[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
        s.cam[i] = c.cm.P[i * 4 + 0] * s.pt[0] + c.cm.P[i * 4 + 1] * s.pt[1] +
                   c.cm.P[i * 4 + 2] * s.pt[2] + c.cm.P[i * 4 + 3];
    s.den = s.cam[2] + 1e-7f;
    const float px = s.cam[0] / s.den, py = s.cam[1] / s.den;
    const float gx = (px / (float)(c.w - 1) - 0.5f) * 2.f;
    const float gy = (py / (float)(c.h - 1) - 0.5f) * 2.f;
    // unnormalise (align_corners=False) and clip (padding_mode="border")
    const float hw = 0.5f * (float)c.w, hh = 0.5f * (float)c.h;
    const float ix = (gx + 1.f) * hw - 0.5f, iy = (gy + 1.f) * hh - 0.5f;
    const float xmax = (float)(c.w - 1), ymax = (float)(c.h - 1);
    const float ixc = fminf(fmaxf(ix, 0.f), xmax), iyc = fminf(fmaxf(iy, 0.f), ymax);
    s.gmx = (ix > 0.f && ix < xmax) ? hw : 0.f;  // borders count as out of bounds
    s.gmy = (iy > 0.f && iy < ymax) ? hh : 0.f;
    const float fx0 = floorf(ixc), fy0 = floorf(iyc);
    s.x0 = (int)fx0;
    s.y0 = (int)fy0;
    s.tx = ixc - fx0;
    s.ty = iyc - fy0;
}

__device__ __forceinline__ float rcpf(float v) { return __builtin_amdgcn_rcpf(v); }

// Same projection as `project` with hardware reciprocals (v_rcp_f32, 1 ulp) in
// place of IEEE divisions, and the normalise/unnormalise pair of layers.py:190-192
// + grid_sample folded into one scale: ix = px * W/(W-1) - 0.5.  Differences to
// the exact form are O(1 ulp) in the sampling position.
struct FastSample {
    float depth;
    float ray[3];
    float pt[3];
    float cam[3];
    float inv_den;
    float px, py;
    float gmx, gmy;  // 0 where grid_sample clips (border), else 1
    int x0, y0;
    float tx, ty;
};

// depth of the upsampled disparity at (y, x) (layers.py:16-25 with v_rcp_f32)
__device__ __forceinline__ float depth_at(const WarpCtx& c, int y, int x) {
    return rcpf(c.min_disp + c.range * disp_at(c, y, x));
}

// component i of the ray inv_K[:3,:3] @ [x, y, 1] (layers.py:164): one expression
// for the projection and the backward's output step, so both round identically
__device__ __forceinline__ float ray_at(const Cam& cm, int i, float fx, float fy) {
    return cm.iK[i * 3 + 0] * fx + cm.iK[i * 3 + 1] * fy + cm.iK[i * 3 + 2];
}

// projection of pixel (y, x) at a given depth
__device__ __forceinline__ void project_depth(const WarpCtx& c, int y, int x, float depth, FastSample& s) {
    s.depth = depth;
    const float fx = (float)x, fy = (float)y;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        s.ray[i] = ray_at(c.cm, i, fx, fy);
        s.pt[i] = s.depth * s.ray[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i)
        s.cam[i] = c.cm.P[i * 4 + 0] * s.pt[0] + c.cm.P[i * 4 + 1] * s.pt[1] +
                   c.cm.P[i * 4 + 2] * s.pt[2] + c.cm.P[i * 4 + 3];
    s.inv_den = rcpf(s.cam[2] + 1e-7f);
    s.px = s.cam[0] * s.inv_den;
    s.py = s.cam[1] * s.inv_den;
    const float ix = s.px * c.sx - 0.5f, iy = s.py * c.sy - 0.5f;
    const float xmax = (float)(c.w - 1), ymax = (float)(c.h - 1);
    const float ixc = fminf(fmaxf(ix, 0.f), xmax), iyc = fminf(fmaxf(iy, 0.f), ymax);
    s.gmx = (ix > 0.f && ix < xmax) ? 1.f : 0.f;
    s.gmy = (iy > 0.f && iy < ymax) ? 1.f : 0.f;
    const float fx0 = floorf(ixc), fy0 = floorf(iyc);
    s.x0 = (int)fx0;
    s.y0 = (int)fy0;
    s.tx = ixc - fx0;
    s.ty = iyc - fy0;
}

__device__ __forceinline__ void project_fast(const WarpCtx& c, int y, int x, FastSample& s) {
    project_depth(c, y, x, depth_at(c, y, x), s);
}

// the four (masked) source corners of a sample for the 3 channels
struct Corners {
    float nw[3], ne[3], sw[3], se[3];
};

// Horizontally adjacent corners (nw, ne) and (sw, se) are fetched as one 8-byte pair
// per row and channel: 6 gather instructions per sample instead of 12, the same
// bytes.  At the right border (x0 = w-1, where ne is masked) the pair starts one
// column to the left.
//
// 8-bit sources (src8): colours that are exactly k/255 — what to_tensor makes of the
// decoded frames (datasets/mono_dataset.py:199-200, the GPU input pipeline likewise) —
// are gathered from one RGBx dword per pixel: 2 gather instructions per sample
// instead of 6, a third of the texture-path work, which binds these kernels when
// the warp scatters (tools/gather_model.hip).  The corners come back as k; interp and
// the bilinear slopes scale by cs = 1/255 once per channel (differences O(1 ulp)).
typedef uint32_t uint2_a4 __attribute__((ext_vector_type(2), aligned(4)));

template <bool U8, class SampleT>
__device__ __forceinline__ void gather(const WarpCtx& c, const SampleT& s, Corners& v) {
    const bool vx1 = s.x0 + 1 < c.w, vy1 = s.y0 + 1 < c.h;
    const int y1 = vy1 ? s.y0 + 1 : s.y0;
    const int xa = vx1 ? s.x0 : s.x0 - 1;
    const int HW = c.h * c.w;
    const int ot = s.y0 * c.w + xa, ob = y1 * c.w + xa;
    if (U8) {
        const uint2_a4 t = *(const uint2_a4*)((const char*)c.src8 + ((uint32_t)ot << 2));
        const uint2_a4 u = *(const uint2_a4*)((const char*)c.src8 + ((uint32_t)ob << 2));
        const uint32_t pnw = vx1 ? t.x : t.y, pne = vx1 ? t.y : 0u;
        const uint32_t psw = vy1 ? (vx1 ? u.x : u.y) : 0u, pse = (vx1 && vy1) ? u.y : 0u;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            v.nw[ch] = (float)((pnw >> (8 * ch)) & 255u);
            v.ne[ch] = (float)((pne >> (8 * ch)) & 255u);
            v.sw[ch] = (float)((psw >> (8 * ch)) & 255u);
            v.se[ch] = (float)((pse >> (8 * ch)) & 255u);
        }
        return;
    }
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float2_a4 t = ldf2(c.src, ch * HW + ot), u = ldf2(c.src, ch * HW + ob);
        v.nw[ch] = vx1 ? t.x : t.y;
        v.ne[ch] = vx1 ? t.y : 0.f;
        v.sw[ch] = vy1 ? (vx1 ? u.x : u.y) : 0.f;
        v.se[ch] = (vx1 && vy1) ? u.y : 0.f;
    }
}

template <bool U8, class SampleT>
__device__ __forceinline__ void interp(const SampleT& s, const Corners& v, float out[3]) {
    const float e = 1.f - s.tx, so = 1.f - s.ty;
    const float wnw = so * e, wne = so * s.tx, wsw = s.ty * e, wse = s.ty * s.tx;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        out[ch] = v.nw[ch] * wnw + v.ne[ch] * wne + v.sw[ch] * wsw + v.se[ch] * wse;
        if (U8) out[ch] *= 1.0f / 255.0f;
    }
}

// ----------------------------------------------------------------------------
// Colour channels as C3: channels 0 and 1 in one 64-bit register pair, channel 2 alone,
// so every per-channel add / mul / fma of the SSIM + L1 chains (and their adjoint) is
// one v_pk_*_f32 for two channels (two lanes of work per issue slot, the f32 VALU peak
// of CDNA4) plus the scalar op for the third.  Round 3 moved the kernels from per-channel
// scalars to C3 (static VALU -12 %: fwdall 117 -> 113 us, photo_bwd 271 -> 257 us at B=12).
// ----------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));
struct C3 {
    f2v a;     // channels 0, 1
    float b;   // channel 2
};
__device__ __forceinline__ C3 operator+(const C3& x, const C3& y) { return {x.a + y.a, x.b + y.b}; }
__device__ __forceinline__ C3 operator-(const C3& x, const C3& y) { return {x.a - y.a, x.b - y.b}; }
__device__ __forceinline__ C3 operator*(const C3& x, const C3& y) { return {x.a * y.a, x.b * y.b}; }
__device__ __forceinline__ C3 operator*(const C3& x, float s) { return {x.a * s, x.b * s}; }
__device__ __forceinline__ C3 operator+(const C3& x, float s) { return {x.a + s, x.b + s}; }
__device__ __forceinline__ C3 shfl_prev3(const C3& v) {
    return {f2v{shfl_prev(v.a.x), shfl_prev(v.a.y)}, shfl_prev(v.b)};
}
__device__ __forceinline__ C3 shfl_next3(const C3& v) {
    return {f2v{shfl_next(v.a.x), shfl_next(v.a.y)}, shfl_next(v.b)};
}
__device__ __forceinline__ C3 ld3(const float* base, int HW, int idx) {
    return {f2v{ldf(base, idx), ldf(base, HW + idx)}, ldf(base, 2 * HW + idx)};
}
__device__ __forceinline__ float clamp01(float v) { return fminf(fmaxf(v, 0.f), 1.f); }
__device__ __forceinline__ float sum3(const C3& v) { return v.a.x + v.a.y + v.b; }
__device__ __forceinline__ C3 abs3(const C3& v) { return {f2v{fabsf(v.a.x), fabsf(v.a.y)}, fabsf(v.b)}; }

template <bool U8, class SampleT>
__device__ __forceinline__ C3 interp3(const SampleT& s, const Corners& v) {
    const float e = 1.f - s.tx, so = 1.f - s.ty;
    const float wnw = so * e, wne = so * s.tx, wsw = s.ty * e, wse = s.ty * s.tx;
    const C3 nw = {f2v{v.nw[0], v.nw[1]}, v.nw[2]}, ne = {f2v{v.ne[0], v.ne[1]}, v.ne[2]};
    const C3 sw = {f2v{v.sw[0], v.sw[1]}, v.sw[2]}, se = {f2v{v.se[0], v.se[1]}, v.se[2]};
    C3 o = nw * wnw + ne * wne + sw * wsw + se * wse;
    if (U8) o = o * (1.0f / 255.0f);
    return o;
}

// ----------------------------------------------------------------------------
// SSIM pieces (layers.py:218-248), three channels at once
// ----------------------------------------------------------------------------
struct H5P {  // horizontal 3-tap sums of x, x^2, x*y, y, y^2
    C3 x, xx, xy, y, yy;
};

__device__ __forceinline__ H5P hsum3(const C3& x, const C3& y) {
    const C3 xl = shfl_prev3(x), xr = shfl_next3(x), yl = shfl_prev3(y), yr = shfl_next3(y);
    return {xl + x + xr, xl * xl + x * x + xr * xr, xl * yl + x * y + xr * yr, yl + y + yr, yl * yl + y * y + yr * yr};
}

__device__ __forceinline__ float ssim1(float n, float d) { return clamp01((1.f - n * rcpf(d)) * 0.5f); }

// sum over the three channels of SSIM at the middle row of (a, b, c) (ssim_from_sums)
__device__ __forceinline__ float ssim_sum3(const H5P& a, const H5P& b, const H5P& c) {
    const C3 mx = (a.x + b.x + c.x) * kInv9, my = (a.y + b.y + c.y) * kInv9;
    const C3 sx = (a.xx + b.xx + c.xx) * kInv9 - mx * mx;
    const C3 sy = (a.yy + b.yy + c.yy) * kInv9 - my * my;
    const C3 sxy = (a.xy + b.xy + c.xy) * kInv9 - mx * my;
    const C3 n = (mx * my * 2.f + kC1) * (sxy * 2.f + kC2);
    const C3 d = (mx * mx + my * my + kC1) * (sx + sy + kC2);
    return ssim1(n.a.x, d.a.x) + ssim1(n.a.y, d.a.y) + ssim1(n.b, d.b);
}

__device__ __forceinline__ float clamp_pass(float raw, float g) { return (raw >= 0.f && raw <= 1.f) ? g : 0.f; }

// ssim_adjoint for the three channels
__device__ __forceinline__ void ssim_adjoint3(const H5P& a, const H5P& b, const H5P& c, float gS, C3& dA, C3& dB,
                                              C3& dC) {
    const C3 mx = (a.x + b.x + c.x) * kInv9, my = (a.y + b.y + c.y) * kInv9;
    const C3 sx = (a.xx + b.xx + c.xx) * kInv9 - mx * mx;
    const C3 sy = (a.yy + b.yy + c.yy) * kInv9 - my * my;
    const C3 sxy = (a.xy + b.xy + c.xy) * kInv9 - mx * my;
    const C3 n1 = mx * my * 2.f + kC1, n2 = sxy * 2.f + kC2;
    const C3 d1 = mx * mx + my * my + kC1, d2 = sx + sy + kC2;
    const C3 n = n1 * n2, d = d1 * d2;
    const C3 inv_d = {f2v{rcpf(d.a.x), rcpf(d.a.y)}, rcpf(d.b)};
    const C3 raw = ((n * inv_d) * -1.f + 1.f) * 0.5f;
    const C3 g = {f2v{clamp_pass(raw.a.x, gS), clamp_pass(raw.a.y, gS)}, clamp_pass(raw.b, gS)};
    const C3 dn = g * -0.5f * inv_d;
    const C3 dd = g * 0.5f * n * inv_d * inv_d;
    dA = dn * (my * 2.f * (n2 - n1)) + dd * (mx * 2.f * (d2 - d1));
    dB = dd * d1;
    dC = dn * 2.f * n1;
}

__device__ __forceinline__ C3 sign3(const C3& v) { return {f2v{signf(v.a.x), signf(v.a.y)}, signf(v.b)}; }

// ----------------------------------------------------------------------------
// smoothness (trainer.py:486-490, layers.py:202-215) — forward partial sums
// ----------------------------------------------------------------------------
struct SmoothArgs {
    int B, num_scales;
    int hs[MD2_MAX_SCALES], ws[MD2_MAX_SCALES], chunks[MD2_MAX_SCALES];
    int block_base[MD2_MAX_SCALES + 1];
    const float* disp[MD2_MAX_SCALES];
    const float* img[MD2_MAX_SCALES];   // target colour at the native scale
    float* part[MD2_MAX_SCALES];        // [B][chunks][3]
    float* sgrad[MD2_MAX_SCALES];       // (B, hs, ws): the smoothness term's per-unit gradient
    int disp_bf16;
    int quad;                           // every ws % 4 == 0: smooth_quad (float4 rows)
};

__device__ __forceinline__ float edge_weight(const float* img, int HW, int o0, int o1) {
    const float g = (fabsf(img[o0] - img[o1]) + fabsf(img[HW + o0] - img[HW + o1]) +
                     fabsf(img[2 * HW + o0] - img[2 * HW + o1])) / 3.f;
    return expf(-g);
}

__device__ __forceinline__ void block_sum3(float& a, float& b, float& c) {
    __shared__ float red[3][kWavesPerBlock];
    a = wave_sum(a);
    b = wave_sum(b);
    c = wave_sum(c);
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) {
        red[0][wid] = a;
        red[1][wid] = b;
        red[2][wid] = c;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        a = red[0][0] + red[0][1] + red[0][2] + red[0][3];
        b = red[1][0] + red[1][1] + red[1][2] + red[1][3];
        c = red[2][0] + red[2][1] + red[2][2] + red[2][3];
    }
}

__device__ __forceinline__ float4 ldd4(const float* base, int idx, bool bf16) {   // idx % 4 == 0
    if (bf16) {
        const uint2 u = *(const uint2*)((const char*)base + ((uint32_t)idx << 1));
        return make_float4(md2::bf2f((uint16_t)(u.x & 0xffffu)), md2::bf2f((uint16_t)(u.x >> 16)),
                           md2::bf2f((uint16_t)(u.y & 0xffffu)), md2::bf2f((uint16_t)(u.y >> 16)));
    }
    return *(const float4*)((const char*)base + ((uint32_t)idx << 2));
}

__device__ __forceinline__ float f4at(const float4& v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; }

// exp(-mean_c |a_c - b_c|) (layers.py:210-211 per edge), the channel mean as div3
__device__ __forceinline__ float edge_w3(float a0, float b0, float a1, float b1, float a2, float b2) {
    return expf(-div3(fabsf(a0 - b0) + fabsf(a1 - b1) + fabsf(a2 - b2)));
}

// One pixel quad (row i, columns j0..j0+3; ws % 4 == 0) of smooth_fwd: every load a
// float4 row segment or one neighbour column, each horizontal edge's weight once.
__device__ __forceinline__ void smooth_quad(const float* d, const float* img, bool bf, int hs, int ws, int i, int j0,
                                            float cx, float cy, float* sg, float& sd, float& sx, float& sy) {
    const int HW = hs * ws, p = i * ws + j0;
    const bool up = i > 0, dn = i + 1 < hs, lf = j0 > 0, rt = j0 + 4 < ws;
    // every load unconditional (border rows / columns clamped to the quad itself, their
    // terms masked below): a conditional load is a branch the wave waits at, and the
    // ~20 loads of a quad then paid ~20 serialised memory latencies (21 us per launch)
    const int pu = up ? p - ws : p, pd = dn ? p + ws : p, pl = lf ? p - 1 : p, pr = rt ? p + 4 : p + 3;
    const float4 dc = ldd4(d, p, bf);
    const float4 du = ldd4(d, pu, bf);
    const float4 dd = ldd4(d, pd, bf);
    const float dl = ldd(d, pl, bf), dr = ldd(d, pr, bf);
    float4 ic[3], iu[3], id[3];
    float il[3], ir[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const float* im = img + c * HW;
        ic[c] = *(const float4*)(im + p);
        iu[c] = *(const float4*)(im + pu);
        id[c] = *(const float4*)(im + pd);
        il[c] = im[pl];
        ir[c] = im[pr];
    }
    // horizontal edges h[k] between columns j0+k-1 and j0+k, k = 0..4
    auto col = [&](int c, int k) { return k < 0 ? il[c] : k > 3 ? ir[c] : f4at(ic[c], k); };
    float h[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) h[k] = edge_w3(col(0, k - 1), col(0, k), col(1, k - 1), col(1, k), col(2, k - 1), col(2, k));
    float g[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const float v = f4at(dc, m);
        const float vl = m == 0 ? dl : f4at(dc, m - 1), vr = m == 3 ? dr : f4at(dc, m + 1);
        sd += v;
        float gx = 0.f, gy = 0.f;
        if (m < 3 || rt) {
            const float dv = v - vr;
            sx += fabsf(dv) * h[m + 1];
            gx += signf(dv) * h[m + 1];
        }
        if (m > 0 || lf) gx -= signf(vl - v) * h[m];
        if (dn) {
            const float e = edge_w3(f4at(ic[0], m), f4at(id[0], m), f4at(ic[1], m), f4at(id[1], m), f4at(ic[2], m),
                                    f4at(id[2], m));
            const float dv = v - f4at(dd, m);
            sy += fabsf(dv) * e;
            gy += signf(dv) * e;
        }
        if (up) {
            const float e = edge_w3(f4at(iu[0], m), f4at(ic[0], m), f4at(iu[1], m), f4at(ic[1], m), f4at(iu[2], m),
                                    f4at(ic[2], m));
            gy -= signf(f4at(du, m) - v) * e;
        }
        g[m] = gx * cx + gy * cy;
    }
    *(float4*)(sg + p) = make_float4(g[0], g[1], g[2], g[3]);
}

// One block's chunk of the smoothness sums (block `bid` of the smoothness grid)
__device__ __forceinline__ void smooth_block(const SmoothArgs& a, int bid) {
    int s = 0;
    while (s + 1 < a.num_scales && bid >= a.block_base[s + 1]) ++s;
    const int local = bid - a.block_base[s];
    const int b = local / a.chunks[s], chunk = local - b * a.chunks[s];
    const int hs = a.hs[s], ws = a.ws[s], HW = hs * ws;
    const bool bf = a.disp_bf16 != 0;
    const float* d = disp_off(a.disp[s], (size_t)b * HW, bf);
    const float* img = a.img[s] + (size_t)b * 3 * HW;
    float sd = 0.f, sx = 0.f, sy = 0.f;
    const int p0 = chunk * kSmoothChunk;
    // per-unit gradient of the smoothness sums (layers.py:202-215): the sign stencil of
    // |d_p - d_q| e_pq over the pixel's four edges, with the x / y means' normalisers
    // folded in.  The backward scales it by dL/dloss_s, the weight and 1/mean
    // (disp_grad_kernel), so it never re-reads the target pyramid or the neighbours
    float* sg = a.sgrad[s] + (size_t)b * HW;
    const float cx = 1.0f / ((float)hs * (float)(ws - 1)), cy = 1.0f / ((float)(hs - 1) * (float)ws);
    static_assert(kSmoothChunk == 4 * kBlock, "one pixel quad per thread");
    if (a.quad) {   // block-uniform
        const int p = p0 + 4 * threadIdx.x;
        if (p < HW) {
            const int i = p / ws;
            smooth_quad(d, img, bf, hs, ws, i, p - i * ws, cx, cy, sg, sd, sx, sy);
        }
    } else
    for (int p = p0 + threadIdx.x; p < min(p0 + kSmoothChunk, HW); p += kBlock) {
        const int i = p / ws, j = p - i * ws;
        const float v = ldd(d, p, bf);
        sd += v;
        float gx = 0.f, gy = 0.f;
        if (j + 1 < ws) {
            const float dv = v - ldd(d, p + 1, bf), e = edge_weight(img, HW, p, p + 1);
            sx += fabsf(dv) * e;
            gx += signf(dv) * e;
        }
        if (j > 0) gx -= signf(ldd(d, p - 1, bf) - v) * edge_weight(img, HW, p - 1, p);
        if (i + 1 < hs) {
            const float dv = v - ldd(d, p + ws, bf), e = edge_weight(img, HW, p, p + ws);
            sy += fabsf(dv) * e;
            gy += signf(dv) * e;
        }
        if (i > 0) gy -= signf(ldd(d, p - ws, bf) - v) * edge_weight(img, HW, p - ws, p);
        sg[p] = gx * cx + gy * cy;
    }
    block_sum3(sd, sx, sy);
    if (threadIdx.x == 0) {
        float* o = a.part[s] + ((size_t)b * a.chunks[s] + chunk) * 3;
        o[0] = sd;
        o[1] = sx;
        o[2] = sy;
    }
}

__global__ __launch_bounds__(kBlock) void smooth_fwd_kernel(SmoothArgs a) {
    // consecutive chunks share their boundary rows (p + ws): keep them on one XCD's L2
    smooth_block(a, xcd_contiguous_block(blockIdx.x, gridDim.x));
}

// ----------------------------------------------------------------------------
// kernel arguments
// ----------------------------------------------------------------------------
struct PhotoArgs {
    int B, h, w, S, nsc;                    // loss resolution of this launch
    int strips, rowblocks, wpi;             // wave grid per image
    int gscale[MD2_MAX_SCALES];             // global scale index of each local scale
    int num_scales;                         // global number of scales
    const float* disp[MD2_MAX_SCALES];      // per local scale
    int dh[MD2_MAX_SCALES], dw[MD2_MAX_SCALES], upsh[MD2_MAX_SCALES];
    const float* tgt;                       // (B,3,h,w)
    const float* src[MD2_MAX_SRC];          // (B,3,h,w)
    const float* K;                         // (B,4,4)
    const float* iK;                        // (B,4,4)
    const float* T[MD2_MAX_SCALES];         // per local scale (S,B,4,4)
    const float* noise[MD2_MAX_SCALES];     // per local scale (B,C,h,w) or null
    uint64_t seed;
    const uint64_t* seed_ptr;               // optional device-side seed (graph replay)
    float min_disp, range;
    uint32_t flags;
    int disp_bf16;                          // disp[] elements are bf16 (md2_desc.disp_dtype)
    float* photo_part[MD2_MAX_SCALES];      // fwd: per local scale [B*wpi]
    uint8_t* sel[MD2_MAX_SCALES];           // per local scale (B,h,w)
    // backward only
    const float* grad_loss;                 // (num_scales + 1)
    float* dfull[MD2_MAX_SCALES];           // per local scale (B,h,w), scales without upsample
    float* upart[MD2_MAX_SCALES];           // per local scale [B][rowblocks][strips][NR][NC], upsampled scales
    float* dP_part[MD2_MAX_SCALES];         // per local scale [S][B*wpi][12]
    // predictive mask (MD2_PREDICTIVE_MASK): per local scale (B,S,h,w)
    const float* mask[MD2_MAX_SCALES];
    float* gmask[MD2_MAX_SCALES];
    // identity losses [S][B][h][w] (forward, written once, read by every scale's waves)
    float* ident;
    // 8-bit copies of the source frames (B,h,w) RGBx and per (frame, image) flags
    // "every colour is exactly k/255" (null: fp32 planes only)
    const uint32_t* src8[MD2_MAX_SRC];
    const int* exact;
    // photo_ident_kernel writes those 8-bit copies itself (it reads every source pixel
    // anyway) when non-null: [S][B][h*w] RGBx, and clears [S][B] flags (preset to 1)
    uint32_t* pack8;
    int* pack_exact;
    // the identity losses are computed inside photo_fwdall_kernel, by the four scale
    // waves of a block (one item) together, into LDS: no photo_ident_kernel, no planes
    int ident_fused;
    // the forward walk's launch also runs the smoothness sums in blocks [fwd_blocks,
    // fwd_blocks + smooth_blocks) (0: a separate smooth_fwd_kernel launch)
    int fwd_blocks, smooth_blocks;
    SmoothArgs sm;
};

__device__ __forceinline__ void make_ctx(const PhotoArgs& a, int ls, int f, int b, WarpCtx& c) {
    const int HW = a.h * a.w;
    c.dh = a.dh[ls];
    c.dw = a.dw[ls];
    c.upsh = a.upsh[ls];
    c.dbf16 = a.disp_bf16 != 0;
    c.disp = disp_off(a.disp[ls], (size_t)b * c.dh * c.dw, c.dbf16);
    c.src = a.src[f] + (size_t)b * 3 * HW;
    c.src8 = (a.src8[f] && (!a.exact || a.exact[f * a.B + b])) ? a.src8[f] + (size_t)b * HW : nullptr;
    c.h = a.h;
    c.w = a.w;
    c.sx = (float)a.w / (float)(a.w - 1);
    c.sy = (float)a.h / (float)(a.h - 1);
    c.min_disp = a.min_disp;
    c.range = a.range;
    load_cam(c.cm, a.K + b * 16, a.iK + b * 16, a.T[ls] + ((size_t)f * a.B + b) * 16);
}

// ----------------------------------------------------------------------------
// Forward: two launches.
//   photo_ident_kernel    identity losses of every source frame, once per step
//                         (scale-invariant, trainer.py:432-439) -> identity planes
//   photo_fwdall_kernel   one wave per (image, 13-row block, strip, scale): window
//                         depths once, then one walk down the rows evaluating every
//                         frame's warp + SSIM/L1 (trainer.py:426-430) with the target's
//                         terms shared, each output row reduced at once to the minimum
//                         over the identity (+ noise) and reprojection candidates
//                         (466-482), automask code, one partial sum per wave
// A 13-row item evaluates 15 rows (1.15x).  Round 2 wrote every reprojection loss
// as a plane (47 MB at B=12) and re-read it in a third launch; those planes are gone,
// and since round 3 the frames no longer walk the rows one after the other through a
// running minimum in LDS (137 -> 124 us at B=12).
// ----------------------------------------------------------------------------
#ifndef MD2_ROWS_P
#define MD2_ROWS_P 13   // 15 window rows; 16 left a 2.06-round grid at B=12 (fwdall 124 -> 118 us)
#endif
constexpr int kRowsP = MD2_ROWS_P;   // output rows per item of the forward passes

// one evaluated window row of the identity walk (target and unwarped source)
struct IRow {
    H5P h;
    C3 x, y;
};

template <bool SSIM_ON>
__device__ __forceinline__ void irow_eval(const float* src, const float* tgt, int HW, int idx, IRow& o) {
    o.x = ld3(src, HW, idx);
    o.y = ld3(tgt, HW, idx);
    if (SSIM_ON) o.h = hsum3(o.x, o.y);
}

// loss of the middle row of (a, b, c) at this lane (trainer.py:393-405)
template <bool SSIM_ON>
__device__ __forceinline__ float irow_loss(const IRow& a, const IRow& b, const IRow& c) {
    const float l1 = sum3(abs3(b.y - b.x));
    return SSIM_ON ? 0.85f * div3(ssim_sum3(a.h, b.h, c.h)) + 0.15f * div3(l1) : div3(l1);
}

// item geometry of the split forward: 62-column strips with one halo lane per side
struct FItem {
    int b, rb, st, r0, c, cc;
    bool colok;
};

__device__ __forceinline__ FItem fitem(const PhotoArgs& a, int t, int lane) {
    FItem it;
    it.st = t % a.strips;
    t /= a.strips;
    it.rb = t % a.rowblocks;
    it.b = t / a.rowblocks;
    it.r0 = it.rb * kRowsP;
    it.c = it.st * kFwdCols - 1 + lane;
    it.cc = reflect_clamp(it.c, a.w);
    it.colok = lane >= 1 && lane <= kFwdCols && it.c < a.w;
    return it;
}

template <int NS, bool SSIM_ON>
__global__ __launch_bounds__(kBlock) void photo_ident_kernel(PhotoArgs a) {
    const int lane = threadIdx.x & (kWave - 1);
    const int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int wv = __builtin_amdgcn_readfirstlane(blk * kWavesPerBlock + (threadIdx.x >> 6));
    if (wv >= a.B * a.wpi * NS) return;
    const int f = wv % NS;
    const FItem it = fitem(a, wv / NS, lane);
    const int h = a.h, w = a.w, HW = h * w;
    WarpCtx ctx;
    ctx.src = a.src[f] + (size_t)it.b * 3 * HW;
    ctx.src8 = nullptr;
    ctx.h = h;
    ctx.w = w;
    float* out = a.ident + ((size_t)f * a.B + it.b) * HW;
    if (a.pack8) {
        // the 8-bit RGBx copy of this wave's own output pixels of source frame f (the
        // pack_src8_kernel arithmetic; these loads also warm the caches for the walk)
        uint32_t* o8 = a.pack8 + ((size_t)f * a.B + it.b) * HW;
        bool ok = true;
        for (int i = 0; i < kRowsP; ++i) {
            const int r = it.r0 + i;
            if (!(it.colok && r < h)) continue;
            uint32_t px = 0u;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch) {
                const float x = ldf(ctx.src, ch * HW + r * w + it.c);
                const float k = rintf(x * 255.0f);
                const bool in = k >= 0.f && k <= 255.f;
                ok = ok && in && div255(k) == x;
                px |= (uint32_t)(in ? k : 0.f) << (8 * ch);
            }
            o8[r * w + it.c] = px;
        }
        if (__ballot(!ok) != 0ull && lane == 0) a.pack_exact[f * a.B + it.b] = 0;
    }
    // window row k = 0 .. kRowsP+1 is image row r0 - 1 + k; rows (k-2, k-1, k) give output
    // row k - 2; the window rotates through three statically named slots (unrolled by 3)
    const float* tgt = a.tgt + (size_t)it.b * 3 * HW;
    auto emit = [&](int i, float v) {
        const int r = it.r0 + i;
        if (it.colok && r < h) out[r * w + it.c] = v;
    };
    IRow R0, R1, R2;
    static_assert((kRowsP + 2) % 3 == 0, "window rows must be a multiple of 3");
#pragma unroll 1
    for (int k = 0; k < kRowsP + 2; k += 3) {
        irow_eval<SSIM_ON>(ctx.src, tgt, HW, reflect_clamp(it.r0 - 1 + k, h) * w + it.cc, R0);
        if (k >= 2) emit(k - 2, irow_loss<SSIM_ON>(R1, R2, R0));
        irow_eval<SSIM_ON>(ctx.src, tgt, HW, reflect_clamp(it.r0 + k, h) * w + it.cc, R1);
        if (k >= 1) emit(k - 1, irow_loss<SSIM_ON>(R2, R0, R1));
        irow_eval<SSIM_ON>(ctx.src, tgt, HW, reflect_clamp(it.r0 + 1 + k, h) * w + it.cc, R2);
        emit(k, irow_loss<SSIM_ON>(R0, R1, R2));
    }
}

// ----------------------------------------------------------------------------
// All-frames forward walk (photo_fwdall_kernel): one pass down the window rows per
// (image, 13-row block, strip, scale) item evaluating every source frame at each row.
// Per row the target's colours, their horizontal sums and the camera ray are formed
// once (not once per frame), the frames' gathers of a row are in flight together, and
// each output row's candidates — identity (+ noise), then the frames in order — are
// reduced to the minimum at once, so no running minimum goes through LDS.
// Arithmetic per frame as the identity walk (irow_eval / irow_loss).
// ----------------------------------------------------------------------------
template <int NS>
struct FRowP {
    C3 y, hy, hyy;                          // target colour, 3-tap sums of y, y^2
    C3 x[NS], hx[NS], hxx[NS], hxy[NS];     // per frame: warped colour, sums of x, x^2, x*y
};

template <int NS, bool SSIM_ON, bool U8>
__device__ __forceinline__ void frowp_eval(const WarpCtx (&c)[NS], const float* tgt, float depth, int rr, int cc,
                                           FRowP<NS>& o) {
    const int HW = c[0].h * c[0].w;
    const float fx = (float)cc, fy = (float)rr;
    float pt[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        pt[i] = depth * (c[0].cm.iK[i * 3 + 0] * fx + c[0].cm.iK[i * 3 + 1] * fy + c[0].cm.iK[i * 3 + 2]);
    o.y = ld3(tgt, HW, rr * c[0].w + cc);
    C3 yl, yr;
    if (SSIM_ON) {
        yl = shfl_prev3(o.y);
        yr = shfl_next3(o.y);
        o.hy = yl + o.y + yr;
        o.hyy = yl * yl + o.y * o.y + yr * yr;
    }
#pragma unroll
    for (int f = 0; f < NS; ++f) {
        FastSample s;
        float cam[3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
            cam[i] = c[f].cm.P[i * 4 + 0] * pt[0] + c[f].cm.P[i * 4 + 1] * pt[1] + c[f].cm.P[i * 4 + 2] * pt[2] +
                     c[f].cm.P[i * 4 + 3];
        const float inv_den = rcpf(cam[2] + 1e-7f);
        const float ix = cam[0] * inv_den * c[f].sx - 0.5f, iy = cam[1] * inv_den * c[f].sy - 0.5f;
        const float xmax = (float)(c[f].w - 1), ymax = (float)(c[f].h - 1);
        const float ixc = fminf(fmaxf(ix, 0.f), xmax), iyc = fminf(fmaxf(iy, 0.f), ymax);
        const float fx0 = floorf(ixc), fy0 = floorf(iyc);
        s.x0 = (int)fx0;
        s.y0 = (int)fy0;
        s.tx = ixc - fx0;
        s.ty = iyc - fy0;
        Corners v;
        gather<U8>(c[f], s, v);
        o.x[f] = interp3<U8>(s, v);
        if (SSIM_ON) {
            const C3 xl = shfl_prev3(o.x[f]), xr = shfl_next3(o.x[f]);
            o.hx[f] = xl + o.x[f] + xr;
            o.hxx[f] = xl * xl + o.x[f] * o.x[f] + xr * xr;
            o.hxy[f] = xl * yl + o.x[f] * o.y + xr * yr;
        }
    }
}

template <int NS, bool SSIM_ON>
__device__ __forceinline__ void frowp_losses(const FRowP<NS>& A, const FRowP<NS>& B, const FRowP<NS>& C,
                                             float (&loss)[NS]) {
    C3 my, sy;
    if (SSIM_ON) {
        my = (A.hy + B.hy + C.hy) * kInv9;
        sy = (A.hyy + B.hyy + C.hyy) * kInv9 - my * my;
    }
#pragma unroll
    for (int f = 0; f < NS; ++f) {
        const float l1 = sum3(abs3(B.y - B.x[f]));
        if (SSIM_ON) {
            const C3 mx = (A.hx[f] + B.hx[f] + C.hx[f]) * kInv9;
            const C3 sx = (A.hxx[f] + B.hxx[f] + C.hxx[f]) * kInv9 - mx * mx;
            const C3 sxy = (A.hxy[f] + B.hxy[f] + C.hxy[f]) * kInv9 - mx * my;
            const C3 n = (mx * my * 2.f + kC1) * (sxy * 2.f + kC2);
            const C3 d = (mx * mx + my * my + kC1) * (sx + sy + kC2);
            const float ss = clamp01((1.f - n.a.x * rcpf(d.a.x)) * 0.5f) + clamp01((1.f - n.a.y * rcpf(d.a.y)) * 0.5f) +
                             clamp01((1.f - n.b * rcpf(d.b)) * 0.5f);
            loss[f] = 0.85f * div3(ss) + 0.15f * div3(l1);
        } else {
            loss[f] = div3(l1);
        }
    }
}

// one identity-walk row with the source from its 8-bit copy: k / 255 decoded correctly
// rounded (div255) is the fp32 colour itself for an exact image, so the losses are
// bit-identical to irow_eval's, from 4 bytes per pixel instead of 12
template <bool SSIM_ON>
__device__ __forceinline__ void irow_eval8(const uint32_t* src8, const float* tgt, int HW, int idx, IRow& o) {
    const uint32_t px = src8[(uint32_t)idx];
    o.x = {f2v{div255((float)(px & 255u)), div255((float)((px >> 8) & 255u))}, div255((float)((px >> 16) & 255u))};
    o.y = ld3(tgt, HW, idx);
    if (SSIM_ON) o.h = hsum3(o.x, o.y);
}

// identity losses (trainer.py:432-439) of source frame f for the item's output rows
// [i0, i1) into LDS rows dst[i] (the photo_ident_kernel walk, rows rotated by copies);
// src8: the frame's exact 8-bit copy for this image, or null (fp32 planes)
template <bool SSIM_ON>
__device__ __forceinline__ void ident_rows_lds(const PhotoArgs& a, int f, const uint32_t* src8, const FItem& it,
                                               int i0, int i1, float (*dst)[kWave], int lane) {
    const int h = a.h, w = a.w, HW = h * w;
    const float* src = a.src[f] + (size_t)it.b * 3 * HW;
    const float* tgt = a.tgt + (size_t)it.b * 3 * HW;
    auto row = [&](int r, IRow& o) {
        const int idx = reflect_clamp(r, h) * w + it.cc;
        if (src8) irow_eval8<SSIM_ON>(src8, tgt, HW, idx, o);
        else irow_eval<SSIM_ON>(src, tgt, HW, idx, o);
    };
    IRow A, Bq, C;
    row(it.r0 + i0 - 1, A);
    row(it.r0 + i0, Bq);
#pragma unroll 1
    for (int i = i0; i < i1; ++i) {
        row(it.r0 + i + 1, C);
        dst[i][lane] = irow_loss<SSIM_ON>(A, Bq, C);
        A = Bq;
        Bq = C;
    }
}

template <int NS, bool SSIM_ON, bool MASK, bool U8, bool IDL>
__device__ __forceinline__ float fwdall_walk(const PhotoArgs& a, const WarpCtx (&ctx)[NS], const FItem& it, int ls,
                                             const float (*dep)[kWave], const float (*idl)[kRowsP][kWave],
                                             int lane) {
    const int h = a.h, w = a.w, HW = h * w;
    const bool automask = !(a.flags & MD2_NO_AUTOMASK);
    const bool avg = (a.flags & MD2_AVG_REPROJECTION) != 0;
    const int C = avg ? 1 : NS;
    const uint64_t seed = a.seed_ptr ? (a.seed ^ (*a.seed_ptr * 0x9E3779B97F4A7C15ULL)) : a.seed;
    const uint32_t key = noise_key(seed, a.gscale[ls]);
    const float* nz = a.noise[ls];
    const float* tgt = a.tgt + (size_t)it.b * 3 * HW;
    uint8_t* sel = a.sel[ls] + (size_t)it.b * HW;
    float lsum = 0.f;
    // output row i = window row k - 2 from rows (k-2, k-1, k)
    using Row = FRowP<NS>;
    auto out_row = [&](int i, const Row& A, const Row& B, const Row& Cr) {
        float lf[NS];
        frowp_losses<NS, SSIM_ON>(A, B, Cr, lf);
        const int r = it.r0 + i;
        if (!(it.colok && r < h)) return;
        const int p = r * w + it.c;
        float bv = INFINITY;
        int bc = 0;
        if (automask) {   // identity candidates + tie-break noise (trainer.py:466-471)
            float nv[NS];
            if (nz) {
#pragma unroll
                for (int ch = 0; ch < NS; ++ch) nv[ch] = ch < C ? nz[((size_t)it.b * C + ch) * HW + p] : 0.f;
            } else {
#pragma unroll
                for (int j = 0; 2 * j < NS; ++j) {
                    const float2 n2 = noise_pair(key, (uint32_t)(it.b * HW + p), j);
                    nv[2 * j] = n2.x;
                    if (2 * j + 1 < NS) nv[2 * j + 1] = n2.y;
                }
            }
            float id[NS];
#pragma unroll
            for (int f = 0; f < NS; ++f)
                id[f] = IDL ? idl[f][i][lane] : a.ident[((size_t)f * a.B + it.b) * HW + p];
            for (int ch = 0; ch < C; ++ch) {
                float v;
                if (avg) {
                    v = 0.f;
#pragma unroll
                    for (int f = 0; f < NS; ++f) v += id[f];
                    v = v / (float)NS;
                } else {
                    v = id[ch];
                }
                v = v + nv[ch] * 1e-5f;
                if (v < bv) {
                    bv = v;
                    bc = ch;
                }
            }
        }
        float accv = 0.f;
#pragma unroll
        for (int f = 0; f < NS; ++f) {
            float v = lf[f];
            if (MASK) v *= a.mask[ls][((size_t)it.b * NS + f) * HW + p];   // trainer.py:455
            if (avg) {
                accv += v;
            } else if (v < bv) {
                bv = v;
                bc = (automask ? NS : 0) + f;
            }
        }
        if (avg) {
            const float ra = accv / (float)NS;
            if (automask) {
                if (ra < bv) {
                    bv = ra;
                    bc = 1;
                }
            } else {
                bv = ra;
            }
        }
        lsum += bv;
        sel[p] = (uint8_t)bc;
    };
    Row R0, R1, R2;
    static_assert((kRowsP + 2) % 3 == 0, "window rows must be a multiple of 3");
#pragma unroll 1
    for (int k = 0; k < kRowsP + 2; k += 3) {
        frowp_eval<NS, SSIM_ON, U8>(ctx, tgt, dep[k][lane], reflect_clamp(it.r0 - 1 + k, h), it.cc, R0);
        if (k >= 2) out_row(k - 2, R1, R2, R0);
        frowp_eval<NS, SSIM_ON, U8>(ctx, tgt, dep[k + 1][lane], reflect_clamp(it.r0 + k, h), it.cc, R1);
        if (k >= 1) out_row(k - 1, R2, R0, R1);
        frowp_eval<NS, SSIM_ON, U8>(ctx, tgt, dep[k + 2][lane], reflect_clamp(it.r0 + 1 + k, h), it.cc, R2);
        out_row(k, R0, R1, R2);
    }
    return lsum;
}

// MD2_FWD_MINB: blocks per CU (= waves per SIMD) the forward walk is compiled for.
// Round 4: 4 — with the identity losses read from LDS the compiler's own choice is 152
// VGPRs (3 waves); at 4 it keeps 128 and spills ~21 dwords outside the row loop's hot
// path: fused forward 0.1245 vs 0.128 ms (profiles/r04/ab_fused_forward.log)
// Three source frames (mono + stereo) carry half as much state again: 2 (~194 VGPRs).
#ifndef MD2_FWD_MINB
#define MD2_FWD_MINB 4
#endif
template <int NS, bool SSIM_ON, bool MASK>
__global__ __launch_bounds__(kBlock, NS <= 2 ? MD2_FWD_MINB : 2) void photo_fwdall_kernel(PhotoArgs a) {
    __shared__ float dep_s[kWavesPerBlock][kRowsP + 2][kWave];
    __shared__ float idl_s[NS][kRowsP][kWave];   // ident_fused: the item's identity losses
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x >> 6;
    float (*dep)[kWave] = dep_s[wid];
    if (a.smooth_blocks && (int)blockIdx.x >= a.fwd_blocks) {   // block-uniform: a smoothness block
        // (fwd_blocks % 8 == 0: the XCD-contiguous numbering of the tail grid holds)
        smooth_block(a.sm, xcd_contiguous_block((int)blockIdx.x - a.fwd_blocks, a.smooth_blocks));
        return;
    }
    const int blk = xcd_contiguous_block(blockIdx.x, a.smooth_blocks ? a.fwd_blocks : (int)gridDim.x);
    const int wv = __builtin_amdgcn_readfirstlane(blk * kWavesPerBlock + wid);
    if (wv >= a.B * a.wpi * a.nsc) return;   // never with ident_fused (exact grid: no barrier skipped)
    const int ls = wv % a.nsc;   // scale fastest: the waves sharing a strip's rows run together
    const int item = wv / a.nsc;
    const FItem it = fitem(a, item, lane);
    WarpCtx ctx[NS];
    bool u8 = true;
#pragma unroll
    for (int f = 0; f < NS; ++f) {
        make_ctx(a, ls, f, it.b, ctx[f]);
        u8 = u8 && ctx[f].src8 != nullptr;
    }
#pragma unroll
    for (int k = 0; k < kRowsP + 2; ++k) dep[k][lane] = depth_at(ctx[0], reflect_clamp(it.r0 - 1 + k, a.h), it.cc);
    const float (*idl)[kRowsP][kWave] = nullptr;
    if (a.ident_fused) {
        // the four waves of the block are the four scales of ONE item (nsc == 4): the
        // identity losses, scale-invariant, are computed once for all of them — the
        // tasks (frame, upper / lower half of the item's rows) spread over the waves
        constexpr int kMid = (kRowsP + 1) / 2;
        const int rows = min(kRowsP, a.h - it.r0);
        for (int task = wid; task < 2 * NS; task += kWavesPerBlock) {
            const int f = task >> 1, i0 = (task & 1) ? kMid : 0, i1 = (task & 1) ? rows : min(kMid, rows);
            // ctx[f] by selects: indexing the array with a runtime f would put all of
            // ctx in scratch memory (320 B per lane, written out by every wave)
            const uint32_t* src8 = ctx[0].src8;
#pragma unroll
            for (int g = 1; g < NS; ++g) src8 = f == g ? ctx[g].src8 : src8;
            if (i0 < i1) ident_rows_lds<SSIM_ON>(a, f, src8, it, i0, i1, idl_s[f], lane);
        }
        __syncthreads();
        idl = idl_s;
    }
    // every frame's sources 8-bit exact (wave-uniform), else all frames on the fp32 planes
    float lsum;
    if (idl)
        lsum = u8 ? fwdall_walk<NS, SSIM_ON, MASK, true, true>(a, ctx, it, ls, dep, idl, lane)
                  : fwdall_walk<NS, SSIM_ON, MASK, false, true>(a, ctx, it, ls, dep, idl, lane);
    else
        lsum = u8 ? fwdall_walk<NS, SSIM_ON, MASK, true, false>(a, ctx, it, ls, dep, idl, lane)
                  : fwdall_walk<NS, SSIM_ON, MASK, false, false>(a, ctx, it, ls, dep, idl, lane);
    const float t = wave_sum(lsum);
    if (lane == 0) a.photo_part[ls][item] = t;
}

// 8-bit source copies: every source colour x with x == RN(k/255) for k = rint(255 x)
// (k/255 by a correctly rounded 3-op Markstein division, exhaustively checked for
// k = 0..255) is stored as byte k of its pixel's RGBx dword; one inexact colour of an
// image clears that image's flag and its gathers read the fp32 planes instead.
struct PackArgs {
    int B, HW, S;
    const float* src[MD2_MAX_SRC];   // (B,3,h,w)
    uint32_t* out;                   // [S][B][HW]
    int* exact;                      // [S][B], preset to nonzero
};

__global__ __launch_bounds__(kBlock) void pack_src8_kernel(PackArgs a) {
    const int per_img = (a.HW + 4 * kBlock - 1) / (4 * kBlock);
    const int fb = blockIdx.x / per_img, chunk = blockIdx.x - fb * per_img;
    const int f = fb / a.B, b = fb - f * a.B;
    const int p0 = (chunk * kBlock + threadIdx.x) * 4;
    const float* src = a.src[f] + (size_t)b * 3 * a.HW;
    uint32_t* out = a.out + ((size_t)f * a.B + b) * a.HW;
    bool ok = true;
    if (p0 < a.HW) {
        const int n = min(4, a.HW - p0);
        uint32_t px[4] = {0u, 0u, 0u, 0u};
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            float x[4];
            if (n == 4 && (a.HW & 3) == 0) {
                const float4 v = *(const float4*)(src + ch * a.HW + p0);
                x[0] = v.x, x[1] = v.y, x[2] = v.z, x[3] = v.w;
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) x[i] = i < n ? src[ch * a.HW + p0 + i] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float k = rintf(x[i] * 255.0f);
                ok = ok && k >= 0.f && k <= 255.f && div255(k) == x[i];
                px[i] |= (uint32_t)(k >= 0.f && k <= 255.f ? k : 0.f) << (8 * ch);
            }
        }
        if (n == 4 && (a.HW & 3) == 0) {
            *(uint4*)(out + p0) = make_uint4(px[0], px[1], px[2], px[3]);
        } else {
            for (int i = 0; i < n; ++i) out[p0 + i] = px[i];
        }
    }
    // a wave that saw an inexact colour clears the image's flag: a plain store of 0
    // (flags only ever go 1 -> 0, so racing writers agree; no read-modify-write)
    if (__ballot(!ok) != 0ull && (threadIdx.x & 63) == 0) a.exact[f * a.B + b] = 0;
}

// ----------------------------------------------------------------------------
// backward: SSIM/L1 adjoint -> grid_sample backward -> projection chain
// ----------------------------------------------------------------------------
// ---- adjoint of the bilinear upsample (trainer.py:350-351), item by item -------------
// A backward item (60 columns x kRowsB rows of one scale's full-resolution grid) folds
// its dL/d(upsampled disp) straight into the native-resolution pixels it touches: a
// partial grid of NR x NC native pixels starting at (ilo, jlo), written once per item.
// disp_grad_kernel then sums the <= 2 x 2 partials of the items whose pixels reach a
// native pixel (the footprint of a native pixel spans 2^(s+1) <= 16 full-resolution
// rows / columns, less than an item), in a fixed order.  This replaces a full-resolution
// dL/d(upsampled disp) plane per scale written here and gathered with a 2^(s+1) x
// 2^(s+1) footprint per native pixel there (~170 MB of L2 traffic per step at B=12).
__host__ __device__ __forceinline__ int up_nc(int upsh) { return (kBwdCols + (1 << upsh) - 1) / (1 << upsh) + 2; }
__host__ __device__ __forceinline__ int up_nr(int upsh) { return (kRowsB + (1 << upsh) - 1) / (1 << upsh) + 2; }
// weight of low-res index i in the upsample of full-res index y (factor 2^sh)
__device__ __forceinline__ float up_weight(int y, int i, int n_in, float sc) {
    const float sy = fmaxf(((float)y + 0.5f) * sc - 0.5f, 0.f);
    const int y0 = min((int)sy, n_in - 1);
    const int y1 = y0 + (y0 < n_in - 1 ? 1 : 0);
    const float l1 = fminf(fmaxf(sy - (float)y0, 0.f), 1.f);
    return (y0 == i ? 1.f - l1 : 0.f) + (y1 == i ? l1 : 0.f);
}
// lower source index of full-resolution index x (ATen area_pixel_compute_source_index,
// align_corners=False, as disp_at / up_weight)
__device__ __forceinline__ int up_src0(int x, int n_in, float sc) {
    const float sx = fmaxf(((float)x + 0.5f) * sc - 0.5f, 0.f);
    return min((int)sx, n_in - 1);
}

// weight of the reflection-padded 3-tap adjoint: how often neighbour (i-1) / (i+1)
// contributes to position i (reflection pad folds index -1 onto 1 and n onto n-2)
__device__ __forceinline__ float fold_lo(int i) { return i == 0 ? 0.f : (i == 1 ? 2.f : 1.f); }
__device__ __forceinline__ float fold_hi(int i, int n) { return i == n - 1 ? 0.f : (i == n - 2 ? 2.f : 1.f); }

// fold weight x value.  The values reaching here are finite (SSIM adjoint terms,
// zeroed where the loss weight is 0; halo lanes read reflect-clamped pixels), so the
// plain product equals the select form (w == 0 -> 0) and costs one instruction.
__device__ __forceinline__ float pick(float wgt, float v) { return wgt * v; }

template <int NS>
__device__ __forceinline__ float frame_weight(int code, int f, bool automask, bool avg) {
    if (avg) {
        if (automask) return code == 1 ? 1.f / (float)NS : 0.f;
        return 1.f / (float)NS;
    }
    return code == (automask ? NS : 0) + f ? 1.f : 0.f;
}

// Per-(item, frame) constants of the backward.
struct BwdFrame {
    WarpCtx ctx;
    const float* tgt;
    const uint8_t* sel;
    const float* pmask;
    float* pgmask;
    const float (*dep)[kWave];   // LDS: depth of window rows k = 0 .. kRowsB+3 (frame-independent)
    int b, f, r0, c, cc;
    bool colok, colreal, automask, avg;
    float wl, wr, gscale;
};

// Carried two rows down the sliding window from an output row's own forward sample
// (instead of re-projecting and re-gathering it): the bilinear slopes and the
// perspective terms.  The rest of the projection chain (ray, camera point, dcam/ddepth)
// is recomputed at the output step from the row's depth in LDS with the same
// expressions (ray_at, the same products), so it rounds exactly as the carried values
// did, while the three ring slots carry 9 floats each instead of 16.
struct CarryP {
    C3 jx, jy;
    float px, py, inv_den;
};
struct RowP {
    H5P h;
    C3 x, y;
    CarryP k;
};
struct CoefP {
    C3 A, B, C;
    float g;
};

// A window row whose projection is done and whose loads are in flight.  The walk is
// software-pipelined by one row: row k+1's corner gathers, target colours and the
// argmin code its step needs are issued right after row k's loads are consumed, so
// row k's SSIM adjoint and output step (most of a step's VALU work) cover their
// latency instead of every step waiting on its own gathers.
template <bool U8>
struct PendRaw;
template <>
struct PendRaw<true> {
    uint2_a4 t, u;            // RGBx corner pairs of the top / bottom row
};
template <>
struct PendRaw<false> {
    float2_a4 t[3], u[3];     // per channel
};
template <bool U8>
struct PendRow {
    float tx, ty, px, py, inv_den, gmx, gmy;
    bool vx1, vy1;
    PendRaw<U8> raw;
    C3 y;
    int code;                 // argmin code of the coefficient row of the step (trainer.py:478)
};

// project window row k at its depth (from LDS, read by the caller) and issue its loads
template <bool U8>
__device__ __forceinline__ void bwd_issue(const BwdFrame& F, int k, float depth, PendRow<U8>& pd) {
    const int h = F.ctx.h, w = F.ctx.w, HW = h * w;
    const int r = F.r0 - 2 + k;
    const int rr = reflect_clamp(r, h);
    FastSample sm;
    project_depth(F.ctx, rr, F.cc, depth, sm);
    pd.tx = sm.tx;
    pd.ty = sm.ty;
    pd.px = sm.px;
    pd.py = sm.py;
    pd.inv_den = sm.inv_den;
    pd.gmx = sm.gmx;
    pd.gmy = sm.gmy;
    pd.vx1 = sm.x0 + 1 < w;
    pd.vy1 = sm.y0 + 1 < h;
    const int y1 = pd.vy1 ? sm.y0 + 1 : sm.y0;
    const int xa = pd.vx1 ? sm.x0 : sm.x0 - 1;
    const int ot = sm.y0 * w + xa, ob = y1 * w + xa;
    if constexpr (U8) {
        pd.raw.t = *(const uint2_a4*)((const char*)F.ctx.src8 + ((uint32_t)ot << 2));
        pd.raw.u = *(const uint2_a4*)((const char*)F.ctx.src8 + ((uint32_t)ob << 2));
    } else {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            pd.raw.t[ch] = ldf2(F.ctx.src, ch * HW + ot);
            pd.raw.u[ch] = ldf2(F.ctx.src, ch * HW + ob);
        }
    }
    pd.y = ld3(F.tgt, HW, rr * w + F.cc);
    // coefficient row p = r - 1, read at a clamped address (used only where it is real)
    const int p = min(max(r - 1, 0), h - 1);
    pd.code = ldb(F.sel, p * w + F.cc);
}

// the four masked corners of a pending row (gather()'s selects)
template <bool U8>
__device__ __forceinline__ void bwd_corners(const PendRow<U8>& pd, Corners& v) {
    const bool vx1 = pd.vx1, vy1 = pd.vy1;
    if constexpr (U8) {
        const uint2_a4 t = pd.raw.t, u = pd.raw.u;
        const uint32_t pnw = vx1 ? t.x : t.y, pne = vx1 ? t.y : 0u;
        const uint32_t psw = vy1 ? (vx1 ? u.x : u.y) : 0u, pse = (vx1 && vy1) ? u.y : 0u;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            v.nw[ch] = (float)((pnw >> (8 * ch)) & 255u);
            v.ne[ch] = (float)((pne >> (8 * ch)) & 255u);
            v.sw[ch] = (float)((psw >> (8 * ch)) & 255u);
            v.se[ch] = (float)((pse >> (8 * ch)) & 255u);
        }
    } else {
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
            const float2_a4 t = pd.raw.t[ch], u = pd.raw.u[ch];
            v.nw[ch] = vx1 ? t.x : t.y;
            v.ne[ch] = vx1 ? t.y : 0.f;
            v.sw[ch] = vy1 ? (vx1 ? u.x : u.y) : 0.f;
            v.se[ch] = (vx1 && vy1) ? u.y : 0.f;
        }
    }
}

template <bool U8, class SampleT>
__device__ __forceinline__ void make_carry3(const WarpCtx& c, const SampleT& s, const Corners& v, CarryP& k) {
    const float e = 1.f - s.tx, so = 1.f - s.ty;
    const float cs = U8 ? 1.0f / 255.0f : 1.0f;
    const float mx = s.gmx * c.sx * cs, my = s.gmy * c.sy * cs;
    const C3 nw = {f2v{v.nw[0], v.nw[1]}, v.nw[2]}, ne = {f2v{v.ne[0], v.ne[1]}, v.ne[2]};
    const C3 sw = {f2v{v.sw[0], v.sw[1]}, v.sw[2]}, se = {f2v{v.se[0], v.se[1]}, v.se[2]};
    k.jx = ((ne - nw) * so + (se - sw) * s.ty) * mx;
    k.jy = ((sw - nw) * e + (se - ne) * s.tx) * my;
    k.px = s.px;
    k.py = s.py;
    k.inv_den = s.inv_den;
}

// One step of the backward row walk at window index k (row r = r0 - 2 + k):
//   row r from the pending loads (warp, target, horizontal sums, carry) into `cur`,
//   then row k+1's loads are issued into `pd`;
//   k >= 2: SSIM adjoint coefficients of row p = r - 1 into `cnew` (from the sums of
//           rows r-2, r-1, r = m2, m1, cur);
//   k >= 4: output row q = r - 2: dL/dwarp from coefficient rows q-1, q, q+1
//           (cm3, cm2, cnew) + the L1 term, through the carried bilinear slopes and
//           projection into dL/dP and dL/d(upsampled disp).
// The window state lives in three statically named ring slots (rows and coefficient
// rows mod 3) that the caller rotates by unrolling three steps, so moving the window
// down costs no register copies; every slot is updated unconditionally.
template <int NS, bool SSIM_ON, bool MASK, bool U8>
__device__ __forceinline__ void bwd_step(const BwdFrame& F, int k, PendRow<U8>& pd, RowP& cur, const RowP& m1,
                                         const RowP& m2, CoefP& cnew, const CoefP& cm2, const CoefP& cm3,
                                         float (&dP)[12], float (*ddacc)[kWave], int lane) {
    constexpr float kThird = 1.0f / 3.0f;
    constexpr int kSteps = kRowsB + 4;
    const float l1w = SSIM_ON ? 0.15f : 1.0f;
    const int h = F.ctx.h, w = F.ctx.w;
    const int r = F.r0 - 2 + k;
    const int q = r - 2;
    // this step's LDS operands, read up front so their latency hides behind the row's
    // interpolation and sums: the next row's depth (its projection), the output row's
    // depth (its recomputed projection chain) and the frames' running dL/ddepth
    const int kn = U8 ? min(k + 1, kSteps - 1) : k;
    const float dep_next = F.dep[kn][lane];
    const bool outrow = k >= 4 && F.colok && q < h;
    const float dep_out = k >= 4 ? F.dep[k - 2][lane] : 0.f;
    const float dd_old = (outrow && F.f != 0) ? ddacc[q - F.r0][lane] : 0.f;
    // the fp32-plane path (12 corner floats per row in flight) issues its own row here:
    // pipelined it would not fit the register file
    if constexpr (!U8) bwd_issue<U8>(F, k, dep_next, pd);
    {
        Corners v;
        bwd_corners<U8>(pd, v);
        cur.x = interp3<U8>(pd, v);
        cur.y = pd.y;
        if (k >= 2 && k < kRowsB + 2) make_carry3<U8>(F.ctx, pd, v, cur.k);   // only output rows need it
    }
    if (SSIM_ON) cur.h = hsum3(cur.x, cur.y);
    const int code = pd.code;
    // the next row's loads (the last step re-issues its own row: same addresses, unused)
    if constexpr (U8) bwd_issue<U8>(F, kn, dep_next, pd);
    if (k < 2) return;
    // coefficient row p = r - 1
    const int p = r - 1;
    float gp = 0.f;
    const bool own = F.colreal && p >= 0 && p < h;
    if (own) gp = F.gscale * frame_weight<NS>(code, F.f, F.automask, F.avg);
    if (MASK) {
        // masked = reproj * mask (trainer.py:455): d/dreproj = g*mask, d/dmask = g*reproj
        const size_t mi = (((size_t)F.b * NS + F.f) * h + (own ? p : 0)) * w + (own ? F.c : 0);
        if (F.pgmask && F.colok && p >= F.r0 && p < F.r0 + kRowsB && p < h) {
            const float ss = SSIM_ON ? ssim_sum3(m2.h, m1.h, cur.h) : 0.f;
            const float l1 = sum3(abs3(m1.y - m1.x));
            const float rep = SSIM_ON ? 0.85f * div3(ss) + 0.15f * div3(l1) : div3(l1);
            F.pgmask[mi] = gp * rep;
        }
        gp *= own ? F.pmask[mi] : 0.f;
    }
    cnew.g = gp;
    if (SSIM_ON) {
        // gp == 0 (a pixel this frame does not win) zeroes dA, dB, dC through the clamp
        // pass already (every factor is finite: d >= C1 C2 > 0)
        const float gS = gp * (0.85f / 3.f);
        C3 dA, dB, dC;
        ssim_adjoint3(m2.h, m1.h, cur.h, gS, dA, dB, dC);
        cnew.A = shfl_prev3(dA) * F.wl + dA + shfl_next3(dA) * F.wr;
        cnew.B = shfl_prev3(dB) * F.wl + dB + shfl_next3(dB) * F.wr;
        cnew.C = shfl_prev3(dC) * F.wl + dC + shfl_next3(dC) * F.wr;
    }
    if (k < 4) return;
    // output row q = r - 2 (coefficient rows q-1, q, q+1 = cm3, cm2, cnew)
    if (!outrow) return;
    const CarryP& k2 = m2.k;
    const float l1c = cm2.g * (l1w * kThird);
    C3 g = sign3(m2.x - m2.y) * l1c;
    if (SSIM_ON) {
        const float wu = fold_lo(q), wd = fold_hi(q, h);
        const C3 aA = cm3.A * wu + cm2.A + cnew.A * wd;
        const C3 aB = cm3.B * wu + cm2.B + cnew.B * wd;
        const C3 aC = cm3.C * wu + cm2.C + cnew.C * wd;
        g = g + (aA + m2.x * 2.f * aB + m2.y * aC) * kInv9;
    }
    const float dpx = sum3(g * k2.jx), dpy = sum3(g * k2.jy);
    float dc[3];
    dc[0] = dpx * k2.inv_den;
    dc[1] = dpy * k2.inv_den;
    dc[2] = -(dpx * k2.px + dpy * k2.py) * k2.inv_den;
    // the sample's ray / camera point / dcam-ddepth, recomputed (output rows are inside
    // the image, so the sample row was q itself, unreflected)
    const float depth = dep_out;
    const float fx = (float)F.cc, fy = (float)q;
    float ray[3], pt[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        ray[i] = ray_at(F.ctx.cm, i, fx, fy);
        pt[i] = depth * ray[i];
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) dP[i * 4 + j] += dc[i] * pt[j];
        dP[i * 4 + 3] += dc[i];
    }
    float u[3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
        u[i] = F.ctx.cm.P[i * 4 + 0] * ray[0] + F.ctx.cm.P[i * 4 + 1] * ray[1] + F.ctx.cm.P[i * 4 + 2] * ray[2];
    const float ddd = -F.ctx.range * depth * depth;
    const float dd = (dc[0] * u[0] + dc[1] * u[1] + dc[2] * u[2]) * ddd;
    ddacc[q - F.r0][lane] = F.f == 0 ? dd : dd_old + dd;
}

template <int NS, bool SSIM_ON, bool MASK, bool U8>
__device__ __forceinline__ void bwd_frame_walk(const BwdFrame& F, float (*ddacc)[kWave], float* dst, int lane) {
    float dP[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) dP[j] = 0.f;
    RowP S0, S1, S2;
    CoefP C0, C1, C2;
    PendRow<U8> pd;
    constexpr int kSteps = kRowsB + 4;
    if constexpr (U8) bwd_issue<U8>(F, 0, F.dep[0][lane], pd);
    int k = 0;
#pragma unroll 1
    for (; k + 3 <= kSteps; k += 3) {
        bwd_step<NS, SSIM_ON, MASK, U8>(F, k + 0, pd, S0, S2, S1, C2, C1, C0, dP, ddacc, lane);
        bwd_step<NS, SSIM_ON, MASK, U8>(F, k + 1, pd, S1, S0, S2, C0, C2, C1, dP, ddacc, lane);
        bwd_step<NS, SSIM_ON, MASK, U8>(F, k + 2, pd, S2, S1, S0, C1, C0, C2, dP, ddacc, lane);
    }
    if (kSteps % 3 >= 1) bwd_step<NS, SSIM_ON, MASK, U8>(F, k + 0, pd, S0, S2, S1, C2, C1, C0, dP, ddacc, lane);
    if (kSteps % 3 >= 2) bwd_step<NS, SSIM_ON, MASK, U8>(F, k + 1, pd, S1, S0, S2, C0, C2, C1, dP, ddacc, lane);
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        const float t = wave_sum(dP[j]);
        if (lane == 0) dst[j] = t;
    }
}

// One work item of the backward: (image b, local scale ls, strip st, row block rb),
// all source frames.  Writes dL/d(upsampled disp) for its 60 x kRowsB pixels and one
// 12-float dL/dP partial per frame.
template <int NS, bool SSIM_ON, bool MASK>
__device__ __forceinline__ void bwd_item(const PhotoArgs& a, int b, int ls, int st, int rb, int lane,
                                         float (*ddacc)[kWave], float (*dep)[kWave]) {
    BwdFrame F;
    F.r0 = rb * kRowsB;
    const int h = a.h, w = a.w, HW = h * w;
    F.b = b;
    F.c = st * kBwdCols - 2 + lane;
    F.cc = reflect_clamp(F.c, w);
    F.colok = lane >= 2 && lane < 2 + kBwdCols && F.c < w;
    F.colreal = F.c >= 0 && F.c < w;
    F.wl = fold_lo(F.c);
    F.wr = fold_hi(F.c, w);
    F.tgt = a.tgt + (size_t)b * 3 * HW;
    F.automask = !(a.flags & MD2_NO_AUTOMASK);
    F.avg = (a.flags & MD2_AVG_REPROJECTION) != 0;
    const int gsc = a.gscale[ls];
    F.gscale = (a.grad_loss[gsc] + a.grad_loss[a.num_scales] / (float)a.num_scales) / ((float)a.B * (float)HW);
    F.sel = a.sel[ls] + (size_t)b * HW;
    const int item_in_scale = b * a.wpi + rb * a.strips + st;
    F.pmask = MASK ? a.mask[ls] : nullptr;
    F.pgmask = MASK ? a.gmask[ls] : nullptr;
    F.dep = dep;
    // the window's depths once per item (both frames warp the same upsampled disparity):
    // all taps issued together instead of one dependent load pair per row and frame
    make_ctx(a, ls, 0, b, F.ctx);
#pragma unroll
    for (int k = 0; k < kRowsB + 4; ++k) dep[k][lane] = depth_at(F.ctx, reflect_clamp(F.r0 - 2 + k, h), F.cc);

    for (int f = 0; f < NS; ++f) {
        F.f = f;
        make_ctx(a, ls, f, b, F.ctx);
        float* dst = a.dP_part[ls] + ((size_t)f * a.B * a.wpi + item_in_scale) * 12;
        if (F.ctx.src8)
            bwd_frame_walk<NS, SSIM_ON, MASK, true>(F, ddacc, dst, lane);
        else
            bwd_frame_walk<NS, SSIM_ON, MASK, false>(F, ddacc, dst, lane);
    }
    const int upsh = a.upsh[ls];
    if (upsh == 0) {   // no upsample: dL/d(disp) at this resolution, written once
        float* dfull = a.dfull[ls] + (size_t)b * HW;
        if (F.colok)
            for (int i = 0; i < kRowsB && F.r0 + i < h; ++i) dfull[(F.r0 + i) * w + F.c] = ddacc[i][lane];
        return;
    }
    // fold into the native pixels: horizontal adjoint of the item's rows into R (LDS,
    // the item's depth rows are no longer needed), then vertical into the partial grid
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int kf = 1 << upsh, half = kf >> 1;
    const float sc = 1.0f / (float)kf;
    const int dh = a.dh[ls], dw = a.dw[ls];
    const int NC = up_nc(upsh), NR = up_nr(upsh);
    const int X0 = st * kBwdCols, X1 = min(X0 + kBwdCols, w), Y0 = F.r0, Y1 = min(F.r0 + kRowsB, h);
    const int jlo = up_src0(X0, dw, sc), ilo = up_src0(Y0, dh, sc);
    float* R = &dep[0][0];   // [kRowsB][NC]
    // lanes 0 .. G*NC-1 own native column jc = lane % NC and every G-th row; the column's
    // taps (<= 2^(s+1) full-resolution columns of this item) and weights once per item
    const int G = kWave / NC, gi = lane / NC, jc = lane - gi * NC, j = jlo + jc;
    const bool jlive = gi < G && j < dw;
    const int xa = max(X0, kf * (j - 1) + half), xb = jlive ? min(X1, kf * (j + 1) + half) : xa;
    float wx[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) wx[t] = (xa + t < xb) ? up_weight(xa + t, j, dw, sc) : 0.f;
    const int nt = xb - xa;
    for (int yi = gi; yi < kRowsB; yi += G) {
        if (!jlive) break;
        float sum = 0.f;
        if (Y0 + yi < Y1) {
            const float* drow = &ddacc[yi][xa - X0 + 2];
#pragma unroll
            for (int t = 0; t < 16; ++t)
                if (t < nt) sum += wx[t] * drow[t];
        }
        R[yi * NC + jc] = sum;
    }
    float* part = a.upart[ls] + (size_t)item_in_scale * NR * NC;
    if (gi < G) {
        for (int ic = gi; ic < NR; ic += G) {
            const int i = ilo + ic;
            float sum = 0.f;
            if (i < dh) {
                const int ya = max(Y0, kf * (i - 1) + half), yb = min(Y1, kf * (i + 1) + half);
                for (int y = ya; y < yb; ++y) sum += up_weight(y, i, dh, sc) * R[(y - Y0) * NC + jc];
            }
            part[ic * NC + jc] = sum;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Resident waves walk the (image, row block, strip, scale) items; each XCD owns a
// contiguous item range (its L2 streams a contiguous slice of the images).
template <int NS, bool SSIM_ON, bool MASK>
__global__ __launch_bounds__(kBlock, MD2_BWD_MINB) void photo_bwd_kernel(PhotoArgs a) {
    __shared__ float ddacc[kWavesPerBlock][kRowsB][kWave];   // dL/d(upsampled disp) summed over frames
    __shared__ float dep[kWavesPerBlock][kRowsB + 4][kWave]; // depth of the item's window rows
    const int lane = threadIdx.x & (kWave - 1);
    // G groups of blocks (the 8 XCDs under round-robin dispatch; fewer for tiny grids)
    const int nb = gridDim.x, G = nb < 8 ? nb : 8, grp = blockIdx.x % G;
    const int blks_here = nb / G + (grp < nb % G ? 1 : 0);
    const int waves_here = blks_here * kWavesPerBlock;
    const int wid = __builtin_amdgcn_readfirstlane((int)(blockIdx.x / G) * kWavesPerBlock + (threadIdx.x >> 6));
    const int items = a.B * a.wpi * a.nsc;
    const int i_begin = (int)((long long)items * grp / G), i_end = (int)((long long)items * (grp + 1) / G);
    for (int it = i_begin + wid; it < i_end; it += waves_here) {
        // item order: b, row block, strip, scale
        int t = it;
        const int ls = t % a.nsc;
        t /= a.nsc;
        const int st = t % a.strips;
        t /= a.strips;
        const int rb = t % a.rowblocks;
        const int b = t / a.rowblocks;
        bwd_item<NS, SSIM_ON, MASK>(a, b, ls, st, rb, lane, ddacc[threadIdx.x >> 6], dep[threadIdx.x >> 6]);
    }
}

// ----------------------------------------------------------------------------
// forward finalize: fixed-order reduction of all partials -> losses + stats
// ----------------------------------------------------------------------------
struct FinalArgs {
    int B, num_scales;
    int lh[MD2_MAX_SCALES], lw[MD2_MAX_SCALES];          // loss resolution per scale
    int hs[MD2_MAX_SCALES], ws[MD2_MAX_SCALES], chunks[MD2_MAX_SCALES];
    int nphoto[MD2_MAX_SCALES];                           // partial count per scale
    const float* photo_part[MD2_MAX_SCALES];
    const float* smooth_part[MD2_MAX_SCALES];
    float* stats;                                         // [scale][B][4]
    float smoothness;
    float* loss_out;
};

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}

// Fixed-order block sum of N doubles per thread: per-wave butterflies, then wave 0
// adds the 4 wave totals in order.  Result valid in every thread.
template <int N>
__device__ __forceinline__ void block_sum_d(double (&v)[N]) {
    __shared__ double red[N][kWavesPerBlock];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int j = 0; j < N; ++j) {
        v[j] = wave_sum_d(v[j]);
        if (lane == 0) red[j][wid] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < N; ++j) v[j] = ((red[j][0] + red[j][1]) + red[j][2]) + red[j][3];
    __syncthreads();
}

// One block of 16 waves, every assignment fixed (deterministic):
//   photometric partials: wave w sums quarter w%4 of scale w/4's partials (four
//   independent accumulators per lane, so the loads of a lane are in flight together);
//   smoothness: 16-lane group g sums the chunk partials of (scale, image) pairs g,
//   g+64, ... (see below);
// then thread 0 combines everything in a fixed order.  (The first version used one
// wave per scale and one thread per image: ~100 dependent load+add steps, 46 us.)
constexpr int kFinWaves = 16;
__global__ __launch_bounds__(kWave * kFinWaves) void finalize_fwd_kernel(FinalArgs a) {
    __shared__ double photo[MD2_MAX_SCALES][4];
    __shared__ double smooth[MD2_MAX_SCALES][kBlock];   // [scale][image], B <= kBlock
    const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
    {
        const int sc = wid >> 2, q = wid & 3;
        if (sc < a.num_scales) {
            const int n = a.nphoto[sc];
            const float* p = a.photo_part[sc];
            double acc[4] = {0.0, 0.0, 0.0, 0.0};
            // batches of 8 unconditional loads (clamped index, masked add): a load under
            // a bound check is a branch the wave waits at, one memory latency per load
            for (int i0 = q * kWave + lane; i0 < n; i0 += 8 * 4 * kWave) {
                float v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int i = i0 + u * 4 * kWave;
                    v[u] = p[i < n ? i : 0];
                }
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (i0 + u * 4 * kWave < n) acc[u & 3] += (double)v[u];
            }
            double v = wave_sum_d((acc[0] + acc[1]) + (acc[2] + acc[3]));
            if (lane == 0) photo[sc][q] = v;
        }
    }
    // smoothness: 16 lanes per (scale, image) pair, every pair at once (48 pairs of 64
    // groups at B = 12); each lane sums chunks gl, gl + 16, ... from batches of 8
    // unconditional loads, then a 4-step xor butterfly inside the group.  (One wave per
    // pair, three pairs in a row per wave, took 6.7 of the kernel's 10.9 us.)
    const int NP = a.num_scales * a.B;
    constexpr int kGL = 16;
    const int gl = t & (kGL - 1);
    for (int pi = t / kGL; pi < NP; pi += kWave * kFinWaves / kGL) {   // uniform per 16-lane group
        const int sc = pi / a.B, b = pi - sc * a.B;
        const int hs = a.hs[sc], ws = a.ws[sc], nch = a.chunks[sc];
        const float* p = a.smooth_part[sc] + (size_t)b * nch * 3;
        double sd = 0.0, sx = 0.0, sy = 0.0;
        for (int k0 = gl; k0 < nch; k0 += 8 * kGL) {
            float v[8][3];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int k = k0 + u * kGL < nch ? k0 + u * kGL : 0;
#pragma unroll
                for (int e = 0; e < 3; ++e) v[u][e] = p[3 * k + e];
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (k0 + u * kGL < nch) {
                    sd += v[u][0];
                    sx += v[u][1];
                    sy += v[u][2];
                }
        }
#pragma unroll
        for (int o = kGL / 2; o > 0; o >>= 1) {
            sd += __shfl_xor(sd, o, kGL);
            sx += __shfl_xor(sx, o, kGL);
            sy += __shfl_xor(sy, o, kGL);
        }
        if (gl == 0) {
            const double m = sd / ((double)hs * ws) + 1e-7;
            smooth[sc][b] = sx / m / ((double)a.B * hs * (ws - 1)) + sy / m / ((double)a.B * (hs - 1) * ws);
            float* st = a.stats + ((size_t)sc * a.B + b) * 4;
            st[0] = (float)m;
            st[1] = (float)sx;
            st[2] = (float)sy;
            st[3] = 0.f;
        }
    }
    __syncthreads();
    if (t == 0) {
        double total = 0.0;
        for (int sc = 0; sc < a.num_scales; ++sc) {
            double sm = 0.0;
            for (int b = 0; b < a.B; ++b) sm += smooth[sc][b];
            const double ph = (photo[sc][0] + photo[sc][1]) + (photo[sc][2] + photo[sc][3]);
            const double loss = ph / ((double)a.B * a.lh[sc] * a.lw[sc]) + (double)a.smoothness * sm / (double)(1 << sc);
            a.loss_out[sc] = (float)loss;
            total += loss;
        }
        a.loss_out[a.num_scales] = (float)(total / a.num_scales);
    }
}

// ----------------------------------------------------------------------------
// dL/ddisp_s: adjoint of the bilinear upsample (gather form) + smoothness grad
// ----------------------------------------------------------------------------
struct DispGradArgs {
    int B, num_scales;
    int hs[MD2_MAX_SCALES], ws[MD2_MAX_SCALES];   // native resolution of each scale
    int lh[MD2_MAX_SCALES], lw[MD2_MAX_SCALES];   // loss resolution (= (hs<<upsh, ws<<upsh))
    int upsh[MD2_MAX_SCALES];
    int strips[MD2_MAX_SCALES], rowblocks[MD2_MAX_SCALES];   // backward item grid per image
    int block_base[MD2_MAX_SCALES + 1];           // first block of each scale (one launch)
    int bpr[MD2_MAX_SCALES];                      // blocks per native row
    const float* dfull[MD2_MAX_SCALES];           // upsh == 0: (B, lh, lw) dL/d(disp)
    const float* upart[MD2_MAX_SCALES];           // upsh > 0: per-item partial grids (bwd_item)
    const float* sgrad[MD2_MAX_SCALES];           // (B, hs, ws) per-unit smoothness gradient (smooth_fwd)
    const float* stats;                           // [scale][B][4]
    const float* grad_loss;
    float smoothness;
    float* out[MD2_MAX_SCALES];                   // (B, 1, hs, ws), fp32 or bf16 as disp
    int disp_bf16;
    int quad;                                     // every ws % 4 == 0: disp_grad_quad
};

// dL/d(disp) of native pixel (i, j) from the photometric term: the sum of the <= 2 x 2
// backward items' partials that reach it (row blocks, then strips, ascending: fixed
// order), or the full-resolution plane's value at scale 0 / v1
__device__ __forceinline__ float disp_photo_acc(const DispGradArgs& a, int s, int b, int i, int j) {
    const int sh = a.upsh[s];
    const int hs = a.hs[s], ws = a.ws[s], lh = a.lh[s], lw = a.lw[s];
    if (sh == 0) return a.dfull[s][(size_t)b * lh * lw + i * lw + j];
    const int kf = 1 << sh, half = kf >> 1;
    const float sc = 1.0f / (float)kf;
    const int NC = up_nc(sh), NR = up_nr(sh);
    const int strips = a.strips[s], rowblocks = a.rowblocks[s];
    // the full-resolution footprint of (i, j) (a superset of the weight-carrying rows /
    // columns) and the items holding it
    const int yf0 = max(0, kf * (i - 1) + half), yf1 = min(lh, kf * (i + 1) + half);
    const int xf0 = max(0, kf * (j - 1) + half), xf1 = min(lw, kf * (j + 1) + half);
    const int rb0 = yf0 / kRowsB, rb1 = (yf1 - 1) / kRowsB;
    const int st0 = xf0 / kBwdCols, st1 = (xf1 - 1) / kBwdCols;
    const float* base = a.upart[s] + (size_t)b * rowblocks * strips * NR * NC;
    // the footprint spans <= 2 row blocks and <= 2 strips (2^(s+1) <= kRowsB, kBwdCols):
    // four candidate partials, all loaded unconditionally (an invalid one reads the
    // image's first partial and adds nothing), summed rows then strips ascending
    static_assert(kRowsB >= (2 << (MD2_MAX_SCALES - 1)) && kBwdCols >= (2 << (MD2_MAX_SCALES - 1)),
                  "a native pixel's footprint spans at most two backward items per axis");
    int idx[4];
    bool ok[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int r = (u >> 1) ? rb1 : rb0, t = (u & 1) ? st1 : st0;
        const int ic = i - up_src0(r * kRowsB, hs, sc), jc = j - up_src0(t * kBwdCols, ws, sc);
        ok[u] = ic >= 0 && ic < NR && jc >= 0 && jc < NC && (!(u >> 1) || rb1 != rb0) && (!(u & 1) || st1 != st0);
        idx[u] = ok[u] ? (r * strips + t) * NR * NC + ic * NC + jc : 0;
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = ldf(base, idx[u]);
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (ok[u]) acc += v[u];
    return acc;
}

// smoothness gradient on disp / (mean + 1e-7): the forward's per-unit stencil gradient
// scaled by dL/dloss_s, the weight / 2^s, 1/B and 1/mean, plus the term through the
// mean (trainer.py:486-490).  sg(x) = k1 * x - k0.
struct SmoothScale {
    float k1, k0;
};
__device__ __forceinline__ SmoothScale smooth_scale(const DispGradArgs& a, int s, int b) {
    const int hs = a.hs[s], ws = a.ws[s];
    const float gl = a.grad_loss[s] + a.grad_loss[a.num_scales] / (float)a.num_scales;
    const float* st = a.stats + ((size_t)s * a.B + b) * 4;
    const float m = st[0];
    const float wsm = gl * a.smoothness / (float)(1 << s);
    const float ax = wsm / ((float)a.B * hs * (ws - 1)) / m;
    const float ay = wsm / ((float)a.B * (hs - 1) * ws) / m;
    return {wsm / ((float)a.B * m), (ax * st[1] + ay * st[2]) / (m * (float)(hs * ws))};
}

// One thread per native pixel; blocks own whole native rows: block_base[s] +
// (b·hs + i)·bpr[s] + chunk (the (scale, image, row) decode is uniform per block).
__device__ __forceinline__ void disp_grad_px(const DispGradArgs& a, int bid) {
    int s = 0;
    while (s + 1 < a.num_scales && bid >= a.block_base[s + 1]) ++s;
    const int hs = a.hs[s], ws = a.ws[s], HWs = hs * ws;
    const int rb = bid - a.block_base[s], bpr = a.bpr[s];
    const int row = rb / bpr, chunk = rb - row * bpr;
    const int b = row / hs, i = row - b * hs;
    const int j = chunk * kBlock + threadIdx.x;
    if (j >= ws) return;
    const int p = i * ws + j;
    const float acc = disp_photo_acc(a, s, b, i, j);
    const SmoothScale k = smooth_scale(a, s, b);
    float sg = k.k1 * a.sgrad[s][(size_t)b * HWs + p];
    sg -= k.k0;
    // the gradient in the disparity's own dtype (bf16: round to nearest even, as the
    // cast-up's autograd backward would)
    if (a.disp_bf16) ((uint16_t*)a.out[s])[(size_t)b * HWs + p] = (uint16_t)md2::f2bf(acc + sg);
    else a.out[s][(size_t)b * HWs + p] = acc + sg;
}

// Every ws % 4 == 0 (a.quad): one thread per pixel quad of a row, blocks over the flat
// quads of each scale (block_base in blocks of kBlock quads): float4 reads of the
// smoothness plane (and the scale-0 plane), one 16-byte (bf16: 8-byte) store.
__device__ __forceinline__ void disp_grad_quad(const DispGradArgs& a, int bid) {
    int s = 0;
    while (s + 1 < a.num_scales && bid >= a.block_base[s + 1]) ++s;
    const int hs = a.hs[s], ws = a.ws[s], HWs = hs * ws, Q = HWs >> 2;
    const int q = (bid - a.block_base[s]) * kBlock + threadIdx.x;
    if (q >= a.B * Q) return;
    const int b = q / Q, p = (q - b * Q) << 2;
    const int i = p / ws, j0 = p - i * ws;
    float acc[4];
    if (a.upsh[s] == 0) {
        const float4 v = *(const float4*)(a.dfull[s] + (size_t)b * HWs + p);   // lh, lw == hs, ws
        acc[0] = v.x, acc[1] = v.y, acc[2] = v.z, acc[3] = v.w;
    } else {
#pragma unroll
        for (int m = 0; m < 4; ++m) acc[m] = disp_photo_acc(a, s, b, i, j0 + m);
    }
    const SmoothScale k = smooth_scale(a, s, b);
    const float4 g = *(const float4*)(a.sgrad[s] + (size_t)b * HWs + p);
    float o[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        float sg = k.k1 * f4at(g, m);
        sg -= k.k0;
        o[m] = acc[m] + sg;
    }
    const size_t e = (size_t)b * HWs + p;
    if (a.disp_bf16) {
        const uint32_t lo = md2::f2bf(o[0]) | ((uint32_t)md2::f2bf(o[1]) << 16);
        const uint32_t hi = md2::f2bf(o[2]) | ((uint32_t)md2::f2bf(o[3]) << 16);
        *(uint2*)((uint16_t*)a.out[s] + e) = make_uint2(lo, hi);
    } else {
        *(float4*)(a.out[s] + e) = make_float4(o[0], o[1], o[2], o[3]);
    }
}

// ----------------------------------------------------------------------------
// dL/dT: fixed-order reduction of per-wave dL/dP partials, dT = K^T [dP; 0]
// ----------------------------------------------------------------------------
struct DTArgs {
    int B, S, num_scales, per_scale;
    int wpi[MD2_MAX_SCALES];
    const float* dP_part[MD2_MAX_SCALES];   // [S][B*wpi][12]
    const float* K[MD2_MAX_SCALES];         // K at each scale's loss resolution
    float* grad_T;                          // (S,B,4,4) or (num_scales,S,B,4,4)
};

__device__ __forceinline__ void grad_T_block(const DTArgs& a, int id) {
    // one block per (tscale, f, b); every thread accumulates all 12 dP entries over
    // a strided share of the partials, then one fixed-order block reduction
    const int b = id % a.B;
    id /= a.B;
    const int f = id % a.S;
    const int ts = id / a.S;
    const int t = threadIdx.x;
    double dT[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) dT[j] = 0.0;
    // dT = sum_s K_s^T [dP_s; 0] is linear in the partials: every thread maps its own
    // partials through K_s^T and sums over the scales, then ONE fixed-order block
    // reduction of the 16 entries (instead of one 12-entry reduction per scale)
    // first every scale's partial k = t, its 12 loads per scale issued together (a
    // loop that waits for each scale's loads before the next pays ~4 memory latencies)
    // (unconditional loads from clamped addresses; unused ones are masked afterwards)
    float first[MD2_MAX_SCALES][12], Ks[MD2_MAX_SCALES][12];
    bool use[MD2_MAX_SCALES];
#pragma unroll
    for (int s = 0; s < MD2_MAX_SCALES; ++s) {
        const int sc = s < a.num_scales ? s : 0;
        const int n = a.wpi[sc];
        use[s] = s < a.num_scales && !(a.per_scale && s != ts) && t < n;
        const float* base = a.dP_part[sc] + ((size_t)f * a.B * n + (size_t)b * n + (use[s] ? t : 0)) * 12;
        const float* K = a.K[sc] + b * 16;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            first[s][j] = base[j];
            Ks[s][j] = K[j];
        }
    }
#pragma unroll
    for (int s = 0; s < MD2_MAX_SCALES; ++s) {
        if (!use[s]) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                dT[r * 4 + c] += (double)Ks[s][0 * 4 + r] * (double)first[s][0 * 4 + c] +
                                 (double)Ks[s][1 * 4 + r] * (double)first[s][1 * 4 + c] +
                                 (double)Ks[s][2 * 4 + r] * (double)first[s][2 * 4 + c];
    }
    for (int s = 0; s < a.num_scales; ++s) {   // the rest (more than kBlock partials per image)
        if (a.per_scale && s != ts) continue;
        const int n = a.wpi[s];
        const float* base = a.dP_part[s] + ((size_t)f * a.B * n + (size_t)b * n) * 12;
        const float* K = a.K[s] + b * 16;
        for (int k = t + kBlock; k < n; k += kBlock) {
            double dP[12];
#pragma unroll
            for (int j = 0; j < 12; ++j) dP[j] = (double)base[(size_t)k * 12 + j];
#pragma unroll
            for (int r = 0; r < 4; ++r)
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    dT[r * 4 + c] += (double)K[0 * 4 + r] * dP[0 * 4 + c] + (double)K[1 * 4 + r] * dP[1 * 4 + c] +
                                     (double)K[2 * 4 + r] * dP[2 * 4 + c];
        }
    }
    block_sum_d<16>(dT);
    if (t < 16) {
        double v = 0.0;
#pragma unroll
        for (int j = 0; j < 16; ++j) v = (j == t) ? dT[j] : v;
        a.grad_T[(((size_t)ts * a.S + f) * a.B + b) * 16 + t] = (float)v;
    }
}

// The backward's tail in one launch: blocks [0, nTb) reduce dL/dT (nT·S·B of them
// work, the rest of the 8-aligned prefix returns), the others write dL/d(disp) —
// the 24 long fp64 reduction blocks run beside the short per-pixel ones instead of
// after them.  nTb % 8 == 0 keeps disp_grad's XCD-contiguous block numbering.
__global__ __launch_bounds__(kBlock) void disp_grad_T_kernel(DispGradArgs g, DTArgs ta, int nT, int nTb) {
    const int bx = blockIdx.x;
    if (bx < nTb) {
        if (bx < nT) grad_T_block(ta, bx);
        return;
    }
    // a block's pixels share partial grids with the neighbouring rows: consecutive
    // blocks on one XCD, so its L2 serves those re-reads
    const int bid = xcd_contiguous_block(bx - nTb, gridDim.x - nTb);
    if (g.quad) disp_grad_quad(g, bid);
    else disp_grad_px(g, bid);
}

// ----------------------------------------------------------------------------
// materialisation of generate_images_pred's outputs (logging / eval steps)
// ----------------------------------------------------------------------------
struct GenArgs {
    PhotoArgs p;
    int ls;
    float* depth;    // (B,1,h,w) or null
    float* sample[MD2_MAX_SRC];
    float* color[MD2_MAX_SRC];
};

__global__ __launch_bounds__(kBlock) void generate_kernel(GenArgs g) {
    const PhotoArgs& a = g.p;
    const int HW = a.h * a.w;
    const int idx = blockIdx.x * kBlock + threadIdx.x;
    if (idx >= a.B * HW) return;
    const int b = idx / HW, p = idx - b * HW;
    const int y = p / a.w, x = p - y * a.w;
    for (int f = 0; f < a.S; ++f) {
        WarpCtx ctx;
        make_ctx(a, g.ls, f, b, ctx);
        Sample s;
        project(ctx, y, x, s);
        if (f == 0 && g.depth) g.depth[idx] = s.depth;
        if (g.sample[f]) {
            const float px = s.cam[0] / s.den, py = s.cam[1] / s.den;
            g.sample[f][(size_t)idx * 2 + 0] = (px / (float)(a.w - 1) - 0.5f) * 2.f;
            g.sample[f][(size_t)idx * 2 + 1] = (py / (float)(a.h - 1) - 0.5f) * 2.f;
        }
        if (g.color[f]) {
            Corners v;
            gather<false>(ctx, s, v);
            float o[3];
            interp<false>(s, v, o);
            for (int ch = 0; ch < 3; ++ch) g.color[f][((size_t)b * 3 + ch) * HW + p] = o[ch];
        }
    }
}

// ----------------------------------------------------------------------------
// host side
// ----------------------------------------------------------------------------
thread_local char g_err[512] = "";

// md2_tiebreak_noise: the combine kernel's in-kernel draw, one thread per pixel
struct NoiseArgs {
    int B, HW, C, gsc;
    uint64_t seed;
    const uint64_t* seed_ptr;
    float* out;
};

__global__ __launch_bounds__(kBlock) void tiebreak_noise_kernel(NoiseArgs a) {
    const int idx = blockIdx.x * kBlock + threadIdx.x;
    if (idx >= a.B * a.HW) return;
    const int b = idx / a.HW, p = idx - b * a.HW;
    const uint64_t seed = a.seed_ptr ? (a.seed ^ (*a.seed_ptr * 0x9E3779B97F4A7C15ULL)) : a.seed;
    const uint32_t key = noise_key(seed, a.gsc);
    for (int j = 0; 2 * j < a.C; ++j) {
        const float2 n2 = noise_pair(key, (uint32_t)idx, j);
        a.out[((size_t)b * a.C + 2 * j) * a.HW + p] = n2.x;
        if (2 * j + 1 < a.C) a.out[((size_t)b * a.C + 2 * j + 1) * a.HW + p] = n2.y;
    }
}

// optional benchmark timing of the photometric kernels (md2_timing_begin/end)
struct Timing {
    std::mutex mu;
    bool on = false;
    int cap = 0, used = 0;
    std::vector<hipEvent_t> ev;     // pairs: [2*i] start, [2*i+1] stop (owned)
    std::vector<hipEvent_t> start;  // the start event slot i measures from (ev[2*i] or another slot's)
    std::vector<int> kind;          // 0 fwd photo kernels, 1 photo_bwd, 2 whole fwd call, 3 whole bwd call
    double call_ms[2] = {0.0, 0.0}; // kinds 2, 3 of the last md2_timing_end
    int call_n[2] = {0, 0};
};
Timing g_timing;

// Reserve a timing slot (or -1).  The events are stamped by hipExtLaunchKernelGGL on
// the kernel dispatch itself, so they measure the kernel, not the queue around it.
// shared_start: measure from that (already reserved) start event instead of the slot's own.
int timing_slot(int kind, hipEvent_t* start, hipEvent_t* stop, hipEvent_t shared_start = nullptr) {
    std::lock_guard<std::mutex> lk(g_timing.mu);
    *start = *stop = nullptr;
    if (!g_timing.on || g_timing.used >= g_timing.cap) return -1;
    const int i = g_timing.used++;
    g_timing.kind[i] = kind;
    g_timing.start[i] = shared_start ? shared_start : g_timing.ev[2 * i];
    *start = g_timing.start[i];
    *stop = g_timing.ev[2 * i + 1];
    return i;
}

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

struct Layout {
    int nscales, S, B;
    bool v1;
    int lh[MD2_MAX_SCALES], lw[MD2_MAX_SCALES];      // loss resolution
    int hs[MD2_MAX_SCALES], ws[MD2_MAX_SCALES];      // native resolution
    int fstrips[MD2_MAX_SCALES], frows[MD2_MAX_SCALES], fwpi[MD2_MAX_SCALES];
    int bstrips[MD2_MAX_SCALES], brows[MD2_MAX_SCALES], bwpi[MD2_MAX_SCALES];
    int chunks[MD2_MAX_SCALES];
    size_t ident_off, src8_off, exact_off;
    size_t photo_off[MD2_MAX_SCALES], dP_off[MD2_MAX_SCALES], smooth_off[MD2_MAX_SCALES];
    size_t sgrad_off[MD2_MAX_SCALES];
    size_t dfull_off[MD2_MAX_SCALES], stats_off, total;
    size_t sel_off[MD2_MAX_SCALES], sel_total;
    size_t noise_off[MD2_MAX_SCALES];
    size_t mask_off[MD2_MAX_SCALES];
};

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

int make_layout(const md2_desc* d, Layout& L) {
    if (!d) return fail(MD2_ERR_ARG, "desc is NULL");
    if (d->batch < 1) return fail(MD2_ERR_ARG, "batch must be >= 1 (got %d)", d->batch);
    if (d->num_src < 1 || d->num_src > MD2_MAX_SRC)
        return fail(MD2_ERR_ARG, "num_src must be 1..%d (got %d)", MD2_MAX_SRC, d->num_src);
    if (d->num_scales < 1 || d->num_scales > MD2_MAX_SCALES)
        return fail(MD2_ERR_ARG, "num_scales must be 1..%d (got %d)", MD2_MAX_SCALES, d->num_scales);
    const int div = 1 << (d->num_scales - 1);
    if (d->height % div || d->width % div)
        return fail(MD2_ERR_ARG, "height/width (%d,%d) must be divisible by 2^(num_scales-1)=%d", d->height,
                    d->width, div);
    if ((d->height >> (d->num_scales - 1)) < 4 || (d->width >> (d->num_scales - 1)) < 4)
        return fail(MD2_ERR_ARG, "coarsest scale must be at least 4x4");
    if (!(d->min_depth > 0.f) || !(d->max_depth > d->min_depth))
        return fail(MD2_ERR_ARG, "need 0 < min_depth < max_depth");
    if (d->disp_dtype != MD2_DTYPE_F32 && d->disp_dtype != MD2_DTYPE_BF16)
        return fail(MD2_ERR_ARG, "disp_dtype must be MD2_DTYPE_F32 or MD2_DTYPE_BF16 (got %u)", d->disp_dtype);
    L.nscales = d->num_scales;
    L.S = d->num_src;
    L.B = d->batch;
    L.v1 = (d->flags & MD2_V1_MULTISCALE) != 0;
    size_t off = 0, soff = 0, noff = 0, moff = 0;
    const int C = (d->flags & MD2_AVG_REPROJECTION) ? 1 : d->num_src;
    for (int s = 0; s < L.nscales; ++s) {
        L.hs[s] = d->height >> s;
        L.ws[s] = d->width >> s;
        L.lh[s] = L.v1 ? L.hs[s] : d->height;
        L.lw[s] = L.v1 ? L.ws[s] : d->width;
        L.fstrips[s] = (L.lw[s] + kFwdCols - 1) / kFwdCols;
        L.frows[s] = (L.lh[s] + kRowsP - 1) / kRowsP;
        L.fwpi[s] = L.fstrips[s] * L.frows[s];
        L.bstrips[s] = (L.lw[s] + kBwdCols - 1) / kBwdCols;
        L.brows[s] = (L.lh[s] + kRowsB - 1) / kRowsB;
        L.bwpi[s] = L.bstrips[s] * L.brows[s];
        L.chunks[s] = (L.hs[s] * L.ws[s] + kSmoothChunk - 1) / kSmoothChunk;
        L.photo_off[s] = off;
        off = align256(off + sizeof(float) * (size_t)L.B * L.fwpi[s]);   // one partial per forward wave
        L.dP_off[s] = off;
        off = align256(off + sizeof(float) * (size_t)L.S * L.B * L.bwpi[s] * 12);
        L.smooth_off[s] = off;
        off = align256(off + sizeof(float) * (size_t)L.B * L.chunks[s] * 3);
        L.sgrad_off[s] = off;   // the smoothness gradient plane, forward -> backward
        off = align256(off + sizeof(float) * (size_t)L.B * L.hs[s] * L.ws[s]);
        L.dfull_off[s] = off;   // upsampled scales: the backward items' partial grids instead
        const int upsh = L.v1 ? 0 : s;
        off = align256(off + sizeof(float) * (upsh == 0 ? (size_t)L.B * L.lh[s] * L.lw[s]
                                                         : (size_t)L.B * L.bwpi[s] * up_nr(upsh) * up_nc(upsh)));
        L.sel_off[s] = soff;
        soff += (size_t)L.B * L.lh[s] * L.lw[s];
        L.noise_off[s] = noff;
        noff += (size_t)L.B * C * L.lh[s] * L.lw[s];
        L.mask_off[s] = moff;
        moff += (size_t)L.B * L.S * L.lh[s] * L.lw[s];
    }
    L.ident_off = off;   // identity losses of one scale group (the largest: scale 0)
    off = align256(off + sizeof(float) * (size_t)L.S * L.B * L.lh[0] * L.lw[0]);
    L.src8_off = off;    // 8-bit source copies (full resolution; not with V1_MULTISCALE)
    off = align256(off + (L.v1 ? 0 : sizeof(uint32_t) * (size_t)L.S * L.B * L.lh[0] * L.lw[0]));
    L.exact_off = off;
    off = align256(off + sizeof(int) * (size_t)L.S * L.B);
    L.stats_off = off;
    off = align256(off + sizeof(float) * (size_t)L.nscales * L.B * 4);
    L.total = off;
    L.sel_total = soff;
    return MD2_OK;
}

int check_tensors(const md2_desc* d, const md2_tensors* t, const Layout& L, bool need_mask = true) {
    if (!t) return fail(MD2_ERR_ARG, "tensors is NULL");
    if (need_mask && (d->flags & MD2_PREDICTIVE_MASK)) {
        if (!(d->flags & MD2_NO_AUTOMASK))
            return fail(MD2_ERR_ARG, "MD2_PREDICTIVE_MASK requires MD2_NO_AUTOMASK (trainer.py:91-92)");
        if (!t->mask) return fail(MD2_ERR_ARG, "MD2_PREDICTIVE_MASK set but mask is NULL");
    }
    if (!t->T) return fail(MD2_ERR_ARG, "T is NULL");
    for (int s = 0; s < L.nscales; ++s) {
        if (!t->disp[s]) return fail(MD2_ERR_ARG, "disp[%d] is NULL", s);
        if (!t->color[s][0]) return fail(MD2_ERR_ARG, "color[%d][0] (target) is NULL", s);
        const int cs = L.v1 ? s : 0;
        for (int f = 1; f <= L.S; ++f)
            if (!t->color[cs][f]) return fail(MD2_ERR_ARG, "color[%d][%d] is NULL", cs, f);
        if (!t->K[cs] || !t->inv_K[cs]) return fail(MD2_ERR_ARG, "K/inv_K[%d] is NULL", cs);
    }
    (void)d;
    return MD2_OK;
}

int hip_check(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return fail(MD2_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
    return MD2_OK;
}

// fill the PhotoArgs for the scale set [s_begin, s_end)
void photo_args(const md2_desc* d, const md2_tensors* t, const Layout& L, int s_begin, int s_end, bool bwd,
                uint8_t* ws, uint8_t* sel, PhotoArgs& a, float* grad_mask = nullptr) {
    memset(&a, 0, sizeof(a));
    const int cs = L.v1 ? s_begin : 0;
    a.B = L.B;
    a.h = L.lh[s_begin];
    a.w = L.lw[s_begin];
    a.S = L.S;
    a.nsc = s_end - s_begin;
    a.strips = bwd ? L.bstrips[s_begin] : L.fstrips[s_begin];
    a.rowblocks = bwd ? L.brows[s_begin] : L.frows[s_begin];
    a.wpi = a.strips * a.rowblocks;
    a.num_scales = L.nscales;
    a.tgt = t->color[cs][0];
    for (int f = 0; f < L.S; ++f) a.src[f] = t->color[cs][f + 1];
    a.K = t->K[cs];
    a.iK = t->inv_K[cs];
    a.seed = d->seed;
    a.seed_ptr = t->seed_ptr;
    a.disp_bf16 = d->disp_dtype == MD2_DTYPE_BF16;
    a.min_disp = 1.0f / d->max_depth;
    a.range = 1.0f / d->min_depth - 1.0f / d->max_depth;
    a.flags = d->flags;
    const size_t Tstride = (size_t)L.S * L.B * 16;
    for (int s = s_begin; s < s_end; ++s) {
        const int ls = s - s_begin;
        a.gscale[ls] = s;
        a.disp[ls] = t->disp[s];
        a.dh[ls] = L.hs[s];
        a.dw[ls] = L.ws[s];
        a.upsh[ls] = L.v1 ? 0 : s;
        a.T[ls] = t->T + ((d->flags & MD2_T_PER_SCALE) ? s * Tstride : 0);
        a.noise[ls] = t->noise ? t->noise + L.noise_off[s] : nullptr;
        a.photo_part[ls] = (float*)(ws + L.photo_off[s]);
        a.sel[ls] = sel ? sel + L.sel_off[s] : nullptr;
        a.dfull[ls] = (float*)(ws + L.dfull_off[s]);
        a.upart[ls] = (float*)(ws + L.dfull_off[s]);
        a.dP_part[ls] = (float*)(ws + L.dP_off[s]);
        a.mask[ls] = t->mask ? t->mask + L.mask_off[s] : nullptr;
        a.gmask[ls] = grad_mask ? grad_mask + L.mask_off[s] : nullptr;
    }
    a.ident = ws ? (float*)(ws + L.ident_off) : nullptr;
    if (ws && !L.v1) {
        // the caller's 8-bit copies (exact by contract: no flags) or the forward's pack
        const uint32_t* s8 = t->src8 ? t->src8 : (const uint32_t*)(ws + L.src8_off);
        for (int f = 0; f < L.S; ++f) a.src8[f] = s8 + (size_t)f * L.B * L.lh[0] * L.lw[0];
        a.exact = t->src8 ? nullptr : (const int*)(ws + L.exact_off);
    }
}

template <int NS, bool SSIM, bool MASK>
void launch_fwd_t(const PhotoArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    // the timing events bracket the three launches (start on the first, stop on the last)
    const bool ident_kernel = !(a.flags & MD2_NO_AUTOMASK) && !a.ident_fused;
    if (ident_kernel) {
        const int blocks = (a.B * a.wpi * NS + kWavesPerBlock - 1) / kWavesPerBlock;
        hipExtLaunchKernelGGL((photo_ident_kernel<NS, SSIM>), dim3(blocks), dim3(kBlock), 0, st, e0, nullptr, 0, a);
    }
    const int rblocks = (a.B * a.wpi * a.nsc + kWavesPerBlock - 1) / kWavesPerBlock;
    // with the smoothness blocks behind the walk's (a.fwd_blocks = rblocks rounded up to 8)
    const int grid = a.smooth_blocks ? a.fwd_blocks + a.smooth_blocks : rblocks;
    hipExtLaunchKernelGGL((photo_fwdall_kernel<NS, SSIM, MASK>), dim3(grid), dim3(kBlock), 0, st,
                          ident_kernel ? nullptr : e0, e1, 0, a);
}
// number of workgroups that can be resident at once for a kernel (cached per
// kernel and device); the persistent-loop kernels launch exactly that many
// (keyed by the kernel's address: every instantiation has the same function type, so a
// per-template static would hand one instantiation's occupancy to all of them)
template <class K>
int resident_blocks(K kernel) {
    static std::mutex mu;
    static std::map<std::pair<const void*, int>, int> cache;
    int dev = 0;
    (void)hipGetDevice(&dev);
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair((const void*)kernel, dev);
    const auto it = cache.find(key);
    if (it != cache.end()) return it->second;
    int cus = 0, per_cu = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, kBlock, 0);
    return cache[key] = max(1, cus) * max(1, per_cu);
}

template <int NS, bool SSIM, bool MASK>
void launch_bwd_t(const PhotoArgs& a, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    const int items = a.B * a.wpi * a.nsc;
    const int need = (items + kWavesPerBlock - 1) / kWavesPerBlock;
    const int blocks = min(need, resident_blocks(photo_bwd_kernel<NS, SSIM, MASK>));
    if (e0)
        hipExtLaunchKernelGGL((photo_bwd_kernel<NS, SSIM, MASK>), dim3(blocks), dim3(kBlock), 0, st, e0, e1, 0, a);
    else
        hipLaunchKernelGGL((photo_bwd_kernel<NS, SSIM, MASK>), dim3(blocks), dim3(kBlock), 0, st, a);
}

template <int NS, bool SSIM, bool MASK>
void launch_one(const PhotoArgs& a, bool bwd, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    if (bwd) launch_bwd_t<NS, SSIM, MASK>(a, st, e0, e1);
    else launch_fwd_t<NS, SSIM, MASK>(a, st, e0, e1);
}

template <int NS>
void launch_ns(const PhotoArgs& a, bool bwd, hipStream_t st, hipEvent_t e0, hipEvent_t e1) {
    const bool ssim = !(a.flags & MD2_NO_SSIM), mask = (a.flags & MD2_PREDICTIVE_MASK) != 0;
    if (ssim) {
        if (mask) launch_one<NS, true, true>(a, bwd, st, e0, e1);
        else launch_one<NS, true, false>(a, bwd, st, e0, e1);
    } else {
        if (mask) launch_one<NS, false, true>(a, bwd, st, e0, e1);
        else launch_one<NS, false, false>(a, bwd, st, e0, e1);
    }
}

void launch_photo(const PhotoArgs& a, bool bwd, hipStream_t st, hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr) {
    if (a.S == 1) launch_ns<1>(a, bwd, st, e0, e1);
    else if (a.S == 2) launch_ns<2>(a, bwd, st, e0, e1);
    else launch_ns<3>(a, bwd, st, e0, e1);
}

}  // namespace

// md2_last_error() for the library's other translation units (not exported).
__attribute__((visibility("hidden"))) int md2_report_error(int code, const char* msg) {
    return fail(code, "%s", msg);
}

// ============================================================================
// C ABI
// ============================================================================
extern "C" {

int md2_abi_version(void) { return MD2_ABI_VERSION; }

const char* md2_last_error(void) { return g_err; }

size_t md2_workspace_bytes(const md2_desc* desc) {
    Layout L;
    if (make_layout(desc, L) != MD2_OK) return 0;
    return L.total;
}

size_t md2_select_bytes(const md2_desc* desc) {
    Layout L;
    if (make_layout(desc, L) != MD2_OK) return 0;
    return L.sel_total;
}

int md2_photometric_fwd(const md2_desc* d, const md2_tensors* t, float* loss_out, uint8_t* select_out,
                        void* workspace, void* stream) {
    Layout L;
    int rc = make_layout(d, L);
    if (rc) return rc;
    if ((rc = check_tensors(d, t, L))) return rc;
    if (!loss_out || !select_out || !workspace) return fail(MD2_ERR_ARG, "loss_out/select_out/workspace is NULL");
    hipStream_t st = (hipStream_t)stream;
    uint8_t* ws = (uint8_t*)workspace;
    SmoothArgs sa;
    memset(&sa, 0, sizeof(sa));
    sa.B = L.B;
    sa.num_scales = L.nscales;
    int blocks = 0;
    for (int s = 0; s < L.nscales; ++s) {
        sa.hs[s] = L.hs[s];
        sa.ws[s] = L.ws[s];
        sa.chunks[s] = L.chunks[s];
        sa.block_base[s] = blocks;
        blocks += L.B * L.chunks[s];
        sa.disp[s] = t->disp[s];
        sa.img[s] = t->color[s][0];
        sa.part[s] = (float*)(ws + L.smooth_off[s]);
        sa.sgrad[s] = (float*)(ws + L.sgrad_off[s]);
    }
    sa.block_base[L.nscales] = blocks;
    sa.disp_bf16 = d->disp_dtype == MD2_DTYPE_BF16;
    sa.quad = 1;
    for (int s = 0; s < L.nscales; ++s) sa.quad &= (L.ws[s] % 4 == 0) ? 1 : 0;
    // the smoothness blocks ride behind the forward walk's in its launch (their ~12 us
    // of latency-bound work fills the walk's tail instead of following it);
    // MD2_SMOOTH_MERGE=0: a separate launch after it
    static const bool merge_on = [] {
        const char* e = getenv("MD2_SMOOTH_MERGE");
        return !(e && e[0] == '0');
    }();
    const bool merged = merge_on && !L.v1;
    PhotoArgs a;
    hipEvent_t c0 = nullptr, c1 = nullptr;
    if (L.v1) {  // one launch per scale (each at its own resolution); not timed
        for (int s = 0; s < L.nscales; ++s) {
            photo_args(d, t, L, s, s + 1, false, ws, select_out, a);
            launch_photo(a, false, st);
        }
    } else {
        // 8-bit source copies for the gathers of this forward and its backward
        PackArgs pk;
        memset(&pk, 0, sizeof(pk));
        pk.B = L.B;
        pk.HW = L.lh[0] * L.lw[0];
        pk.S = L.S;
        for (int f = 0; f < L.S; ++f) pk.src[f] = t->color[0][f + 1];
        pk.out = (uint32_t*)(ws + L.src8_off);
        pk.exact = (int*)(ws + L.exact_off);
        if (!t->src8 && hipMemsetAsync(pk.exact, 0x01, sizeof(int) * (size_t)L.S * L.B, st) != hipSuccess)
            return fail(MD2_ERR_HIP, "hipMemsetAsync failed");
        const int per_img = (pk.HW + 4 * kBlock - 1) / (4 * kBlock);
        timing_slot(2, &c0, &c1);   // the whole call: pack .. finalize
        hipEvent_t e0, e1;
        timing_slot(0, &e0, &e1);
        photo_args(d, t, L, 0, L.nscales, false, ws, select_out, a);
        if (merged) {
            a.fwd_blocks = ((L.B * a.wpi * a.nsc + kWavesPerBlock - 1) / kWavesPerBlock + 7) / 8 * 8;
            a.smooth_blocks = blocks;
            a.sm = sa;
        }
        // four scales: the forward walk's blocks are (item, 4 scales) and compute the
        // identity losses themselves (no identity planes: round 4, -24 MB of traffic
        // and one launch per step); otherwise the identity pass writes them, and the
        // 8-bit copies too (it reads every source pixel anyway)
        a.ident_fused = (L.nscales == kWavesPerBlock && !(d->flags & MD2_NO_AUTOMASK)) ? 1 : 0;
        if (t->src8) {   // the caller's copies: nothing to pack
            if (c0 && hipEventRecord(c0, st) != hipSuccess) return fail(MD2_ERR_HIP, "hipEventRecord failed");
        } else if (!(d->flags & MD2_NO_AUTOMASK) && !a.ident_fused) {
            a.pack8 = pk.out;
            a.pack_exact = pk.exact;
            if (c0 && hipEventRecord(c0, st) != hipSuccess) return fail(MD2_ERR_HIP, "hipEventRecord failed");
        } else {
            hipExtLaunchKernelGGL(pack_src8_kernel, dim3(L.S * L.B * per_img), dim3(kBlock), 0, st, c0, nullptr, 0,
                                  pk);
        }
        launch_photo(a, false, st, e0, e1);
    }
    if ((rc = hip_check("photo forward kernels"))) return rc;

    if (!merged) {
        hipLaunchKernelGGL(smooth_fwd_kernel, dim3(blocks), dim3(kBlock), 0, st, sa);
        if ((rc = hip_check("smooth_fwd_kernel"))) return rc;
    }

    FinalArgs fa;
    memset(&fa, 0, sizeof(fa));
    fa.B = L.B;
    fa.num_scales = L.nscales;
    for (int s = 0; s < L.nscales; ++s) {
        fa.lh[s] = L.lh[s];
        fa.lw[s] = L.lw[s];
        fa.hs[s] = L.hs[s];
        fa.ws[s] = L.ws[s];
        fa.chunks[s] = L.chunks[s];
        fa.nphoto[s] = L.B * L.fwpi[s];
        fa.photo_part[s] = (const float*)(ws + L.photo_off[s]);
        fa.smooth_part[s] = (const float*)(ws + L.smooth_off[s]);
    }
    fa.stats = (float*)(ws + L.stats_off);
    fa.smoothness = d->disparity_smoothness;
    fa.loss_out = loss_out;
    if (L.B > kBlock) return fail(MD2_ERR_ARG, "batch > %d not supported by the finalize kernel", kBlock);
    if (c1)
        hipExtLaunchKernelGGL(finalize_fwd_kernel, dim3(1), dim3(kWave * kFinWaves), 0, st, nullptr, c1, 0, fa);
    else
        hipLaunchKernelGGL(finalize_fwd_kernel, dim3(1), dim3(kWave * kFinWaves), 0, st, fa);
    return hip_check("finalize_fwd_kernel");
}

int md2_photometric_bwd(const md2_desc* d, const md2_tensors* t, const float* grad_loss, const uint8_t* select,
                        float* const* grad_disp, float* grad_T, float* grad_mask, void* workspace, void* stream) {
    Layout L;
    int rc = make_layout(d, L);
    if (rc) return rc;
    if ((rc = check_tensors(d, t, L))) return rc;
    if (!grad_loss || !select || !grad_disp || !grad_T || !workspace)
        return fail(MD2_ERR_ARG, "grad_loss/select/grad_disp/grad_T/workspace is NULL");
    if ((d->flags & MD2_PREDICTIVE_MASK) && !grad_mask)
        return fail(MD2_ERR_ARG, "MD2_PREDICTIVE_MASK needs grad_mask");
    for (int s = 0; s < L.nscales; ++s)
        if (!grad_disp[s]) return fail(MD2_ERR_ARG, "grad_disp[%d] is NULL", s);
    hipStream_t st = (hipStream_t)stream;
    uint8_t* ws = (uint8_t*)workspace;
    PhotoArgs a;
    hipEvent_t c0 = nullptr, c1 = nullptr;
    if (L.v1) {
        for (int s = 0; s < L.nscales; ++s) {
            photo_args(d, t, L, s, s + 1, true, ws, (uint8_t*)select, a, grad_mask);
            a.grad_loss = grad_loss;
            launch_photo(a, true, st);
        }
    } else {
        hipEvent_t e0, e1;
        timing_slot(1, &e0, &e1);
        timing_slot(3, &c0, &c1, e0);   // the whole call: photo_bwd .. grad_T
        photo_args(d, t, L, 0, L.nscales, true, ws, (uint8_t*)select, a, grad_mask);
        a.grad_loss = grad_loss;
        launch_photo(a, true, st, e0, e1);
    }
    if ((rc = hip_check("photo_bwd_kernel"))) return rc;

    DispGradArgs g;
    memset(&g, 0, sizeof(g));
    g.B = L.B;
    g.num_scales = L.nscales;
    g.stats = (const float*)(ws + L.stats_off);
    g.grad_loss = grad_loss;
    g.smoothness = d->disparity_smoothness;
    g.disp_bf16 = d->disp_dtype == MD2_DTYPE_BF16;
    int gblocks = 0;
    g.quad = 1;
    for (int s = 0; s < L.nscales; ++s) g.quad &= (L.ws[s] % 4 == 0) ? 1 : 0;
    for (int s = 0; s < L.nscales; ++s) {   // all scales in one launch
        g.hs[s] = L.hs[s];
        g.ws[s] = L.ws[s];
        g.lh[s] = L.lh[s];
        g.lw[s] = L.lw[s];
        g.upsh[s] = L.v1 ? 0 : s;
        g.dfull[s] = (const float*)(ws + L.dfull_off[s]);
        g.upart[s] = (const float*)(ws + L.dfull_off[s]);
        g.strips[s] = L.bstrips[s];
        g.rowblocks[s] = L.brows[s];
        g.sgrad[s] = (const float*)(ws + L.sgrad_off[s]);
        g.out[s] = grad_disp[s];
        g.block_base[s] = gblocks;
        g.bpr[s] = (L.ws[s] + kBlock - 1) / kBlock;
        gblocks += g.quad ? (L.B * L.hs[s] * L.ws[s] / 4 + kBlock - 1) / kBlock : L.B * L.hs[s] * g.bpr[s];
    }
    g.block_base[L.nscales] = gblocks;

    DTArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.B = L.B;
    ta.S = L.S;
    ta.num_scales = L.nscales;
    ta.per_scale = (d->flags & MD2_T_PER_SCALE) ? 1 : 0;
    for (int s = 0; s < L.nscales; ++s) {
        ta.wpi[s] = L.B ? L.bwpi[s] : 0;
        ta.dP_part[s] = (const float*)(ws + L.dP_off[s]);
        ta.K[s] = t->K[L.v1 ? s : 0];
    }
    ta.grad_T = grad_T;
    const int nT = (ta.per_scale ? L.nscales : 1) * L.S * L.B, nTb = (nT + 7) / 8 * 8;
    if (c1)
        hipExtLaunchKernelGGL(disp_grad_T_kernel, dim3(nTb + gblocks), dim3(kBlock), 0, st, nullptr, c1, 0, g, ta, nT,
                              nTb);
    else
        hipLaunchKernelGGL(disp_grad_T_kernel, dim3(nTb + gblocks), dim3(kBlock), 0, st, g, ta, nT, nTb);
    return hip_check("disp_grad_T_kernel");
}

int md2_generate_images(const md2_desc* d, const md2_tensors* t, float* const* depth_out, float* const* sample_out,
                        float* const* color_out, void* stream) {
    Layout L;
    int rc = make_layout(d, L);
    if (rc) return rc;
    if ((rc = check_tensors(d, t, L, false))) return rc;
    hipStream_t st = (hipStream_t)stream;
    for (int s = 0; s < L.nscales; ++s) {
        GenArgs g;
        memset(&g, 0, sizeof(g));
        photo_args(d, t, L, L.v1 ? s : 0, L.v1 ? s + 1 : L.nscales, false, nullptr, nullptr, g.p);
        g.ls = L.v1 ? 0 : s;
        g.depth = depth_out ? depth_out[s] : nullptr;
        for (int f = 0; f < L.S; ++f) {
            g.sample[f] = sample_out ? sample_out[s * L.S + f] : nullptr;
            g.color[f] = color_out ? color_out[s * L.S + f] : nullptr;
        }
        const int n = L.B * L.lh[s] * L.lw[s];
        hipLaunchKernelGGL(generate_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, st, g);
    }
    return hip_check("generate_kernel");
}

int md2_tiebreak_noise(const md2_desc* d, const uint64_t* seed_ptr, int scale, float* out, void* stream) {
    Layout L;
    int rc = make_layout(d, L);
    if (rc) return rc;
    if (scale < 0 || scale >= L.nscales) return fail(MD2_ERR_ARG, "scale %d out of range", scale);
    if (!out) return fail(MD2_ERR_ARG, "out is NULL");
    NoiseArgs na;
    na.B = L.B;
    na.HW = L.lh[scale] * L.lw[scale];
    na.C = (d->flags & MD2_AVG_REPROJECTION) ? 1 : L.S;
    na.gsc = scale;
    na.seed = d->seed;
    na.seed_ptr = seed_ptr;
    na.out = out;
    const int n = na.B * na.HW;
    hipLaunchKernelGGL(tiebreak_noise_kernel, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, (hipStream_t)stream, na);
    return hip_check("tiebreak_noise_kernel");
}

int md2_timing_begin(int max_launches) {
    std::lock_guard<std::mutex> lk(g_timing.mu);
    if (max_launches < 1) return fail(MD2_ERR_ARG, "max_launches must be >= 1");
    for (hipEvent_t e : g_timing.ev) (void)hipEventDestroy(e);
    g_timing.ev.assign(2 * (size_t)max_launches, nullptr);
    g_timing.start.assign(max_launches, nullptr);
    g_timing.kind.assign(max_launches, 0);
    for (auto& e : g_timing.ev)
        if (hipEventCreate(&e) != hipSuccess) return fail(MD2_ERR_HIP, "hipEventCreate failed");
    g_timing.cap = max_launches;
    g_timing.used = 0;
    g_timing.on = true;
    return MD2_OK;
}

int md2_timing_end(double* fwd_ms, int* n_fwd, double* bwd_ms, int* n_bwd) {
    std::lock_guard<std::mutex> lk(g_timing.mu);
    if (!g_timing.on) return fail(MD2_ERR_ARG, "md2_timing_begin was not called");
    g_timing.on = false;
    double tot[4] = {0.0, 0.0, 0.0, 0.0};
    int cnt[4] = {0, 0, 0, 0};
    for (int i = 0; i < g_timing.used; ++i) {
        if (hipEventSynchronize(g_timing.ev[2 * i + 1]) != hipSuccess)
            return fail(MD2_ERR_HIP, "hipEventSynchronize failed");
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, g_timing.start[i], g_timing.ev[2 * i + 1]) != hipSuccess)
            return fail(MD2_ERR_HIP, "hipEventElapsedTime failed");
        tot[g_timing.kind[i]] += ms;
        cnt[g_timing.kind[i]] += 1;
    }
    g_timing.call_ms[0] = tot[2];
    g_timing.call_ms[1] = tot[3];
    g_timing.call_n[0] = cnt[2];
    g_timing.call_n[1] = cnt[3];
    if (fwd_ms) *fwd_ms = tot[0];
    if (n_fwd) *n_fwd = cnt[0];
    if (bwd_ms) *bwd_ms = tot[1];
    if (n_bwd) *n_bwd = cnt[1];
    return MD2_OK;
}

int md2_timing_calls(double* fwd_ms, int* n_fwd, double* bwd_ms, int* n_bwd) {
    std::lock_guard<std::mutex> lk(g_timing.mu);
    if (fwd_ms) *fwd_ms = g_timing.call_ms[0];
    if (n_fwd) *n_fwd = g_timing.call_n[0];
    if (bwd_ms) *bwd_ms = g_timing.call_ms[1];
    if (n_bwd) *n_bwd = g_timing.call_n[1];
    return MD2_OK;
}

}  // extern "C"
