// augment.hip — GPU input pipeline for gfx950.
//
// MonoDataset.__getitem__ (datasets/mono_dataset.py:136-200) runs flip, the cascaded
// PIL Resize(ANTIALIAS) pyramid, ToTensor and ColorJitter on the CPU workers, per
// image.  Here one batch of decoded frames is processed on the device with the same
// integer / float arithmetic as Pillow, so every output byte equals the reference's:
//
//   resize   Pillow's two-pass LANCZOS (Resample.c): per output column/row a window
//            [xmin, xmin+n) of 22-bit fixed-point weights, int32 accumulation from
//            1<<21, >>22, clipped to uint8; horizontal pass, uint8 image, vertical
//            pass.  Tables are built on the host in double exactly as Pillow does.
//            The flip is a pure column permutation, folded into the level-0
//            horizontal gather.  Level s resizes level s-1 (mono_dataset.py:99-101).
//   jitter   ImageEnhance.{Brightness,Contrast,Color} = Image.blend(degenerate,
//            image, f) in C float, truncated (clipped when f > 1); Contrast's
//            degenerate is int(mean(L) + 0.5) of the image as it stands when
//            contrast runs, so a reduction pass first replays the ops before it;
//            adjust_hue = RGB->HSV (Convert.c), uint8 hue add, HSV->RGB.
//   to_tensor  float(u8) / 255 for color and color_aug.
//
// Launches per batch: a memset, one fused (h+v, LDS-tiled, contrast-mean summing)
// resize per pyramid level, then one jitter/to_tensor pass over all levels.
// Integer atomics only (the contrast sums), so results are deterministic.

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <new>
#include <vector>

#include "md2hot.h"

int md2_report_error(int code, const char* msg);

// C float semantics for the blends / HSV maths: no FMA contraction in this file.
#pragma clang fp contract(off)

namespace {

constexpr int kPrecisionBits = 32 - 8 - 2;   // Resample.c PRECISION_BITS
constexpr int kThreads = 256;
constexpr int kRing = 4;   // pinned item-staging slots per plan

struct Rgb {
    int r, g, b;
};

__device__ __forceinline__ uint8_t clip8(int v) {
    v >>= kPrecisionBits;
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// Horizontal LANCZOS pass: (N, h, sw, 3) -> (N, h, dw, 3).  flip_items != nullptr
// (level 0 only): item b = n % B reads its source columns mirrored.
__global__ void __launch_bounds__(kThreads) resize_h_kernel(const uint8_t* __restrict__ src,
                                                            uint8_t* __restrict__ dst, int N, int h, int sw,
                                                            int dw, const int2* __restrict__ bounds,
                                                            const int* __restrict__ kk, int ksize,
                                                            const md2_aug_item* __restrict__ items, int B) {
    const size_t total = (size_t)N * h * dw;
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= total) return;
    const int x = (int)(i % dw);
    const size_t row = i / dw;   // n*h + y
    const bool flip = items && items[(int)((row / h) % B)].flip;
    const int2 bd = bounds[x];
    const int* k = kk + (size_t)x * ksize;
    const uint8_t* s = src + row * sw * 3;
    int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
    for (int t = 0; t < bd.y; ++t) {
        const int c = flip ? sw - 1 - (bd.x + t) : bd.x + t;
        const int w = k[t];
        a0 += (int)s[3 * c] * w;
        a1 += (int)s[3 * c + 1] * w;
        a2 += (int)s[3 * c + 2] * w;
    }
    uint8_t* o = dst + i * 3;
    o[0] = clip8(a0);
    o[1] = clip8(a1);
    o[2] = clip8(a2);
}

// Vertical LANCZOS pass: (N, sh, w, 3) -> (N, dh, w, 3).
__global__ void __launch_bounds__(kThreads) resize_v_kernel(const uint8_t* __restrict__ src,
                                                            uint8_t* __restrict__ dst, int N, int sh, int dh,
                                                            int w, const int2* __restrict__ bounds,
                                                            const int* __restrict__ kk, int ksize,
                                                            float* __restrict__ color, uint32_t* __restrict__ rgbx,
                                                            int B) {
    const size_t total = (size_t)N * dh * w;
    const size_t i = (size_t)blockIdx.x * kThreads + threadIdx.x;
    if (i >= total) return;
    const int x = (int)(i % w);
    const int y = (int)((i / w) % dh);
    const size_t n = i / ((size_t)w * dh);
    const int2 bd = bounds[y];
    const int* k = kk + (size_t)y * ksize;
    const uint8_t* s = src + ((n * sh + bd.x) * w + x) * 3;
    const size_t stride = (size_t)w * 3;
    int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
    for (int t = 0; t < bd.y; ++t) {
        const int wt = k[t];
        a0 += (int)s[t * stride] * wt;
        a1 += (int)s[t * stride + 1] * wt;
        a2 += (int)s[t * stride + 2] * wt;
    }
    uint8_t* o = dst + i * 3;
    o[0] = clip8(a0);
    o[1] = clip8(a1);
    o[2] = clip8(a2);
    const size_t hw = (size_t)dh * w;
    float* c = color + n * 3 * hw + (i - n * hw);
    c[0] = (float)o[0] / 255.f;
    c[hw] = (float)o[1] / 255.f;
    c[2 * hw] = (float)o[2] / 255.f;
    if (rgbx && n >= (size_t)B)   // frames 1.. (the photometric sources) as RGBx dwords
        rgbx[(n - B) * hw + (i - n * hw)] = (uint32_t)o[0] | ((uint32_t)o[1] << 8) | ((uint32_t)o[2] << 16);
}

// Both LANCZOS passes of one pyramid level for a TW x TH output tile, through LDS:
// the tile's input rows are staged once by LDS-DMA (global_load_lds_dword, every row
// in flight at once); the horizontal pass reads each lane's whole KX-tap window as
// aligned dwords, realigns them with v_alignbyte and takes the bytes at compile-time
// positions (sub-dword LDS reads at odd addresses run at a fraction of the rate);
// taps past a clipped window carry zero weight.  The uint8 intermediate is one
// aligned RGBx dword per pixel; the vertical pass writes the level (uint8, for the
// next level and the jitter) and its to_tensor (color), and adds the tile's share of
// the contrast degenerate sum (see mean_kernel).  A flipped item reads its staged
// rows mirrored (the flip is a column permutation of the source).  One wave per row,
// lane = output column.  Weights are < 2^23 in magnitude: 24-bit multiplies.
constexpr int kTileW = 64;
constexpr int kTileH = 16;
constexpr int kPatchPad = 64;   // bytes before / after the staged rows (clipped windows)

struct FusedLds {
    int patch, inter;   // byte offsets (patch includes kPatchPad in front)
    int cin_max, rin_max;
    int pitch;          // bytes per staged row (multiple of 4, >= cin_max*3 + 3)
    int bytes;
};

__device__ __forceinline__ int gray(const Rgb& p);
__device__ __forceinline__ int contrast_pos(const md2_aug_item& it);
__device__ int contrast_gray(int r, int g, int b, uint32_t order, float fb, float fc, float fs, int hue, int stop);

// Accumulate KX taps from the realigned window e[] (byte 3p+c = pixel p, channel c);
// tap t reads pixel t, or KX-1-t for a flipped row.
template <int KX, int ND, bool FLIP>
__device__ __forceinline__ void window_taps(const uint32_t (&e)[ND - 1], const int (&wx)[KX], int& a0, int& a1,
                                            int& a2) {
#pragma unroll
    for (int t = 0; t < KX; ++t) {
        const int o = 3 * (FLIP ? KX - 1 - t : t);
        const int w = wx[t];
        a0 += __mul24((int)((e[o >> 2] >> (8 * (o & 3))) & 255), w);
        a1 += __mul24((int)((e[(o + 1) >> 2] >> (8 * ((o + 1) & 3))) & 255), w);
        a2 += __mul24((int)((e[(o + 2) >> 2] >> (8 * ((o + 2) & 3))) & 255), w);
    }
}

template <int KX, int KY>
__global__ void __launch_bounds__(kThreads) resize_fused_kernel(
    const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, float* __restrict__ color, int sh, int sw, int dh,
    int dw, const int2* __restrict__ bx, const int* __restrict__ kx, const int2* __restrict__ by,
    const int* __restrict__ ky, FusedLds L, const md2_aug_item* __restrict__ items, int B, int flip_level,
    unsigned long long* __restrict__ sums, uint32_t* __restrict__ rgbx) {
    extern __shared__ __align__(16) uint8_t lds[];
    uint8_t* patch = lds + L.patch;
    uint32_t* inter = (uint32_t*)(lds + L.inter);
    const int n = blockIdx.z;
    const int x0 = blockIdx.x * kTileW, y0 = blockIdx.y * kTileH;
    const int tw = min(kTileW, dw - x0), th = min(kTileH, dh - y0);
    const int c0 = bx[x0].x, c1 = bx[x0 + tw - 1].x + bx[x0 + tw - 1].y;
    const int r0 = by[y0].x, r1 = by[y0 + th - 1].x + by[y0 + th - 1].y;
    const int cin3 = (c1 - c0) * 3, rin = r1 - r0;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const md2_aug_item it = items[n % B];
    const bool flip = flip_level && it.flip;
    const int pc0 = flip ? sw - c1 : c0;   // first source column of the staged segment
    // stage: row r's segment [pc0, pc0 + (c1-c0)) from its 4-byte-aligned start
    for (int r = wave; r < rin; r += kThreads / 64) {
        const uint8_t* g = src + (((size_t)n * sh + r0 + r) * sw + pc0) * 3;
        const uint32_t* ga = (const uint32_t*)((uintptr_t)g & ~(uintptr_t)3);
        const int nd = ((int)((uintptr_t)g & 3) + cin3 + 3) >> 2;
        for (int j0 = 0; j0 < nd; j0 += 64)
            if (j0 + lane < nd)
                __builtin_amdgcn_global_load_lds(ga + j0 + lane, (uint32_t*)(patch + r * L.pitch) + j0, 4, 0, 0);
    }
    // this lane's horizontal weights, in registers for every row
    int wx[KX];
    const int xo = min(x0 + lane, dw - 1);
    const int2 b = bx[xo];
#pragma unroll
    for (int t = 0; t < KX; ++t) wx[t] = kx[(size_t)xo * KX + t];
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    // horizontal pass -> RGBx intermediate (rin rows x tw columns)
    constexpr int ND = (3 * KX + 3 + 3) / 4 + 1;   // dwords covering a window at any byte offset
    if (lane < tw) {
        // first staged pixel of the window: tap t sits at pixel (first + t), or (first + KX-1-t) flipped
        const int first = flip ? (c1 - 1 - b.x) - (KX - 1) : (b.x - c0);
        for (int r = wave; r < rin; r += kThreads / 64) {
            const int shift = (int)((uintptr_t)(src + (((size_t)n * sh + r0 + r) * sw + pc0) * 3) & 3);
            const int byte0 = r * L.pitch + shift + first * 3;   // may be < 0 (pad) when clipped
            const uint32_t* q = (const uint32_t*)(patch + (byte0 & ~3));
            const int off = byte0 & 3;
            uint32_t d[ND];
#pragma unroll
            for (int k = 0; k < ND; ++k) d[k] = q[k];
            uint32_t e[ND - 1];
#pragma unroll
            for (int k = 0; k < ND - 1; ++k) e[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], off);
            int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
            if (flip)   // block-uniform; two unrolled bodies keep e[] indices compile-time
                window_taps<KX, ND, true>(e, wx, a0, a1, a2);
            else
                window_taps<KX, ND, false>(e, wx, a0, a1, a2);
            inter[r * kTileW + lane] = (uint32_t)clip8(a0) | ((uint32_t)clip8(a1) << 8) | ((uint32_t)clip8(a2) << 16);
        }
    }
    __syncthreads();
    // vertical pass -> level output + to_tensor (+ contrast-mean share)
    unsigned long long msum = 0;
    if (lane < tw) {
        const size_t hw = (size_t)dh * dw;
        const int stop = it.color_aug ? contrast_pos(it) : 0;
        const uint32_t order = (uint32_t)it.order[0] | ((uint32_t)it.order[1] << 8) | ((uint32_t)it.order[2] << 16) |
                               ((uint32_t)it.order[3] << 24);
        for (int y = wave; y < th; y += kThreads / 64) {
            const int2 bb = by[y0 + y];
            const int* k = ky + (size_t)(y0 + y) * KY;
            const uint32_t* p = inter + (bb.x - r0) * kTileW + lane;
            int a0 = 1 << (kPrecisionBits - 1), a1 = a0, a2 = a0;
#pragma unroll
            for (int t = 0; t < KY; ++t) {
                if (t < bb.y) {   // wave-uniform; rows past a clipped window are not staged
                    const int w = k[t];
                    const uint32_t v = p[t * kTileW];
                    a0 += __mul24((int)(v & 255), w);
                    a1 += __mul24((int)((v >> 8) & 255), w);
                    a2 += __mul24((int)((v >> 16) & 255), w);
                }
            }
            const size_t pix = (size_t)(y0 + y) * dw + x0 + lane;
            uint8_t* o = dst + ((size_t)n * hw + pix) * 3;
            const uint8_t v0 = clip8(a0), v1 = clip8(a1), v2 = clip8(a2);
            o[0] = v0;
            o[1] = v1;
            o[2] = v2;
            float* c = color + (size_t)n * 3 * hw + pix;
            c[0] = (float)v0 / 255.f;
            c[hw] = (float)v1 / 255.f;
            c[2 * hw] = (float)v2 / 255.f;
            if (rgbx && n >= B)   // block-uniform: frames 1.. (the photometric sources) as RGBx dwords
                rgbx[(size_t)(n - B) * hw + pix] = (uint32_t)v0 | ((uint32_t)v1 << 8) | ((uint32_t)v2 << 16);
            if (it.color_aug)
                msum += (unsigned long long)contrast_gray(v0, v1, v2, order, it.brightness, it.contrast,
                                                          it.saturation, it.hue_shift, stop);
        }
    }
    if (it.color_aug) {   // block-uniform
        for (int off = 32; off > 0; off >>= 1) msum += __shfl_down(msum, off, 64);
        __shared__ unsigned long long part[kThreads / 64];
        if (lane == 0) part[wave] = msum;
        __syncthreads();
        if (threadIdx.x == 0) atomicAdd(sums + n, part[0] + part[1] + part[2] + part[3]);
    }
}

// ---- the ColorJitter ops, in Pillow's C arithmetic ---------------------------------
__device__ __forceinline__ int gray(const Rgb& p) {   // Convert.c rgb2l
    return (p.r * 19595 + p.g * 38470 + p.b * 7471 + 0x8000) >> 16;
}

// Image.blend(deg, img, alpha) per channel (Blend.c).
__device__ __forceinline__ int blend1(int in1, int in2, float alpha) {
    const float v = (float)in1 + alpha * (float)(in2 - in1);
    if (alpha >= 0.f && alpha <= 1.f) return (int)(uint8_t)v;
    if (v <= 0.f) return 0;
    if (v >= 255.f) return 255;
    return (int)(uint8_t)v;
}

__device__ __forceinline__ Rgb blend(const Rgb& d, const Rgb& p, float alpha) {
    if (alpha == 0.f) return d;
    if (alpha == 1.f) return p;
    return {blend1(d.r, p.r, alpha), blend1(d.g, p.g, alpha), blend1(d.b, p.b, alpha)};
}

__device__ __forceinline__ int clip8i(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// Convert.c rgb2hsv_row, then the uint8 hue add of adjust_hue, then hsv2rgb.
__device__ Rgb hue_op(const Rgb& p, int shift) {
    const int maxc = max(p.r, max(p.g, p.b));
    const int minc = min(p.r, min(p.g, p.b));
    int uh, us;
    const int uv = maxc;
    if (minc == maxc) {
        uh = 0;
        us = 0;
    } else {
        const float cr = (float)(maxc - minc);
        const float s = cr / (float)maxc;
        const float rc = (float)(maxc - p.r) / cr;
        const float gc = (float)(maxc - p.g) / cr;
        const float bc = (float)(maxc - p.b) / cr;
        float h;
        if (p.r == maxc)
            h = bc - gc;
        else if (p.g == maxc)
            h = (float)(2.0 + (double)rc - (double)bc);
        else
            h = (float)(4.0 + (double)gc - (double)rc);
        const double y = (double)h / 6.0 + 1.0;   // in [5/6, 11/6): fmod(y, 1) is y or y - 1, exact
        h = (float)(y >= 1.0 ? y - 1.0 : y);
        uh = clip8i((int)((double)h * 255.0));
        us = clip8i((int)((double)s * 255.0));
    }
    const int hh = (uh + shift) & 255;
    if (us == 0) return {uv, uv, uv};
    const double hf = (double)(float)hh * 6.0 / 255.0;
    const int i = (int)floor(hf);
    const float f = (float)(hf - (double)(float)i);
    const float fs = (float)((double)(float)us / 255.0);
    const double v = (double)(float)uv;
    const int pp = clip8i((int)round(v * (1.0 - (double)fs)));
    const int q = clip8i((int)round(v * (1.0 - (double)(fs * f))));
    const int t = clip8i((int)round(v * (1.0 - (double)fs * (1.0 - (double)f))));
    switch (i % 6) {
        case 0: return {uv, t, pp};
        case 1: return {q, uv, pp};
        case 2: return {pp, uv, t};
        case 3: return {pp, q, uv};
        case 4: return {t, pp, uv};
        default: return {uv, pp, q};
    }
}

__device__ __forceinline__ Rgb apply_op(int op, const Rgb& p, const md2_aug_item& it, int mean) {
    switch (op) {
        case MD2_AUG_BRIGHTNESS: return blend({0, 0, 0}, p, it.brightness);
        case MD2_AUG_CONTRAST: return blend({mean, mean, mean}, p, it.contrast);
        case MD2_AUG_SATURATION: {
            const int l = gray(p);
            return blend({l, l, l}, p, it.saturation);
        }
        default: return hue_op(p, it.hue_shift);
    }
}

__device__ __forceinline__ int contrast_pos(const md2_aug_item& it) {
    for (int k = 0; k < 4; ++k)
        if (it.order[k] == MD2_AUG_CONTRAST) return k;
    return 4;
}

// gray() of the pixel after the ops that precede contrast (its degenerate's input).
// (Out of line and by value: it is called once per pixel, from every resize instance.)
__device__ __noinline__ int contrast_gray(int r, int g, int b, uint32_t order, float fb, float fc, float fs, int hue,
                                          int stop) {
    md2_aug_item it{};
    it.brightness = fb;
    it.contrast = fc;
    it.saturation = fs;
    it.hue_shift = (uint8_t)hue;
    Rgb v{r, g, b};
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (k < stop) v = apply_op((int)((order >> (8 * k)) & 255u), v, it, 0);
    return gray(v);
}

// The pyramid levels of one batch, for the all-level mean / apply launches.
struct Levels {
    const uint8_t* img[MD2_MAX_SCALES];   // nullptr: level skipped (mean_kernel)
    float* aug[MD2_MAX_SCALES];
    int hw[MD2_MAX_SCALES];
    int first[MD2_MAX_SCALES + 1];   // first block of each level along gridDim.x
    int nlev, N;
};

__device__ __forceinline__ int level_of(const Levels& L, int bx) {
    int s = 0;
    while (s + 1 < L.nlev && bx >= L.first[s + 1]) ++s;
    return s;
}

// Contrast degenerate: sum of L over the image as it stands when contrast runs
// (ImageEnhance.Contrast, ImageStat mean).  Exact integer sums per (level, image).
__global__ void __launch_bounds__(kThreads) mean_kernel(Levels L, int B, const md2_aug_item* __restrict__ items,
                                                        unsigned long long* __restrict__ sums) {
    const int n = blockIdx.y;
    const md2_aug_item it = items[n % B];
    if (!it.color_aug) return;
    const int s = level_of(L, blockIdx.x);
    if (!L.img[s]) return;   // fused level: summed inside resize_fused_kernel
    const int hw = L.hw[s], nb = L.first[s + 1] - L.first[s];
    const int stop = contrast_pos(it);
    const uint8_t* img = L.img[s] + (size_t)n * hw * 3;
    unsigned long long acc = 0;
    for (int p = (blockIdx.x - L.first[s]) * kThreads + threadIdx.x; p < hw; p += nb * kThreads) {
        const uint8_t* q = img + (size_t)p * 3;
        Rgb v{q[0], q[1], q[2]};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (k < stop) v = apply_op(it.order[k], v, it, 0);
        acc += (unsigned long long)gray(v);
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    __shared__ unsigned long long part[kThreads / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kThreads / 64; ++w) t += part[w];
        atomicAdd(sums + (size_t)s * L.N + n, t);
    }
}

// to_tensor(color_aug(img)) -> color_aug (planar float), every level in one launch.
__global__ void __launch_bounds__(kThreads) apply_kernel(Levels L, int B, const md2_aug_item* __restrict__ items,
                                                         const unsigned long long* __restrict__ sums) {
    const int n = blockIdx.y;
    const int s = level_of(L, blockIdx.x);
    const int hw = L.hw[s];
    const int p = (blockIdx.x - L.first[s]) * kThreads + threadIdx.x;
    if (p >= hw) return;
    const md2_aug_item it = items[n % B];
    const uint8_t* q = L.img[s] + ((size_t)n * hw + p) * 3;
    Rgb v{q[0], q[1], q[2]};
    if (it.color_aug) {
        const int mean = (int)((double)sums[(size_t)s * L.N + n] / (double)hw + 0.5);
        for (int k = 0; k < 4; ++k) v = apply_op(it.order[k], v, it, mean);
    }
    float* a = L.aug[s] + (size_t)n * 3 * hw + p;
    a[0] = (float)v.r / 255.f;
    a[hw] = (float)v.g / 255.f;
    a[2 * hw] = (float)v.b / 255.f;
}

// ---- host: Pillow's precompute_coeffs + normalize_coeffs_8bpc ----------------------
double sinc(double x) {
    if (x == 0.0) return 1.0;
    x = x * M_PI;
    return sin(x) / x;
}

double lanczos(double x) { return (-3.0 <= x && x < 3.0) ? sinc(x) * sinc(x / 3.0) : 0.0; }

int lanczos_ksize(int in_size, int out_size) {
    double fs = (double)in_size / out_size;
    if (fs < 1.0) fs = 1.0;
    return (int)ceil(3.0 * fs) * 2 + 1;
}

void lanczos_tables(int in_size, int out_size, std::vector<int2>& bounds, std::vector<int>& kk) {
    const double scale = (double)in_size / out_size;
    const double filterscale = scale < 1.0 ? 1.0 : scale;
    const double support = 3.0 * filterscale;
    const int ksize = lanczos_ksize(in_size, out_size);
    bounds.assign(out_size, int2{0, 0});
    kk.assign((size_t)out_size * ksize, 0);
    std::vector<double> w(ksize);
    const double ss = 1.0 / filterscale;
    for (int xx = 0; xx < out_size; ++xx) {
        const double center = (xx + 0.5) * scale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        double ww = 0.0;
        for (int x = 0; x < xmax; ++x) {
            w[x] = lanczos((x + xmin - center + 0.5) * ss);
            ww += w[x];
        }
        for (int x = 0; x < xmax; ++x) {
            const double k = ww != 0.0 ? w[x] / ww : w[x];
            kk[(size_t)xx * ksize + x] =
                k < 0 ? (int)(-0.5 + k * (1 << kPrecisionBits)) : (int)(0.5 + k * (1 << kPrecisionBits));
        }
        bounds[xx] = int2{xmin, xmax};
    }
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// resize_fused_kernel instantiation for the two window sizes (2*ceil(3*max(scale,1))+1:
// 7 up-scaling, 9/11/13 down to 2x), nullptr for wider windows (two-pass kernels).
using FusedFn = void (*)(const uint8_t*, uint8_t*, float*, int, int, int, int, const int2*, const int*,
                         const int2*, const int*, FusedLds, const md2_aug_item*, int, int, unsigned long long*,
                         uint32_t*);

template <int KX>
FusedFn fused_for_ky(int ky) {
    switch (ky) {
        case 7: return resize_fused_kernel<KX, 7>;
        case 9: return resize_fused_kernel<KX, 9>;
        case 11: return resize_fused_kernel<KX, 11>;
        case 13: return resize_fused_kernel<KX, 13>;
        default: return nullptr;
    }
}

FusedFn fused_kernel(int kx, int ky) {
    switch (kx) {
        case 7: return fused_for_ky<7>(ky);
        case 9: return fused_for_ky<9>(ky);
        case 11: return fused_for_ky<11>(ky);
        case 13: return fused_for_ky<13>(ky);
        default: return nullptr;
    }
}

// LDS layout of resize_fused_kernel for one level: the widest input patch over all
// tiles.  bytes > 64 KB (extreme down-scaling) selects the two-pass kernels instead.
FusedLds fused_layout(const std::vector<int2>& bx, const std::vector<int2>& by) {
    FusedLds L{};
    const int dw = (int)bx.size(), dh = (int)by.size();
    for (int x0 = 0; x0 < dw; x0 += kTileW) {
        const int xl = std::min(x0 + kTileW, dw) - 1;
        L.cin_max = std::max(L.cin_max, bx[xl].x + bx[xl].y - bx[x0].x);
    }
    for (int y0 = 0; y0 < dh; y0 += kTileH) {
        const int yl = std::min(y0 + kTileH, dh) - 1;
        L.rin_max = std::max(L.rin_max, by[yl].x + by[yl].y - by[y0].x);
    }
    L.pitch = (L.cin_max * 3 + 3 + 3) & ~3;
    L.patch = kPatchPad;
    L.inter = (kPatchPad + L.rin_max * L.pitch + kPatchPad + 15) & ~15;
    L.bytes = L.inter + L.rin_max * kTileW * 4;
    return L;
}

unsigned blocks_for(size_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

}  // namespace

struct md2_aug_plan {
    md2_aug_desc d;
    int N = 0;
    int h[MD2_MAX_SCALES], w[MD2_MAX_SCALES];     // level sizes
    int sh[MD2_MAX_SCALES], sw[MD2_MAX_SCALES];   // their sources
    int kx[MD2_MAX_SCALES], ky[MD2_MAX_SCALES];   // ksize per pass
    int2* bx[MD2_MAX_SCALES];
    int2* by[MD2_MAX_SCALES];
    int* wx[MD2_MAX_SCALES];
    int* wy[MD2_MAX_SCALES];
    uint8_t* pyr[MD2_MAX_SCALES];
    FusedLds lds[MD2_MAX_SCALES];
    bool fused[MD2_MAX_SCALES];
    uint8_t* mid = nullptr;   // two-pass intermediate (levels that are not fused)
    unsigned long long* sums = nullptr;
    md2_aug_item* dev_items = nullptr;    // kRing slots of d.items on the device
    md2_aug_item* host_items = nullptr;   // pinned staging, same shape
    hipEvent_t staged[kRing] = {};        // slot reusable once its upload has run
    int slot = 0;
    void* block = nullptr;
};

extern "C" {

md2_aug_plan* md2_aug_plan_create(const md2_aug_desc* d) {
    if (!d) return md2_report_error(MD2_ERR_ARG, "aug desc is NULL"), nullptr;
    if (d->items < 1 || d->frames < 1 || d->frames > 8)
        return md2_report_error(MD2_ERR_ARG, "aug: need items >= 1 and frames in 1..8"), nullptr;
    if (d->num_scales < 1 || d->num_scales > MD2_MAX_SCALES)
        return md2_report_error(MD2_ERR_ARG, "aug: num_scales must be 1..4"), nullptr;
    if (d->in_height < 1 || d->in_width < 1 || (d->height >> (d->num_scales - 1)) < 1 ||
        (d->width >> (d->num_scales - 1)) < 1)
        return md2_report_error(MD2_ERR_ARG, "aug: every pyramid level must be at least 1x1"), nullptr;
    auto* P = new (std::nothrow) md2_aug_plan();
    if (!P) return md2_report_error(MD2_ERR_ARG, "aug: out of host memory"), nullptr;
    P->d = *d;
    P->N = d->items * d->frames;
    std::vector<int2> bxh[MD2_MAX_SCALES], byh[MD2_MAX_SCALES];
    std::vector<int> wxh[MD2_MAX_SCALES], wyh[MD2_MAX_SCALES];
    size_t off = 0, mid = 0;
    size_t o_bx[MD2_MAX_SCALES], o_by[MD2_MAX_SCALES], o_wx[MD2_MAX_SCALES], o_wy[MD2_MAX_SCALES],
        o_pyr[MD2_MAX_SCALES];
    for (int s = 0; s < d->num_scales; ++s) {
        P->h[s] = d->height >> s;
        P->w[s] = d->width >> s;
        P->sh[s] = s ? P->h[s - 1] : d->in_height;
        P->sw[s] = s ? P->w[s - 1] : d->in_width;
        P->kx[s] = lanczos_ksize(P->sw[s], P->w[s]);
        P->ky[s] = lanczos_ksize(P->sh[s], P->h[s]);
        lanczos_tables(P->sw[s], P->w[s], bxh[s], wxh[s]);
        lanczos_tables(P->sh[s], P->h[s], byh[s], wyh[s]);
        o_bx[s] = off; off = align256(off + bxh[s].size() * sizeof(int2));
        o_by[s] = off; off = align256(off + byh[s].size() * sizeof(int2));
        o_wx[s] = off; off = align256(off + wxh[s].size() * sizeof(int));
        o_wy[s] = off; off = align256(off + wyh[s].size() * sizeof(int));
        o_pyr[s] = off; off = align256(off + (size_t)P->N * P->h[s] * P->w[s] * 3);
        P->lds[s] = fused_layout(bxh[s], byh[s]);
        P->fused[s] = P->lds[s].bytes <= 64 * 1024 && fused_kernel(P->kx[s], P->ky[s]) != nullptr;
        const size_t m = (size_t)P->N * P->sh[s] * P->w[s] * 3;
        if (!P->fused[s] && m > mid) mid = m;
    }
    const size_t o_mid = off;
    off = align256(off + mid);
    const size_t o_sums = off;
    off = align256(off + (size_t)P->N * d->num_scales * sizeof(unsigned long long));
    const size_t o_items = off;
    const size_t item_bytes = (size_t)kRing * d->items * sizeof(md2_aug_item);
    off = align256(off + item_bytes);
    if (hipMalloc(&P->block, off) != hipSuccess) {
        delete P;
        return md2_report_error(MD2_ERR_HIP, "aug: hipMalloc of the pyramid scratch failed"), nullptr;
    }
    char* base = (char*)P->block;
    for (int s = 0; s < d->num_scales; ++s) {
        P->bx[s] = (int2*)(base + o_bx[s]);
        P->by[s] = (int2*)(base + o_by[s]);
        P->wx[s] = (int*)(base + o_wx[s]);
        P->wy[s] = (int*)(base + o_wy[s]);
        P->pyr[s] = (uint8_t*)(base + o_pyr[s]);
        hipError_t e = hipMemcpy(P->bx[s], bxh[s].data(), bxh[s].size() * sizeof(int2), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(P->by[s], byh[s].data(), byh[s].size() * sizeof(int2), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(P->wx[s], wxh[s].data(), wxh[s].size() * sizeof(int), hipMemcpyHostToDevice);
        if (e == hipSuccess)
            e = hipMemcpy(P->wy[s], wyh[s].data(), wyh[s].size() * sizeof(int), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipFree(P->block);
            delete P;
            return md2_report_error(MD2_ERR_HIP, "aug: uploading the LANCZOS tables failed"), nullptr;
        }
    }
    P->mid = (uint8_t*)(base + o_mid);
    P->sums = (unsigned long long*)(base + o_sums);
    P->dev_items = (md2_aug_item*)(base + o_items);
    bool ok = hipHostMalloc((void**)&P->host_items, item_bytes, hipHostMallocDefault) == hipSuccess;
    for (int r = 0; ok && r < kRing; ++r)
        ok = hipEventCreateWithFlags(&P->staged[r], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        md2_aug_plan_destroy(P);
        return md2_report_error(MD2_ERR_HIP, "aug: pinned staging / events allocation failed"), nullptr;
    }
    return P;
}

void md2_aug_plan_destroy(md2_aug_plan* P) {
    if (!P) return;
    for (int r = 0; r < kRing; ++r)
        if (P->staged[r]) {
            (void)hipEventSynchronize(P->staged[r]);
            (void)hipEventDestroy(P->staged[r]);
        }
    if (P->host_items) (void)hipHostFree(P->host_items);
    if (P->block) (void)hipFree(P->block);
    delete P;
}

int md2_aug_run(md2_aug_plan* P, const uint8_t* frames, const md2_aug_item* host_items, float* const* color,
                float* const* color_aug, void* stream) {
    return md2_aug_run2(P, frames, host_items, color, color_aug, nullptr, stream);
}

int md2_aug_run2(md2_aug_plan* P, const uint8_t* frames, const md2_aug_item* host_items, float* const* color,
                 float* const* color_aug, uint32_t* src8, void* stream) {
    if (!P || !frames || !host_items || !color || !color_aug)
        return md2_report_error(MD2_ERR_ARG, "aug: plan/frames/items/color/color_aug is NULL");
    const md2_aug_desc& d = P->d;
    for (int s = 0; s < d.num_scales; ++s)
        if (!color[s] || !color_aug[s]) return md2_report_error(MD2_ERR_ARG, "aug: color[s]/color_aug[s] is NULL");
    for (int b = 0; b < d.items; ++b) {
        const md2_aug_item& it = host_items[b];
        unsigned seen = 0;
        for (int k = 0; k < 4; ++k) seen |= it.order[k] < 4 ? 1u << it.order[k] : 16u;
        if (seen != 15u) return md2_report_error(MD2_ERR_ARG, "aug: items[b].order must be a permutation of 0..3");
    }
    hipStream_t st = (hipStream_t)stream;
    const int N = P->N, B = d.items;
    // stage the item parameters: pinned slot -> device slot, asynchronously on `st`
    const int r = P->slot;
    P->slot = (P->slot + 1) % kRing;
    if (hipEventSynchronize(P->staged[r]) != hipSuccess)
        return md2_report_error(MD2_ERR_HIP, "aug: waiting for a staging slot failed");
    memcpy(P->host_items + (size_t)r * B, host_items, (size_t)B * sizeof(md2_aug_item));
    const md2_aug_item* items = P->dev_items + (size_t)r * B;
    if (hipMemcpyAsync((void*)items, P->host_items + (size_t)r * B, (size_t)B * sizeof(md2_aug_item),
                       hipMemcpyHostToDevice, st) != hipSuccess ||
        hipEventRecord(P->staged[r], st) != hipSuccess)
        return md2_report_error(MD2_ERR_HIP, "aug: staging the item parameters failed");
    if (hipMemsetAsync(P->sums, 0, (size_t)N * d.num_scales * sizeof(unsigned long long), st) != hipSuccess)
        return md2_report_error(MD2_ERR_HIP, "aug: hipMemsetAsync failed");
    for (int s = 0; s < d.num_scales; ++s) {
        const uint8_t* src = s ? P->pyr[s - 1] : frames;
        const md2_aug_item* flip = s ? nullptr : items;
        if (P->fused[s]) {
            const dim3 grid((P->w[s] + kTileW - 1) / kTileW, (P->h[s] + kTileH - 1) / kTileH, N);
            hipLaunchKernelGGL(fused_kernel(P->kx[s], P->ky[s]), grid, dim3(kThreads), P->lds[s].bytes, st, src,
                               P->pyr[s], color[s], P->sh[s], P->sw[s], P->h[s], P->w[s], P->bx[s], P->wx[s],
                               P->by[s], P->wy[s], P->lds[s], items, B, s == 0 ? 1 : 0, P->sums + (size_t)s * N,
                               s == 0 ? src8 : nullptr);
        } else {
            hipLaunchKernelGGL(resize_h_kernel, dim3(blocks_for((size_t)N * P->sh[s] * P->w[s])), dim3(kThreads), 0,
                               st, src, P->mid, N, P->sh[s], P->sw[s], P->w[s], P->bx[s], P->wx[s], P->kx[s], flip, B);
            hipLaunchKernelGGL(resize_v_kernel, dim3(blocks_for((size_t)N * P->h[s] * P->w[s])), dim3(kThreads), 0,
                               st, P->mid, P->pyr[s], N, P->sh[s], P->h[s], P->w[s], P->by[s], P->wy[s], P->ky[s],
                               color[s], s == 0 ? src8 : nullptr, B);
        }
    }
    Levels L{};
    L.nlev = d.num_scales;
    L.N = N;
    Levels M = L;   // the mean pass caps blocks per image at 64 per level
    bool any_two_pass = false;
    for (int s = 0; s < d.num_scales; ++s) {
        any_two_pass |= !P->fused[s];
        L.img[s] = P->pyr[s];
        M.img[s] = P->fused[s] ? nullptr : P->pyr[s];
        L.aug[s] = M.aug[s] = color_aug[s];
        L.hw[s] = M.hw[s] = P->h[s] * P->w[s];
        const int nb = (int)blocks_for(L.hw[s]);
        L.first[s + 1] = L.first[s] + nb;
        M.first[s + 1] = M.first[s] + std::min(nb, 64);
    }
    if (any_two_pass)
        hipLaunchKernelGGL(mean_kernel, dim3(M.first[d.num_scales], N), dim3(kThreads), 0, st, M, B, items, P->sums);
    hipLaunchKernelGGL(apply_kernel, dim3(L.first[d.num_scales], N), dim3(kThreads), 0, st, L, B, items, P->sums);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
