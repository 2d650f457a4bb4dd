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
// Launches per batch: 2 per pyramid level (h, v), one memset + one mean pass + one
// apply pass per level.  All passes are thread-per-output-pixel gathers; integer
// atomics only (the contrast sums), so results are deterministic.

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <string.h>

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
                                                            const int* __restrict__ kk, int ksize) {
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
        h = (float)fmod((double)h / 6.0 + 1.0, 1.0);
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

// Contrast degenerate: sum of L over the image as it stands when contrast runs
// (ImageEnhance.Contrast, ImageStat mean).  Exact integer sums per image.
__global__ void __launch_bounds__(kThreads) mean_kernel(const uint8_t* __restrict__ img, int hw, int B,
                                                        const md2_aug_item* __restrict__ items,
                                                        unsigned long long* __restrict__ sums) {
    const int n = blockIdx.y;
    const md2_aug_item it = items[n % B];
    if (!it.color_aug) return;
    const int stop = contrast_pos(it);
    unsigned long long acc = 0;
    for (int p = blockIdx.x * kThreads + threadIdx.x; p < hw; p += gridDim.x * kThreads) {
        const uint8_t* s = img + ((size_t)n * hw + p) * 3;
        Rgb v{s[0], s[1], s[2]};
        for (int k = 0; k < stop; ++k) v = apply_op(it.order[k], v, it, 0);
        acc += (unsigned long long)gray(v);
    }
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
    __shared__ unsigned long long part[kThreads / 64];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kThreads / 64; ++w) t += part[w];
        atomicAdd(sums + n, t);
    }
}

// to_tensor(img) -> color, to_tensor(color_aug(img)) -> color_aug (planar float).
__global__ void __launch_bounds__(kThreads) apply_kernel(const uint8_t* __restrict__ img, int hw, int B,
                                                         const md2_aug_item* __restrict__ items,
                                                         const unsigned long long* __restrict__ sums,
                                                         float* __restrict__ color, float* __restrict__ color_aug) {
    const int n = blockIdx.y;
    const int p = blockIdx.x * kThreads + threadIdx.x;
    if (p >= hw) return;
    const md2_aug_item it = items[n % B];
    const uint8_t* s = img + ((size_t)n * hw + p) * 3;
    Rgb v{s[0], s[1], s[2]};
    float* c = color + (size_t)n * 3 * hw + p;
    c[0] = (float)v.r / 255.f;
    c[hw] = (float)v.g / 255.f;
    c[2 * hw] = (float)v.b / 255.f;
    if (it.color_aug) {
        const int mean = (int)((double)sums[n] / (double)hw + 0.5);
        for (int k = 0; k < 4; ++k) v = apply_op(it.order[k], v, it, mean);
    }
    float* a = color_aug + (size_t)n * 3 * hw + p;
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
    uint8_t* mid = nullptr;
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
        const size_t m = (size_t)P->N * P->sh[s] * P->w[s] * 3;
        if (m > mid) mid = m;
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
        hipLaunchKernelGGL(resize_h_kernel, dim3(blocks_for((size_t)N * P->sh[s] * P->w[s])), dim3(kThreads), 0, st,
                           src, P->mid, N, P->sh[s], P->sw[s], P->w[s], P->bx[s], P->wx[s], P->kx[s],
                           s ? nullptr : items, B);
        hipLaunchKernelGGL(resize_v_kernel, dim3(blocks_for((size_t)N * P->h[s] * P->w[s])), dim3(kThreads), 0, st,
                           P->mid, P->pyr[s], N, P->sh[s], P->h[s], P->w[s], P->by[s], P->wy[s], P->ky[s]);
    }
    for (int s = 0; s < d.num_scales; ++s) {
        const int hw = P->h[s] * P->w[s];
        const unsigned gx = blocks_for(hw);
        unsigned long long* sums = P->sums + (size_t)s * N;
        hipLaunchKernelGGL(mean_kernel, dim3(gx < 64 ? gx : 64, N), dim3(kThreads), 0, st, P->pyr[s], hw, B, items,
                           sums);
        hipLaunchKernelGGL(apply_kernel, dim3(gx, N), dim3(kThreads), 0, st, P->pyr[s], hw, B, items, sums,
                           color[s], color_aug[s]);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
