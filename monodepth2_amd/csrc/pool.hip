// pool.hip — the ResNet stem's MaxPool2d(kernel 3, stride 2, padding 1)
// (torchvision ResNet behind networks/resnet_encoder.py:62-98) for NHWC activations
// on gfx950, fp32 or bf16 storage.
//
// Forward: one thread per (image, output pixel, channel quad): the max of the 3x3
// window (padding never wins), with PyTorch's rules — the first maximum in scan
// order wins ties, NaN propagates — and the winning window position (0..8) as one
// byte per value.  Backward: one thread per input quad gathers from the at most 4
// windows that contain it the gradients whose window picked it: a fixed-order sum, so
// deterministic (no atomics, unlike a scatter).

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "md2_bf16.h"
#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

constexpr int kThreads = 256;

struct PoolArgs {
    int B, H, W, C, Ho, Wo;
};

__device__ __forceinline__ void take(float v, int k, float& m, int& a) {
    if (v > m || isnan(v)) {   // ATen max_pool2d: strictly greater, or NaN
        m = v;
        a = k;
    }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) maxpool_fwd_kernel(PoolArgs p, const void* __restrict__ x,
                                                               void* __restrict__ y, uint32_t* __restrict__ idx) {
    const int C4 = p.C / 4;
    const int n = p.B * p.Ho * p.Wo * C4;   // < 2^31 (make()); 32-bit index math
    for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        const int c = 4 * (i % C4);
        int t = i / C4;
        const int ox = t % p.Wo;
        t /= p.Wo;
        const int oy = t % p.Ho;
        const int b = t / p.Ho;
        float m[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
        const int k0 = (oy == 0 ? 3 : 0) + (ox == 0 ? 1 : 0);   // first tap inside the image
        int a[4] = {k0, k0, k0, k0};
        for (int ky = 0; ky < 3; ++ky) {
            const int iy = 2 * oy - 1 + ky;
            if (iy < 0 || iy >= p.H) continue;
            for (int kx = 0; kx < 3; ++kx) {
                const int ix = 2 * ox - 1 + kx;
                if (ix < 0 || ix >= p.W) continue;
                const float4 v = md2::ld4T<T>(x, (((size_t)b * p.H + iy) * p.W + ix) * p.C + c);
                const int k = ky * 3 + kx;
                take(v.x, k, m[0], a[0]);
                take(v.y, k, m[1], a[1]);
                take(v.z, k, m[2], a[2]);
                take(v.w, k, m[3], a[3]);
            }
        }
        md2::st4T<T>(y, 4 * i, make_float4(m[0], m[1], m[2], m[3]));
        idx[i] = (uint32_t)a[0] | ((uint32_t)a[1] << 8) | ((uint32_t)a[2] << 16) | ((uint32_t)a[3] << 24);
    }
}

template <typename T>
__global__ void __launch_bounds__(kThreads) maxpool_bwd_kernel(PoolArgs p, const uint32_t* __restrict__ idx,
                                                               const void* __restrict__ gy, const void* __restrict__ gy2,
                                                               const void* __restrict__ ga, void* __restrict__ gx) {
    const int C4 = p.C / 4;
    const int n = p.B * p.H * p.W * C4;
    for (int i = blockIdx.x * kThreads + threadIdx.x; i < n; i += gridDim.x * kThreads) {
        const int c4 = i % C4;
        int t = i / C4;
        const int ix = t % p.W;
        t /= p.W;
        const int iy = t % p.H;
        const int b = t / p.H;
        float s[4] = {0.f, 0.f, 0.f, 0.f};
        // windows oy with 2*oy-1 <= iy <= 2*oy+1 (likewise x), in increasing order
        for (int oy = iy / 2; oy <= (iy + 1) / 2; ++oy) {
            if (oy < 0 || oy >= p.Ho || 2 * oy - 1 > iy || 2 * oy + 1 < iy) continue;
            for (int ox = ix / 2; ox <= (ix + 1) / 2; ++ox) {
                if (ox < 0 || ox >= p.Wo || 2 * ox - 1 > ix || 2 * ox + 1 < ix) continue;
                const size_t o = (((size_t)b * p.Ho + oy) * p.Wo + ox) * C4 + c4;
                const uint32_t w = idx[o];
                const int k = (iy - (2 * oy - 1)) * 3 + (ix - (2 * ox - 1));
                float4 g = md2::ld4T<T>(gy, 4 * o);
                if (gy2) {
                    const float4 h = md2::ld4T<T>(gy2, 4 * o);
                    g.x += h.x; g.y += h.y; g.z += h.z; g.w += h.w;
                }
                if ((int)(w & 255u) == k) s[0] += g.x;
                if ((int)((w >> 8) & 255u) == k) s[1] += g.y;
                if ((int)((w >> 16) & 255u) == k) s[2] += g.z;
                if ((int)(w >> 24) == k) s[3] += g.w;
            }
        }
        if (ga) {
            const float4 v = md2::ld4T<T>(ga, 4 * (size_t)i);
            s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
        }
        md2::st4T<T>(gx, 4 * i, make_float4(s[0], s[1], s[2], s[3]));
    }
}

// Same gather, one block row per input row (blockIdx.y = b·H + iy, decoded once per
// block) and C/4 a power of two: the per-element (ix, c4) split is a shift and a mask
// instead of six integer divisions (the kernel was VALU bound on them).
template <typename T>
__global__ void __launch_bounds__(kThreads) maxpool_bwd_rows_kernel(PoolArgs p, int c4_shift,
                                                                    const uint32_t* __restrict__ idx,
                                                                    const void* __restrict__ gy,
                                                                    const void* __restrict__ gy2,
                                                                    const void* __restrict__ ga, void* __restrict__ gx) {
    const int C4 = p.C / 4;
    const int j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= p.W * C4) return;
    const int row = blockIdx.y, b = row / p.H, iy = row - b * p.H;
    const int c4 = j & (C4 - 1), ix = j >> c4_shift;
    float s[4] = {0.f, 0.f, 0.f, 0.f};
    for (int oy = iy / 2; oy <= (iy + 1) / 2; ++oy) {
        if (oy >= p.Ho || 2 * oy - 1 > iy || 2 * oy + 1 < iy) continue;
        for (int ox = ix / 2; ox <= (ix + 1) / 2; ++ox) {
            if (ox >= p.Wo || 2 * ox - 1 > ix || 2 * ox + 1 < ix) continue;
            const size_t o = (((size_t)b * p.Ho + oy) * p.Wo + ox) * C4 + c4;
            const uint32_t w = idx[o];
            const int k = (iy - (2 * oy - 1)) * 3 + (ix - (2 * ox - 1));
            float4 g = md2::ld4T<T>(gy, 4 * o);
            if (gy2) {   // the pooled map's second consumer (the first block's shortcut)
                const float4 h = md2::ld4T<T>(gy2, 4 * o);
                g.x += h.x; g.y += h.y; g.z += h.z; g.w += h.w;
            }
            if ((int)(w & 255u) == k) s[0] += g.x;
            if ((int)((w >> 8) & 255u) == k) s[1] += g.y;
            if ((int)((w >> 16) & 255u) == k) s[2] += g.z;
            if ((int)(w >> 24) == k) s[3] += g.w;
        }
    }
    const size_t e = 4 * ((size_t)row * p.W * C4 + j);
    if (ga) {   // a second consumer's gradient of the pool input (the decoder skip)
        const float4 v = md2::ld4T<T>(ga, e);
        s[0] += v.x; s[1] += v.y; s[2] += v.z; s[3] += v.w;
    }
    md2::st4T<T>(gx, e, make_float4(s[0], s[1], s[2], s[3]));
}

// V channels per thread (V = 4: one float4 of fp32; V = 8: one 16-byte load of bf16 —
// the quad form moved 8 bytes per bf16 access and ran 2.5-4x its HBM bound at C5's
// batch).  Same per-element arithmetic and order as the quad kernels: bitwise equal.
template <typename T, int V>
__device__ __forceinline__ void ldV(const void* p, size_t off, float (&v)[V]) {
    if constexpr (V == 4) {
        const float4 q = md2::ld4T<T>(p, off);
        v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
    } else {
        static_assert(V == 8 && sizeof(T) == 2, "8 channels: bf16");
        const uint4 r = *(const uint4*)((const uint16_t*)p + off);
        const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = md2::bf2f(w[i] & 0xffffu);
            v[2 * i + 1] = md2::bf2f(w[i] >> 16);
        }
    }
}
template <typename T, int V>
__device__ __forceinline__ void stV(void* p, size_t off, const float (&v)[V]) {
    if constexpr (V == 4) {
        md2::st4T<T>(p, off, make_float4(v[0], v[1], v[2], v[3]));
    } else {
        *(uint4*)((uint16_t*)p + off) =
            make_uint4(md2::f2bf(v[0]) | (md2::f2bf(v[1]) << 16), md2::f2bf(v[2]) | (md2::f2bf(v[3]) << 16),
                       md2::f2bf(v[4]) | (md2::f2bf(v[5]) << 16), md2::f2bf(v[6]) | (md2::f2bf(v[7]) << 16));
    }
}

// Forward, one block row per output row (blockIdx.y = b·Ho + oy), C/V a power of two
template <typename T, int V>
__global__ void __launch_bounds__(kThreads) maxpool_fwd_rows_kernel(PoolArgs p, int cv_shift,
                                                                    const void* __restrict__ x,
                                                                    void* __restrict__ y, uint32_t* __restrict__ idx) {
    const int CV = p.C / V;
    const int j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= p.Wo * CV) return;
    const int row = blockIdx.y, b = row / p.Ho, oy = row - b * p.Ho;
    const int c = V * (j & (CV - 1)), ox = j >> cv_shift;
    float m[V];
    int a[V];
    const int k0 = (oy == 0 ? 3 : 0) + (ox == 0 ? 1 : 0);
#pragma unroll
    for (int i = 0; i < V; ++i) {
        m[i] = -INFINITY;
        a[i] = k0;
    }
    for (int ky = 0; ky < 3; ++ky) {
        const int iy = 2 * oy - 1 + ky;
        if (iy < 0 || iy >= p.H) continue;
        for (int kx = 0; kx < 3; ++kx) {
            const int ix = 2 * ox - 1 + kx;
            if (ix < 0 || ix >= p.W) continue;
            float v[V];
            ldV<T, V>(x, (((size_t)b * p.H + iy) * p.W + ix) * p.C + c, v);
            const int k = ky * 3 + kx;
#pragma unroll
            for (int i = 0; i < V; ++i) take(v[i], k, m[i], a[i]);
        }
    }
    const size_t o = (((size_t)b * p.Ho + oy) * p.Wo + ox) * p.C + c;
    stV<T, V>(y, o, m);
    if constexpr (V == 4) {
        idx[o / 4] = (uint32_t)a[0] | ((uint32_t)a[1] << 8) | ((uint32_t)a[2] << 16) | ((uint32_t)a[3] << 24);
    } else {
        *(uint2*)(idx + o / 4) =
            make_uint2((uint32_t)a[0] | ((uint32_t)a[1] << 8) | ((uint32_t)a[2] << 16) | ((uint32_t)a[3] << 24),
                       (uint32_t)a[4] | ((uint32_t)a[5] << 8) | ((uint32_t)a[6] << 16) | ((uint32_t)a[7] << 24));
    }
}

// Backward gather, V channels per thread (maxpool_bwd_rows_kernel at V = 8 for bf16)
template <typename T, int V>
__global__ void __launch_bounds__(kThreads) maxpool_bwd_rowsV_kernel(PoolArgs p, int cv_shift,
                                                                     const uint32_t* __restrict__ idx,
                                                                     const void* __restrict__ gy,
                                                                     const void* __restrict__ gy2,
                                                                     const void* __restrict__ ga, void* __restrict__ gx) {
    const int CV = p.C / V;
    const int j = blockIdx.x * kThreads + threadIdx.x;
    if (j >= p.W * CV) return;
    const int row = blockIdx.y, b = row / p.H, iy = row - b * p.H;
    const int c = V * (j & (CV - 1)), ix = j >> cv_shift;
    float s[V];
#pragma unroll
    for (int i = 0; i < V; ++i) s[i] = 0.f;
    for (int oy = iy / 2; oy <= (iy + 1) / 2; ++oy) {
        if (oy >= p.Ho || 2 * oy - 1 > iy || 2 * oy + 1 < iy) continue;
        for (int ox = ix / 2; ox <= (ix + 1) / 2; ++ox) {
            if (ox >= p.Wo || 2 * ox - 1 > ix || 2 * ox + 1 < ix) continue;
            const size_t o = (((size_t)b * p.Ho + oy) * p.Wo + ox) * p.C + c;
            uint32_t w[V / 4];
            if constexpr (V == 4) {
                w[0] = idx[o / 4];
            } else {
                const uint2 ww = *(const uint2*)(idx + o / 4);
                w[0] = ww.x;
                w[1] = ww.y;
            }
            const int k = (iy - (2 * oy - 1)) * 3 + (ix - (2 * ox - 1));
            float g[V];
            ldV<T, V>(gy, o, g);
            if (gy2) {
                float h[V];
                ldV<T, V>(gy2, o, h);
#pragma unroll
                for (int i = 0; i < V; ++i) g[i] += h[i];
            }
#pragma unroll
            for (int i = 0; i < V; ++i)
                if ((int)((w[i / 4] >> (8 * (i & 3))) & 255u) == k) s[i] += g[i];
        }
    }
    const size_t e = ((size_t)row * p.W + ix) * p.C + c;
    if (ga) {
        float v[V];
        ldV<T, V>(ga, e, v);
#pragma unroll
        for (int i = 0; i < V; ++i) s[i] += v[i];
    }
    stV<T, V>(gx, e, s);
}

// the row kernels' channel vector: 8 bf16 (16 bytes) where C allows, else a quad; 0 = none
int rows_vec(const md2_pool_desc* d, const PoolArgs& p, int rows) {
    static const bool v8 = [] {   // A/B knob: MD2_POOL_V8=0 keeps the bf16 quad kernels
        const char* e = getenv("MD2_POOL_V8");
        return !(e && e[0] == '0');
    }();
    const bool bf = (d->flags & MD2_POOL_BF16) != 0;
    const int V = (bf && v8 && p.C % 8 == 0) ? 8 : 4;
    const int CV = p.C / V;
    return ((CV & (CV - 1)) == 0 && rows <= 65535) ? V : 0;
}

int grid_for(long long n) {
    const long long g = (n + kThreads - 1) / kThreads;
    return (int)(g < 8192 ? g : 8192);
}

bool make(const md2_pool_desc* d, PoolArgs& p) {
    if (!d || d->batch < 1 || d->channels < 4 || d->channels % 4 || d->height < 1 || d->width < 1) return false;
    p.B = d->batch;
    p.C = d->channels;
    p.H = d->height;
    p.W = d->width;
    p.Ho = (d->height + 2 - 3) / 2 + 1;
    p.Wo = (d->width + 2 - 3) / 2 + 1;
    return (long long)p.B * p.H * p.W * (p.C / 4) < (1ll << 31);   // 32-bit quad indices
}

}  // namespace

extern "C" {

int md2_maxpool3s2_fwd(const md2_pool_desc* d, const void* x, void* y, uint32_t* idx, void* stream) {
    PoolArgs p;
    if (!make(d, p) || !x || !y || !idx) return md2_report_error(MD2_ERR_ARG, "maxpool: bad desc or NULL operand");
    const long long n = (long long)p.B * p.Ho * p.Wo * (p.C / 4);
    const bool bf = (d->flags & MD2_POOL_BF16) != 0;
    const int V = rows_vec(d, p, p.B * p.Ho);
    if (V == 8 || (V == 4 && bf)) {   // bf16; fp32 keeps the quad grid-stride kernel
        const int CV = p.C / V;
        int sh = 0;
        while ((1 << sh) < CV) ++sh;
        auto k = V == 8 ? maxpool_fwd_rows_kernel<uint16_t, 8> : maxpool_fwd_rows_kernel<uint16_t, 4>;
        hipLaunchKernelGGL(k, dim3((p.Wo * CV + kThreads - 1) / kThreads, p.B * p.Ho), dim3(kThreads), 0,
                           (hipStream_t)stream, p, sh, x, y, idx);
    } else {
        auto k = bf ? maxpool_fwd_kernel<uint16_t> : maxpool_fwd_kernel<float>;
        hipLaunchKernelGGL(k, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, p, x, y, idx);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_maxpool3s2_bwd_multi(const md2_pool_desc* d, const uint32_t* idx, const void* grad_y, const void* grad_y2,
                             const void* grad_add, void* grad_x, void* stream) {
    PoolArgs p;
    if (!make(d, p) || !idx || !grad_y || !grad_x)
        return md2_report_error(MD2_ERR_ARG, "maxpool: bad desc or NULL operand");
    const long long n = (long long)p.B * p.H * p.W * (p.C / 4);
    const int C4 = p.C / 4;
    if ((long long)p.B * p.H <= 65535 && rows_vec(d, p, p.B * p.H) == 8) {
        int sh = 0;
        while ((1 << sh) < p.C / 8) ++sh;
        hipLaunchKernelGGL((maxpool_bwd_rowsV_kernel<uint16_t, 8>), dim3((p.W * (p.C / 8) + kThreads - 1) / kThreads,
                           p.B * p.H), dim3(kThreads), 0, (hipStream_t)stream, p, sh, idx, grad_y, grad_y2, grad_add,
                           grad_x);
    } else if ((C4 & (C4 - 1)) == 0 && (long long)p.B * p.H <= 65535) {
        int sh = 0;
        while ((1 << sh) < C4) ++sh;
        auto k = (d->flags & MD2_POOL_BF16) ? maxpool_bwd_rows_kernel<uint16_t> : maxpool_bwd_rows_kernel<float>;
        hipLaunchKernelGGL(k, dim3((p.W * C4 + kThreads - 1) / kThreads, p.B * p.H), dim3(kThreads), 0,
                           (hipStream_t)stream, p, sh, idx, grad_y, grad_y2, grad_add, grad_x);
    } else {
        auto k = (d->flags & MD2_POOL_BF16) ? maxpool_bwd_kernel<uint16_t> : maxpool_bwd_kernel<float>;
        hipLaunchKernelGGL(k, dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, p, idx, grad_y, grad_y2,
                           grad_add, grad_x);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_maxpool3s2_bwd_add(const md2_pool_desc* d, const uint32_t* idx, const void* grad_y, const void* grad_add,
                           void* grad_x, void* stream) {
    return md2_maxpool3s2_bwd_multi(d, idx, grad_y, nullptr, grad_add, grad_x, stream);
}

int md2_maxpool3s2_bwd(const md2_pool_desc* d, const uint32_t* idx, const void* grad_y, void* grad_x, void* stream) {
    return md2_maxpool3s2_bwd_multi(d, idx, grad_y, nullptr, nullptr, grad_x, stream);
}

}  // extern "C"
