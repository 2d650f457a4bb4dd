// bnorm.hip — training-mode BatchNorm2d (+ residual add) (+ ReLU) for NHWC
// activations on gfx950.
//
// The ResNet encoders (networks/resnet_encoder.py -> torchvision BasicBlock /
// Bottleneck) run relu(bn(conv(x))) and relu(bn(conv(x)) + identity) about 60 times
// per training step (three encoders).  MIOpen's BatchNorm is three kernels each way,
// and the ReLU / residual add are separate passes over the same activation.  Here:
//
//   forward   bn_stats_kernel        per-block partial Σx, Σx² (float4 along C)
//             bn_stats_final_kernel  one block per channel: fixed-order double sums of
//                                    the partials -> saved mean / invstd, running
//                                    statistics (momentum, unbiased var, as nn.BatchNorm2d)
//             bn_apply_kernel        y = relu((x - mean)·invstd·γ + β [+ r])
//   backward  bn_bwd_reduce_kernel   g' = g·[y > 0]; partial Σg', Σg'·(x - mean)
//             bn_bwd_final_kernel    dγ, dβ and the dx coefficients, per channel
//             bn_bwd_apply_kernel    dx = γ·invstd·(g' - Σg'/N - x̂·Σg'x̂/N), d(residual) = g'
//
// Three launches each way, as MIOpen's BatchNorm, with the ReLU and the residual add
// folded into the passes.  (A single-pass "last block finalises" variant measured
// ~15 µs per layer on this chip: device-scope fences + ticket atomic + the finalising
// block's reads of the partials from memory form a serial chain.)
//
// Layout: x, y, r, g, dx, dr (N·H·W, C) fp32 — a channels_last NCHW tensor; C a
// multiple of 4 (every ResNet width is).  Deterministic: fixed-order reductions, no
// atomics.

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include "md2_bf16.h"
#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

constexpr int kThreads = 256;
constexpr int kMaxBlocks = 1024;   // partial rows per channel (the finalise reads them in parallel)

// thread -> (channel quad, pixel lane) mapping for C channels
struct Map {
    int Q;     // quads per pixel (C/4)
    int QPT;   // quads per thread (Q > 256 only)
    int PPB;   // pixels per block iteration
};

__host__ __device__ inline Map make_map(int C) {
    Map m;
    m.Q = C / 4;
    m.QPT = m.Q > kThreads ? m.Q / kThreads : 1;
    m.PPB = m.Q >= kThreads ? 1 : kThreads / m.Q;
    return m;
}

// workspace layout (floats): partial[2][C][NG*G] (channel-major: a channel's partials,
// row = group*G + block, contiguous for the finalising block's coalesced reads) |
// coef[3][NG][C]
struct Work {
    float* part;
    float* coef;
};

__host__ __device__ __forceinline__ Work work(void* ws, int G, int C, int NG) {
    Work w;
    w.part = (float*)ws;
    w.coef = w.part + 2 * (size_t)NG * G * C;
    return w;
}

__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ void st4(float* p, float4 v) { *(float4*)p = v; }

// Activation storage (fp32 or bf16): md2_bf16.h
template <typename T>
__device__ __forceinline__ float4 ldT(const void* p, size_t off) { return md2::ld4T<T>(p, off); }
template <typename T>
__device__ __forceinline__ void stT(void* p, size_t off, float4 v) { md2::st4T<T>(p, off, v); }

// Reduce the per-thread float4 pair over the PPB pixel lanes of the block (LDS tree)
// into the block's partial rows.  Ends with a barrier (LDS reused by the caller).
__device__ void block_partials(float4 a, float4 b, int q, int pl, const Map& m, int C, int rows, int row, Work w,
                               float4 (*lds)[kThreads]) {
    lds[0][threadIdx.x] = a;
    lds[1][threadIdx.x] = b;
    __syncthreads();
    for (int half = m.PPB / 2; half > 0; half /= 2) {   // PPB is a power of 2
        if (pl < half) {
            const int o = threadIdx.x + half * m.Q;
            const float4 u = lds[0][o], v = lds[1][o];
            a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
            b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
            lds[0][threadIdx.x] = a;
            lds[1][threadIdx.x] = b;
        }
        __syncthreads();
    }
    if (pl == 0) {
        float* pa = w.part + (size_t)(4 * q) * rows + row;
        float* pb = w.part + ((size_t)C + 4 * q) * rows + row;
        pa[0] = a.x; pa[rows] = a.y; pa[2 * (size_t)rows] = a.z; pa[3 * (size_t)rows] = a.w;
        pb[0] = b.x; pb[rows] = b.y; pb[2 * (size_t)rows] = b.z; pb[3 * (size_t)rows] = b.w;
    }
    __syncthreads();
}

// Per-channel Σx and Σx² partials of this block's pixels.
// Grouped BatchNorm (NG > 1): the pixels are NG equal contiguous groups (batch
// chunks), each normalised with its own statistics — what NG separate BatchNorm calls
// on the chunks compute.  P is the pixel count of one group; blockIdx.y the group.
template <typename T>
__global__ void __launch_bounds__(kThreads) bn_stats_kernel(const void* __restrict__ x, long long P, int C, int G,
                                                            void* ws) {
    const Map m = make_map(C);
    const int NG = gridDim.y, grp = blockIdx.y;
    const Work w = work(ws, G, C, NG);
    x = (const char*)x + (size_t)grp * P * C * sizeof(T);
    __shared__ float4 lds[2][kThreads];
    for (int qq = 0; qq < m.QPT; ++qq) {
        const int q = (threadIdx.x % m.Q) + qq * kThreads, pl = threadIdx.x / m.Q;
        float4 s = {0.f, 0.f, 0.f, 0.f}, ss = {0.f, 0.f, 0.f, 0.f};
        auto acc = [&](const float4 v) {
            s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
            ss.x += v.x * v.x; ss.y += v.y * v.y; ss.z += v.z * v.z; ss.w += v.w * v.w;
        };
        const long long stride = (long long)G * m.PPB;
        long long p = (long long)blockIdx.x * m.PPB + pl;
        for (; p + 3 * stride < P; p += 4 * stride) {   // four loads in flight per lane
            const float4 v0 = ldT<T>(x, p * C + 4 * q), v1 = ldT<T>(x, (p + stride) * C + 4 * q),
                         v2 = ldT<T>(x, (p + 2 * stride) * C + 4 * q), v3 = ldT<T>(x, (p + 3 * stride) * C + 4 * q);
            acc(v0); acc(v1); acc(v2); acc(v3);
        }
        for (; p < P; p += stride) acc(ldT<T>(x, p * C + 4 * q));
        block_partials(s, ss, q, pl, m, C, NG * G, grp * G + blockIdx.x, w, lds);
    }
}

// One block per channel: fixed-order double sums of its G partial pairs — thread t
// sums rows t, t + 256, ... in order, a fixed xor butterfly per wave, then the four wave
// sums in wave order (one barrier; an 8-level LDS tree cost ~1.5 us of the ~6 us
// launch, and a single wave per channel had too few loads in flight).  Returns the
// sums in thread 0.
__device__ bool channel_sums(Work w, int rows, int r0, int G, int C, int c, double& a, double& b) {
    __shared__ double red[2][kThreads / 64];
    // G <= kMaxBlocks = 4 x 256: all of a thread's (up to four) partial pairs are loaded
    // at once, coalesced (the channel's partials are contiguous), then added in row order
    static_assert(kMaxBlocks <= 4 * kThreads, "four partial rows per thread at most");
    const float* ca = w.part + (size_t)c * rows + r0;
    const float* cb = w.part + ((size_t)C + c) * rows + r0;
    float pa[4], pb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int g = threadIdx.x + u * kThreads;
        pa[u] = g < G ? ca[g] : 0.f;
        pb[u] = g < G ? cb[g] : 0.f;
    }
    a = 0.0;
    b = 0.0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        a += pa[u];
        b += pb[u];
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o, 64);
        b += __shfl_xor(b, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        red[0][threadIdx.x >> 6] = a;
        red[1][threadIdx.x >> 6] = b;
    }
    __syncthreads();
    a = red[0][0];
    b = red[1][0];
#pragma unroll
    for (int i = 1; i < kThreads / 64; ++i) {
        a += red[0][i];
        b += red[1][i];
    }
    __syncthreads();   // red is reused by the next group
    return threadIdx.x == 0;
}

// mean, 1/sqrt(var + eps), running statistics (nn.BatchNorm2d: momentum, unbiased var)
__global__ void __launch_bounds__(kThreads) bn_stats_final_kernel(long long P, int C, int G, int NG, float eps,
                                                                  float momentum, float* __restrict__ rmean,
                                                                  float* __restrict__ rvar,
                                                                  float* __restrict__ smean,
                                                                  float* __restrict__ sinvstd, void* ws) {
    const int c = blockIdx.x;
    const Work w = work(ws, G, C, NG);
    for (int grp = 0; grp < NG; ++grp) {   // groups in order: the running statistics update as NG calls
        double a, b;
        if (!channel_sums(w, NG * G, grp * G, G, C, c, a, b)) continue;
        const double mean = a / (double)P;
        double var = b / (double)P - mean * mean;
        var = var > 0.0 ? var : 0.0;
        smean[grp * C + c] = (float)mean;
        sinvstd[grp * C + c] = (float)(1.0 / sqrt(var + (double)eps));
        if (rmean) {
            rmean[c] = (float)((1.0 - momentum) * rmean[c] + momentum * mean);
            rvar[c] = (float)((1.0 - momentum) * rvar[c] + momentum * var * (double)P / (double)(P - 1));
        }
    }
}

// Elementwise passes: blockIdx.y = BatchNorm group, 32-bit quad index inside the group
// (valid() bounds it), channel quad = index & (Q - 1) (Q a power of two) — no 64-bit
// division or modulo per element.
// y > 0 as stored (a bf16 y is compared after rounding, as the backward would read it)
template <typename T>
__device__ __forceinline__ bool stored_pos(float o) {
    if constexpr (sizeof(T) == 4) return o > 0.f;
    else return md2::bf2f(md2::f2bf(o)) > 0.f;
}

// ReLU mask (MOUT): one byte per element quad, bit i = (y[4 i' + i] > 0) — what the
// backward needs of y, at 1/16 (fp32) or 1/8 (bf16) of its bytes
template <typename T, bool RELU, bool RES, bool MOUT = false>
__global__ void __launch_bounds__(kThreads) bn_apply_kernel(const void* __restrict__ x, const void* __restrict__ r,
                                                            const float* __restrict__ gamma,
                                                            const float* __restrict__ beta,
                                                            const float* __restrict__ smean,
                                                            const float* __restrict__ sinvstd, void* __restrict__ y,
                                                            int n4g, int Q, uint8_t* __restrict__ mask = nullptr) {
    const size_t base = (size_t)blockIdx.y * n4g;   // this group's first quad
    const float* mug = smean + (size_t)blockIdx.y * 4 * Q;
    const float* isg = sinvstd + (size_t)blockIdx.y * 4 * Q;
    for (int j = blockIdx.x * kThreads + threadIdx.x; j < n4g; j += gridDim.x * kThreads) {
        const size_t i = base + j;
        const int c = 4 * (j & (Q - 1));
        const float4 v = ldT<T>(x, 4 * i), mu = ld4(mug + c), is = ld4(isg + c), ga = ld4(gamma + c),
                     be = ld4(beta + c);
        float4 o;
        o.x = (v.x - mu.x) * is.x * ga.x + be.x;
        o.y = (v.y - mu.y) * is.y * ga.y + be.y;
        o.z = (v.z - mu.z) * is.z * ga.z + be.z;
        o.w = (v.w - mu.w) * is.w * ga.w + be.w;
        if (RES) {
            const float4 rv = ldT<T>(r, 4 * i);
            o.x += rv.x; o.y += rv.y; o.z += rv.z; o.w += rv.w;
        }
        if (RELU) {
            o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
        }
        stT<T>(y, 4 * i, o);
        if (MOUT)
            mask[i] = (uint8_t)((stored_pos<T>(o.x) ? 1 : 0) | (stored_pos<T>(o.y) ? 2 : 0) |
                                (stored_pos<T>(o.z) ? 4 : 0) | (stored_pos<T>(o.w) ? 8 : 0));
    }
}

// the ReLU gate of the backward from y (fp32 / bf16) or from the forward's mask byte
template <typename T, bool MIN>
__device__ __forceinline__ float4 relu_gate(const void* y, size_t off, float4 g) {
    if constexpr (MIN) {
        const uint32_t m = ((const uint8_t*)y)[off >> 2];
        g.x = (m & 1) ? g.x : 0.f; g.y = (m & 2) ? g.y : 0.f; g.z = (m & 4) ? g.z : 0.f; g.w = (m & 8) ? g.w : 0.f;
    } else {
        const float4 yv = ldT<T>(y, off);
        g.x = yv.x > 0.f ? g.x : 0.f; g.y = yv.y > 0.f ? g.y : 0.f;
        g.z = yv.z > 0.f ? g.z : 0.f; g.w = yv.w > 0.f ? g.w : 0.f;
    }
    return g;
}

// the output gradient: g (+ g2 + g3, the gradients of the output's aliases — its
// other consumers, summed here instead of by separate add passes)
template <typename T>
__device__ __forceinline__ float4 ld_grad(const void* g, const void* g2, const void* g3, size_t off) {
    float4 v = ldT<T>(g, off);
    if (g2) {
        const float4 u = ldT<T>(g2, off);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    if (g3) {
        const float4 u = ldT<T>(g3, off);
        v.x += u.x; v.y += u.y; v.z += u.z; v.w += u.w;
    }
    return v;
}

template <typename T, bool RELU, bool MIN = false>
__global__ void __launch_bounds__(kThreads) bn_bwd_reduce_kernel(const void* __restrict__ x,
                                                                 const void* __restrict__ y,
                                                                 const void* __restrict__ g,
                                                                 const void* __restrict__ g2,
                                                                 const void* __restrict__ g3, long long P, int C,
                                                                 int G, const float* __restrict__ smean, void* ws) {
    const Map m = make_map(C);
    const int NG = gridDim.y, grp = blockIdx.y;
    const Work w = work(ws, G, C, NG);
    const size_t base = (size_t)grp * P * C;   // this group's first element
    __shared__ float4 lds[2][kThreads];
    for (int qq = 0; qq < m.QPT; ++qq) {
        const int q = (threadIdx.x % m.Q) + qq * kThreads, pl = threadIdx.x / m.Q;
        const float4 mu = ld4(smean + grp * C + 4 * q);
        float4 s = {0.f, 0.f, 0.f, 0.f}, sx = {0.f, 0.f, 0.f, 0.f};
        auto acc = [&](float4 gv, const float4 v) {   // gv already ReLU-gated
            s.x += gv.x; s.y += gv.y; s.z += gv.z; s.w += gv.w;
            sx.x += gv.x * (v.x - mu.x); sx.y += gv.y * (v.y - mu.y);
            sx.z += gv.z * (v.z - mu.z); sx.w += gv.w * (v.w - mu.w);
        };
        const long long stride = (long long)G * m.PPB;
        long long p = (long long)blockIdx.x * m.PPB + pl;
        for (; p + stride < P; p += 2 * stride) {   // two pixels (up to six loads) in flight per lane
            const size_t o0 = base + p * C + 4 * q, o1 = base + (p + stride) * C + 4 * q;
            float4 g0 = ld_grad<T>(g, g2, g3, o0), g1 = ld_grad<T>(g, g2, g3, o1);
            if (RELU) {
                g0 = relu_gate<T, MIN>(y, o0, g0);
                g1 = relu_gate<T, MIN>(y, o1, g1);
            }
            const float4 v0 = ldT<T>(x, o0), v1 = ldT<T>(x, o1);
            acc(g0, v0);
            acc(g1, v1);
        }
        for (; p < P; p += stride) {
            const size_t o = base + p * C + 4 * q;
            float4 gv = ld_grad<T>(g, g2, g3, o);
            if (RELU) gv = relu_gate<T, MIN>(y, o, gv);
            acc(gv, ldT<T>(x, o));
        }
        block_partials(s, sx, q, pl, m, C, NG * G, grp * G + blockIdx.x, w, lds);
    }
}

// dγ = Σg'x̂, dβ = Σg' and the dx coefficients, one block per channel
__global__ void __launch_bounds__(kThreads) bn_bwd_final_kernel(long long P, int C, int G, int NG,
                                                                const float* __restrict__ gamma,
                                                                const float* __restrict__ sinvstd,
                                                                float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                void* ws) {
    const int c = blockIdx.x;
    const Work w = work(ws, G, C, NG);
    double sdg = 0.0, sdb = 0.0;   // parameter gradients: sum over the groups in order
    for (int grp = 0; grp < NG; ++grp) {
        double a, b;
        if (!channel_sums(w, NG * G, grp * G, G, C, c, a, b)) continue;
        const double is = sinvstd[grp * C + c];
        const double dg = b * is;   // Σ g'·x̂
        sdg += dg;
        sdb += a;
        const size_t gc = (size_t)grp * C + c;
        w.coef[gc] = (float)((double)gamma[c] * is);                     // γ·invstd
        w.coef[(size_t)NG * C + gc] = (float)(a / (double)P);            // Σg'/N
        w.coef[2 * (size_t)NG * C + gc] = (float)(dg * is / (double)P);  // Σg'x̂/N · invstd
    }
    if (threadIdx.x == 0) {
        dgamma[c] = (float)sdg;
        dbeta[c] = (float)sdb;
    }
}

template <typename T, bool RELU, bool RES, bool MIN = false>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply_kernel(const void* __restrict__ x,
                                                                const void* __restrict__ y,
                                                                const void* __restrict__ g,
                                                                const void* __restrict__ g2,
                                                                const void* __restrict__ g3,
                                                                const float* __restrict__ smean, const float* coef,
                                                                void* __restrict__ dx, void* __restrict__ dr,
                                                                int n4g, int Q, int C, int NG) {
    const size_t base = (size_t)blockIdx.y * n4g;
    const size_t gc = (size_t)blockIdx.y * C;   // group * C
    for (int j = blockIdx.x * kThreads + threadIdx.x; j < n4g; j += gridDim.x * kThreads) {
        const size_t i = base + j;
        const size_t c = gc + 4 * (j & (Q - 1));
        float4 gv = ld_grad<T>(g, g2, g3, 4 * i);
        if (RELU) gv = relu_gate<T, MIN>(y, 4 * i, gv);
        const float4 v = ldT<T>(x, 4 * i), mu = ld4(smean + c), k1 = ld4(coef + c),
                     k2 = ld4(coef + (size_t)NG * C + c), k3 = ld4(coef + 2 * (size_t)NG * C + c);
        float4 o;
        o.x = k1.x * (gv.x - k2.x - (v.x - mu.x) * k3.x);
        o.y = k1.y * (gv.y - k2.y - (v.y - mu.y) * k3.y);
        o.z = k1.z * (gv.z - k2.z - (v.z - mu.z) * k3.z);
        o.w = k1.w * (gv.w - k2.w - (v.w - mu.w) * k3.w);
        stT<T>(dx, 4 * i, o);
        if (RES) stT<T>(dr, 4 * i, gv);
    }
}

// bf16 elementwise passes on eight channels (one 16-byte access) per thread: the quad
// kernels moved 8 bytes per bf16 access (1.5-1.8x the fp32 kernels' time at C5's batch
// for ~1.3x the bytes).  Per-element arithmetic as the quad kernels: bitwise equal.
// The ReLU mask keeps its layout (one byte per quad): two bytes per thread.
__device__ __forceinline__ void ld8bf(const void* p, size_t off, float (&v)[8]) {
    const uint4 r = *(const uint4*)((const uint16_t*)p + off);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = md2::bf2f(w[i] & 0xffffu);
        v[2 * i + 1] = md2::bf2f(w[i] >> 16);
    }
}
__device__ __forceinline__ void st8bf(void* p, size_t off, const float (&v)[8]) {
    *(uint4*)((uint16_t*)p + off) =
        make_uint4(md2::f2bf(v[0]) | (md2::f2bf(v[1]) << 16), md2::f2bf(v[2]) | (md2::f2bf(v[3]) << 16),
                   md2::f2bf(v[4]) | (md2::f2bf(v[5]) << 16), md2::f2bf(v[6]) | (md2::f2bf(v[7]) << 16));
}
__device__ __forceinline__ void ld8f(const float* p, float (&v)[8]) {
    const float4 a = ld4(p), b = ld4(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <bool RELU, bool RES, bool MOUT = false>
__global__ void __launch_bounds__(kThreads) bn_apply8_kernel(const void* __restrict__ x, const void* __restrict__ r,
                                                             const float* __restrict__ gamma,
                                                             const float* __restrict__ beta,
                                                             const float* __restrict__ smean,
                                                             const float* __restrict__ sinvstd, void* __restrict__ y,
                                                             int n8g, int Q8, uint8_t* __restrict__ mask = nullptr) {
    const size_t base = (size_t)blockIdx.y * n8g;
    const float* mug = smean + (size_t)blockIdx.y * 8 * Q8;
    const float* isg = sinvstd + (size_t)blockIdx.y * 8 * Q8;
    for (int j = blockIdx.x * kThreads + threadIdx.x; j < n8g; j += gridDim.x * kThreads) {
        const size_t i = base + j;
        const int c = 8 * (j & (Q8 - 1));
        float v[8], mu[8], is[8], ga[8], be[8], o[8];
        ld8bf(x, 8 * i, v);
        ld8f(mug + c, mu);
        ld8f(isg + c, is);
        ld8f(gamma + c, ga);
        ld8f(beta + c, be);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[e] - mu[e]) * is[e] * ga[e] + be[e];
        if (RES) {
            float rv[8];
            ld8bf(r, 8 * i, rv);
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] += rv[e];
        }
        if (RELU) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = fmaxf(o[e], 0.f);
        }
        st8bf(y, 8 * i, o);
        if (MOUT) {
            uint32_t m = 0;
#pragma unroll
            for (int e = 0; e < 8; ++e) m |= (stored_pos<uint16_t>(o[e]) ? 1u : 0u) << ((e & 3) + 8 * (e >> 2));
            ((uint16_t*)mask)[i] = (uint16_t)m;
        }
    }
}

template <bool RELU, bool RES, bool MIN = false>
__global__ void __launch_bounds__(kThreads) bn_bwd_apply8_kernel(const void* __restrict__ x,
                                                                 const void* __restrict__ y,
                                                                 const void* __restrict__ g,
                                                                 const void* __restrict__ g2,
                                                                 const void* __restrict__ g3,
                                                                 const float* __restrict__ smean, const float* coef,
                                                                 void* __restrict__ dx, void* __restrict__ dr,
                                                                 int n8g, int Q8, int C, int NG) {
    const size_t base = (size_t)blockIdx.y * n8g;
    const size_t gc = (size_t)blockIdx.y * C;
    for (int j = blockIdx.x * kThreads + threadIdx.x; j < n8g; j += gridDim.x * kThreads) {
        const size_t i = base + j;
        const size_t c = gc + 8 * (j & (Q8 - 1));
        float gv[8];
        ld8bf(g, 8 * i, gv);
        if (g2) {
            float u[8];
            ld8bf(g2, 8 * i, u);
#pragma unroll
            for (int e = 0; e < 8; ++e) gv[e] += u[e];
        }
        if (g3) {
            float u[8];
            ld8bf(g3, 8 * i, u);
#pragma unroll
            for (int e = 0; e < 8; ++e) gv[e] += u[e];
        }
        if (RELU) {
            if constexpr (MIN) {
                const uint32_t m = ((const uint16_t*)y)[i];
#pragma unroll
                for (int e = 0; e < 8; ++e) gv[e] = ((m >> ((e & 3) + 8 * (e >> 2))) & 1u) ? gv[e] : 0.f;
            } else {
                float yv[8];
                ld8bf(y, 8 * i, yv);
#pragma unroll
                for (int e = 0; e < 8; ++e) gv[e] = yv[e] > 0.f ? gv[e] : 0.f;
            }
        }
        float v[8], mu[8], k1[8], k2[8], k3[8], o[8];
        ld8bf(x, 8 * i, v);
        ld8f(smean + c, mu);
        ld8f(coef + c, k1);
        ld8f(coef + (size_t)NG * C + c, k2);
        ld8f(coef + 2 * (size_t)NG * C + c, k3);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = k1[e] * (gv[e] - k2[e] - (v[e] - mu[e]) * k3[e]);
        st8bf(dx, 8 * i, o);
        if (RES) st8bf(dr, 8 * i, gv);
    }
}

// The two reductions on eight channels per thread as well (bf16): Σx, Σx² and Σg', Σg'(x-μ)
// per channel with the same block partial rows (two block_partials calls, one per
// channel quad of the octet) — a different fixed order than the quad kernels (fp32
// partials of twice as many pixels per block step), equally deterministic.
template <bool UNUSED = false>
__global__ void __launch_bounds__(kThreads) bn_stats8_kernel(const void* __restrict__ x, long long P, int C, int G,
                                                             void* ws) {
    const int Q8 = C / 8;
    const Map m8 = {Q8, 1, kThreads / Q8};
    const int NG = gridDim.y, grp = blockIdx.y;
    const Work w = work(ws, G, C, NG);
    x = (const char*)x + (size_t)grp * P * C * 2;
    __shared__ float4 lds[2][kThreads];
    const int q8 = threadIdx.x % Q8, pl = threadIdx.x / Q8;
    float v[8], s[8], ss[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = ss[e] = 0.f;
    auto acc = [&]() {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            s[e] += v[e];
            ss[e] += v[e] * v[e];
        }
    };
    const long long stride = (long long)G * m8.PPB;
    for (long long p = (long long)blockIdx.x * m8.PPB + pl; p < P; p += stride) {
        ld8bf(x, p * C + 8 * q8, v);
        acc();
    }
    block_partials(make_float4(s[0], s[1], s[2], s[3]), make_float4(ss[0], ss[1], ss[2], ss[3]), 2 * q8, pl, m8, C,
                   NG * G, grp * G + blockIdx.x, w, lds);
    block_partials(make_float4(s[4], s[5], s[6], s[7]), make_float4(ss[4], ss[5], ss[6], ss[7]), 2 * q8 + 1, pl, m8,
                   C, NG * G, grp * G + blockIdx.x, w, lds);
}

template <bool RELU, bool MIN = false>
__global__ void __launch_bounds__(kThreads) bn_bwd_reduce8_kernel(const void* __restrict__ x,
                                                                  const void* __restrict__ y,
                                                                  const void* __restrict__ g,
                                                                  const void* __restrict__ g2,
                                                                  const void* __restrict__ g3, long long P, int C,
                                                                  int G, const float* __restrict__ smean, void* ws) {
    const int Q8 = C / 8;
    const Map m8 = {Q8, 1, kThreads / Q8};
    const int NG = gridDim.y, grp = blockIdx.y;
    const Work w = work(ws, G, C, NG);
    const size_t base = (size_t)grp * P * C;
    __shared__ float4 lds[2][kThreads];
    const int q8 = threadIdx.x % Q8, pl = threadIdx.x / Q8;
    float mu[8], s[8], sx[8];
    ld8f(smean + grp * C + 8 * q8, mu);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = sx[e] = 0.f;
    const long long stride = (long long)G * m8.PPB;
    for (long long p = (long long)blockIdx.x * m8.PPB + pl; p < P; p += stride) {
        const size_t o = base + p * C + 8 * q8;   // element offset; o / 8 = octet index
        float gv[8], v[8];
        ld8bf(g, o, gv);
        if (g2) {
            float u[8];
            ld8bf(g2, o, u);
#pragma unroll
            for (int e = 0; e < 8; ++e) gv[e] += u[e];
        }
        if (g3) {
            float u[8];
            ld8bf(g3, o, u);
#pragma unroll
            for (int e = 0; e < 8; ++e) gv[e] += u[e];
        }
        if (RELU) {
            if constexpr (MIN) {
                const uint32_t m = ((const uint16_t*)y)[o / 8];
#pragma unroll
                for (int e = 0; e < 8; ++e) gv[e] = ((m >> ((e & 3) + 8 * (e >> 2))) & 1u) ? gv[e] : 0.f;
            } else {
                float yv[8];
                ld8bf(y, o, yv);
#pragma unroll
                for (int e = 0; e < 8; ++e) gv[e] = yv[e] > 0.f ? gv[e] : 0.f;
            }
        }
        ld8bf(x, o, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            s[e] += gv[e];
            sx[e] += gv[e] * (v[e] - mu[e]);
        }
    }
    block_partials(make_float4(s[0], s[1], s[2], s[3]), make_float4(sx[0], sx[1], sx[2], sx[3]), 2 * q8, pl, m8, C,
                   NG * G, grp * G + blockIdx.x, w, lds);
    block_partials(make_float4(s[4], s[5], s[6], s[7]), make_float4(sx[4], sx[5], sx[6], sx[7]), 2 * q8 + 1, pl, m8,
                   C, NG * G, grp * G + blockIdx.x, w, lds);
}

bool reduce8_on() {   // A/B knob: MD2_BN_RED8=0 keeps the bf16 quad reductions
    static const bool on = [] {
        const char* e = getenv("MD2_BN_RED8");
        return !(e && e[0] == '0');
    }();
    return on;
}

bool apply8_on() {   // A/B knob: MD2_BN_V8=0 keeps the bf16 quad elementwise kernels
    static const bool on = [] {
        const char* e = getenv("MD2_BN_V8");
        return !(e && e[0] == '0');
    }();
    return on;
}

int blocks_for_stats(long long P, int C) {
    const Map m = make_map(C);
    const long long rows = (P + m.PPB - 1) / m.PPB;
    const long long g = (rows + 7) / 8;   // about 8 pixel steps per lane
    return (int)(g < 1 ? 1 : (g > kMaxBlocks ? kMaxBlocks : g));
}

int grid_elem(long long n4, int NG) {   // blocks per group (about 4096 in all)
    const long long cap = (4096 + NG - 1) / NG;
    const long long g = (n4 + kThreads - 1) / kThreads;
    return (int)(g < cap ? g : cap);
}

int groups_of(const md2_bn_desc* d) { return d->groups > 1 ? d->groups : 1; }

bool valid(const md2_bn_desc* d) {
    if (!d || d->channels < 4 || d->channels % 4) return false;
    if (d->groups < 0 || d->pixels % groups_of(d) || d->pixels / groups_of(d) < 2) return false;
    const int Q = d->channels / 4;
    if ((Q & (Q - 1)) != 0) return false;   // channel quads a power of two (every ResNet width)
    if ((long long)d->pixels / groups_of(d) * Q >= (1ll << 31)) return false;   // 32-bit quad index per group
    return Q >= kThreads ? (Q % kThreads == 0) : (kThreads % Q == 0);
}

template <typename T>
void launch_fwd(const md2_bn_desc* d, const void* x, const float* gamma, const float* beta, const void* residual,
                float* running_mean, float* running_var, void* y, float* save_mean, float* save_invstd,
                void* workspace, hipStream_t st, uint8_t* mask = nullptr) {
    const int NG = groups_of(d);
    const long long P = d->pixels / NG;   // per group
    const int C = d->channels, G = blocks_for_stats(P, C);
    if (sizeof(T) == 2 && C % 8 == 0 && C <= 8 * kThreads && reduce8_on())
        hipLaunchKernelGGL(bn_stats8_kernel<>, dim3(G, NG), dim3(kThreads), 0, st, x, P, C, G, workspace);
    else
        hipLaunchKernelGGL(bn_stats_kernel<T>, dim3(G, NG), dim3(kThreads), 0, st, x, P, C, G, workspace);
    hipLaunchKernelGGL(bn_stats_final_kernel, dim3(C), dim3(kThreads), 0, st, P, C, G, NG, d->eps, d->momentum,
                       running_mean, running_var, save_mean, save_invstd, workspace);
    const int n4g = (int)(P * C / 4);
    const bool relu = d->flags & MD2_BN_RELU, res = d->flags & MD2_BN_RESIDUAL;
    if (sizeof(T) == 2 && C % 8 == 0 && apply8_on()) {
        auto k8 = relu ? (mask ? (res ? bn_apply8_kernel<true, true, true> : bn_apply8_kernel<true, false, true>)
                               : (res ? bn_apply8_kernel<true, true> : bn_apply8_kernel<true, false>))
                       : (res ? bn_apply8_kernel<false, true> : bn_apply8_kernel<false, false>);
        hipLaunchKernelGGL(k8, dim3(grid_elem(n4g / 2, NG), NG), dim3(kThreads), 0, st, x, residual, gamma, beta,
                           save_mean, save_invstd, y, n4g / 2, C / 8, mask);
        return;
    }
    auto k = relu ? (mask ? (res ? bn_apply_kernel<T, true, true, true> : bn_apply_kernel<T, true, false, true>)
                          : (res ? bn_apply_kernel<T, true, true> : bn_apply_kernel<T, true, false>))
                  : (res ? bn_apply_kernel<T, false, true> : bn_apply_kernel<T, false, false>);
    hipLaunchKernelGGL(k, dim3(grid_elem(n4g, NG), NG), dim3(kThreads), 0, st, x, residual, gamma, beta, save_mean,
                       save_invstd, y, n4g, C / 4, mask);
}

template <typename T>
void launch_bwd(const md2_bn_desc* d, const void* x, const void* y, const void* grad_y, const void* grad_y2,
                const void* grad_y3, const float* gamma,
                const float* save_mean, const float* save_invstd, void* grad_x, void* grad_residual,
                float* grad_gamma, float* grad_beta, void* workspace, hipStream_t st, bool mask_in = false) {
    const int NG = groups_of(d);
    const long long P = d->pixels / NG;
    const int C = d->channels, G = blocks_for_stats(P, C);
    const bool relu = d->flags & MD2_BN_RELU, res = d->flags & MD2_BN_RESIDUAL;
    // mask_in: y is the forward's ReLU mask (one byte per element quad), not y itself
    auto red = relu ? (mask_in ? bn_bwd_reduce_kernel<T, true, true> : bn_bwd_reduce_kernel<T, true>)
                    : bn_bwd_reduce_kernel<T, false>;
    if (sizeof(T) == 2 && C % 8 == 0 && C <= 8 * kThreads && reduce8_on())
        red = relu ? (mask_in ? bn_bwd_reduce8_kernel<true, true> : bn_bwd_reduce8_kernel<true>)
                   : bn_bwd_reduce8_kernel<false>;
    hipLaunchKernelGGL(red, dim3(G, NG), dim3(kThreads), 0, st, x, y, grad_y, grad_y2, grad_y3, P, C, G, save_mean,
                       workspace);
    hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(C), dim3(kThreads), 0, st, P, C, G, NG, gamma, save_invstd,
                       grad_gamma, grad_beta, workspace);
    const int n4g = (int)(P * C / 4);
    const float* coef = work(workspace, G, C, NG).coef;
    if (sizeof(T) == 2 && C % 8 == 0 && apply8_on()) {
        auto k8 = relu ? (mask_in ? (res ? bn_bwd_apply8_kernel<true, true, true> : bn_bwd_apply8_kernel<true, false, true>)
                                  : (res ? bn_bwd_apply8_kernel<true, true> : bn_bwd_apply8_kernel<true, false>))
                       : (res ? bn_bwd_apply8_kernel<false, true> : bn_bwd_apply8_kernel<false, false>);
        hipLaunchKernelGGL(k8, dim3(grid_elem(n4g / 2, NG), NG), dim3(kThreads), 0, st, x, y, grad_y, grad_y2,
                           grad_y3, save_mean, coef, grad_x, grad_residual, n4g / 2, C / 8, C, NG);
        return;
    }
    auto k = relu ? (mask_in ? (res ? bn_bwd_apply_kernel<T, true, true, true> : bn_bwd_apply_kernel<T, true, false, true>)
                             : (res ? bn_bwd_apply_kernel<T, true, true> : bn_bwd_apply_kernel<T, true, false>))
                  : (res ? bn_bwd_apply_kernel<T, false, true> : bn_bwd_apply_kernel<T, false, false>);
    hipLaunchKernelGGL(k, dim3(grid_elem(n4g, NG), NG), dim3(kThreads), 0, st, x, y, grad_y, grad_y2, grad_y3,
                       save_mean, coef, grad_x, grad_residual, n4g, C / 4, C, NG);
}

}  // namespace

extern "C" {

size_t md2_bn_workspace_bytes(const md2_bn_desc* d) {
    if (!valid(d)) return 0;
    const int NG = groups_of(d);
    const int G = blocks_for_stats(d->pixels / NG, d->channels);
    return (2 * (size_t)NG * G * d->channels + 3 * (size_t)NG * d->channels) * sizeof(float);
}

int md2_bn_fwd_mask(const md2_bn_desc* d, const void* x, const float* gamma, const float* beta, const void* residual,
                    float* running_mean, float* running_var, void* y, uint8_t* relu_mask, float* save_mean,
                    float* save_invstd, void* workspace, void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "bn: need pixels >= 2 and channels a multiple of 4 "
                                                        "with channels/4 dividing (or a multiple of) 256");
    if (!x || !gamma || !beta || !y || !save_mean || !save_invstd || !workspace ||
        ((d->flags & MD2_BN_RESIDUAL) && !residual) || (!running_mean != !running_var))
        return md2_report_error(MD2_ERR_ARG, "bn_fwd: NULL operand");
    if (relu_mask && !(d->flags & MD2_BN_RELU)) return md2_report_error(MD2_ERR_ARG, "bn_fwd: relu_mask without MD2_BN_RELU");
    if (d->flags & MD2_BN_BF16)
        launch_fwd<uint16_t>(d, x, gamma, beta, residual, running_mean, running_var, y, save_mean, save_invstd,
                             workspace, (hipStream_t)stream, relu_mask);
    else
        launch_fwd<float>(d, x, gamma, beta, residual, running_mean, running_var, y, save_mean, save_invstd,
                          workspace, (hipStream_t)stream, relu_mask);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_bn_fwd(const md2_bn_desc* d, const void* x, const float* gamma, const float* beta, const void* residual,
               float* running_mean, float* running_var, void* y, float* save_mean, float* save_invstd,
               void* workspace, void* stream) {
    return md2_bn_fwd_mask(d, x, gamma, beta, residual, running_mean, running_var, y, nullptr, save_mean, save_invstd,
                           workspace, stream);
}

static int bn_bwd_impl(const md2_bn_desc* d, const void* x, const void* y, bool mask_in, const void* grad_y,
                       const void* grad_y2, const void* grad_y3, const float* gamma, const float* save_mean,
                       const float* save_invstd, void* grad_x, void* grad_residual, float* grad_gamma,
                       float* grad_beta, void* workspace, void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "bn: unsupported shape");
    const bool relu = d->flags & MD2_BN_RELU, res = d->flags & MD2_BN_RESIDUAL;
    if (!x || !grad_y || !gamma || !save_mean || !save_invstd || !grad_x || !grad_gamma || !grad_beta ||
        !workspace || (relu && !y) || (res && !grad_residual) || (grad_y3 && !grad_y2))
        return md2_report_error(MD2_ERR_ARG, "bn_bwd: NULL operand");
    if (d->flags & MD2_BN_BF16)
        launch_bwd<uint16_t>(d, x, y, grad_y, grad_y2, grad_y3, gamma, save_mean, save_invstd, grad_x,
                             grad_residual, grad_gamma, grad_beta, workspace, (hipStream_t)stream, mask_in);
    else
        launch_bwd<float>(d, x, y, grad_y, grad_y2, grad_y3, gamma, save_mean, save_invstd, grad_x, grad_residual,
                          grad_gamma, grad_beta, workspace, (hipStream_t)stream, mask_in);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_bn_bwd_multi(const md2_bn_desc* d, const void* x, const void* y, const void* grad_y, const void* grad_y2,
                     const void* grad_y3, const float* gamma, const float* save_mean, const float* save_invstd,
                     void* grad_x, void* grad_residual, float* grad_gamma, float* grad_beta, void* workspace,
                     void* stream) {
    return bn_bwd_impl(d, x, y, false, grad_y, grad_y2, grad_y3, gamma, save_mean, save_invstd, grad_x, grad_residual,
                       grad_gamma, grad_beta, workspace, stream);
}

int md2_bn_bwd_mask(const md2_bn_desc* d, const void* x, const uint8_t* relu_mask, const void* grad_y,
                    const void* grad_y2, const void* grad_y3, const float* gamma, const float* save_mean,
                    const float* save_invstd, void* grad_x, void* grad_residual, float* grad_gamma, float* grad_beta,
                    void* workspace, void* stream) {
    if (!(d && (d->flags & MD2_BN_RELU))) return md2_report_error(MD2_ERR_ARG, "bn_bwd_mask: needs MD2_BN_RELU");
    return bn_bwd_impl(d, x, relu_mask, true, grad_y, grad_y2, grad_y3, gamma, save_mean, save_invstd, grad_x,
                       grad_residual, grad_gamma, grad_beta, workspace, stream);
}

int md2_bn_bwd(const md2_bn_desc* d, const void* x, const void* y, const void* grad_y, const float* gamma,
               const float* save_mean, const float* save_invstd, void* grad_x, void* grad_residual,
               float* grad_gamma, float* grad_beta, void* workspace, void* stream) {
    return md2_bn_bwd_multi(d, x, y, grad_y, nullptr, nullptr, gamma, save_mean, save_invstd, grad_x, grad_residual,
                            grad_gamma, grad_beta, workspace, stream);
}

}  // extern "C"
