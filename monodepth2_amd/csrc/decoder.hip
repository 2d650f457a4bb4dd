// decoder.hip — DepthDecoder block fusion for gfx950.
//
// The reference decoder (networks/depth_decoder.py:50-65) builds every conv input
// with separate ops: ELU of the previous conv (layers.py:113-118), nearest x2
// upsample (layers.py:196-199), torch.cat with the encoder skip feature
// (depth_decoder.py:57-58) and ReflectionPad2d(1) (layers.py:127-135).  Each is an
// HBM round trip of a full-resolution activation (up to 12x32x194x642 fp32 at
// 640x192).  Here one pass produces the padded conv input directly from the raw
// conv output and the skip tensor, and one pass computes its adjoint (ELU
// derivative x upsample fold x reflection fold; the skip gradient falls out of the
// same sweep).  The convolutions themselves stay MIOpen's.
//
// Layouts: fp32, all three tensors NCHW contiguous, or all NHWC (channels_last,
// MD2_PAD_NHWC: what MIOpen's NHWC convolutions read and write, so no layout copy
// sits between them and this pass).  x: (B, C, h, w) pre-activation (or the raw
// feature when ELU is off); skip: (B, Cs, H, W) with (H, W) = (2h, 2w) when
// upsampling else (h, w); out: (B, C + Cs, H + 2, W + 2).  In NHWC the channel is
// the fastest index of every loop, so loads and stores stay coalesced.

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include "md2_bf16.h"
#include "md2hot.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ int reflect1(int i, int n) {  // index -1 -> 1, n -> n-2
    return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i);
}

__device__ __forceinline__ float elu(float v) { return v > 0.f ? v : expm1f(v); }
// torch's ELU backward from the result: grad * (out > 0 ? 1 : out + 1)
__device__ __forceinline__ float elu_grad(float v) { return v > 0.f ? 1.f : expm1f(v) + 1.f; }

struct PadArgs {
    int B, C, Cs, h, w, H, W;  // H, W: size after the optional upsample
    const float* x;
    const float* skip;
    float* out;
    const float* gout;
    const float* gout2;        // v4 bwd: a second gradient of the padded map (its other consumer), or null
    float* gx;
    float* gskip;
    const float* bias;         // (C,) fp32 bias of the conv that produced x, or null
    float* gbias_part;         // bwd with bias: per-block partial sums [C][gridDim.x]
};

// element (b, c, y, x) of a (B, C, Hh, Ww) tensor
template <bool NHWC>
__device__ __forceinline__ size_t at(int b, int c, int y, int x, int C, int Hh, int Ww) {
    return NHWC ? (((size_t)b * Hh + y) * Ww + x) * C + c : (((size_t)b * C + c) * Hh + y) * Ww + x;
}

template <bool ELU, bool UP, bool NHWC>
__global__ __launch_bounds__(kThreads) void pad_fwd_kernel(PadArgs a) {
    const int Hp = a.H + 2, Wp = a.W + 2, Ct = a.C + a.Cs;
    const long long total = (long long)a.B * Ct * Hp * Wp;
    for (long long idx = (long long)blockIdx.x * kThreads + threadIdx.x; idx < total;
         idx += (long long)gridDim.x * kThreads) {
        int px, py, c, b;
        long long t;
        if (NHWC) {
            c = (int)(idx % Ct);
            t = idx / Ct;
            px = (int)(t % Wp);
            t /= Wp;
            py = (int)(t % Hp);
            b = (int)(t / Hp);
        } else {
            px = (int)(idx % Wp);
            t = idx / Wp;
            py = (int)(t % Hp);
            t /= Hp;
            c = (int)(t % Ct);
            b = (int)(t / Ct);
        }
        const int yy = reflect1(py - 1, a.H), xx = reflect1(px - 1, a.W);
        float v;
        if (c < a.C) {
            const int sy = UP ? (yy >> 1) : yy, sx = UP ? (xx >> 1) : xx;
            v = a.x[at<NHWC>(b, c, sy, sx, a.C, a.h, a.w)];
            if (ELU) v = elu(v);
        } else {
            v = a.skip[at<NHWC>(b, c - a.C, yy, xx, a.Cs, a.H, a.W)];
        }
        a.out[idx] = v;
    }
}

// sum of the padded gradient over every padded position that reads source (yy, xx);
// g points at (b, c, 0, 0) of the padded gradient, es = element stride of a pixel
// (1 in NCHW, C + Cs in NHWC).
__device__ __forceinline__ float fold(const float* g, int Wp, int H, int W, int yy, int xx, int es) {
    auto G = [&](int y, int x) { return g[((size_t)y * Wp + x) * es]; };
    float s = G(yy + 1, xx + 1);
    const bool ry = (yy == 1), ry2 = (yy == H - 2), rx = (xx == 1), rx2 = (xx == W - 2);
    if (rx) s += G(yy + 1, 0);
    if (rx2) s += G(yy + 1, W + 1);
    if (ry) {
        s += G(0, xx + 1);
        if (rx) s += G(0, 0);
        if (rx2) s += G(0, W + 1);
    }
    if (ry2) {
        s += G(H + 1, xx + 1);
        if (rx) s += G(H + 1, 0);
        if (rx2) s += G(H + 1, W + 1);
    }
    return s;
}

// (b, c, y, x) of flat index k over a (B, C, Hh, Ww) tensor in the given layout
template <bool NHWC>
__device__ __forceinline__ void coords(long long k, int C, int Hh, int Ww, int& b, int& c, int& y, int& x) {
    if (NHWC) {
        c = (int)(k % C);
        k /= C;
        x = (int)(k % Ww);
        k /= Ww;
        y = (int)(k % Hh);
        b = (int)(k / Hh);
    } else {
        x = (int)(k % Ww);
        k /= Ww;
        y = (int)(k % Hh);
        k /= Hh;
        c = (int)(k % C);
        b = (int)(k / C);
    }
}

template <bool ELU, bool UP, bool NHWC>
__global__ __launch_bounds__(kThreads) void pad_bwd_kernel(PadArgs a) {
    const int Hp = a.H + 2, Wp = a.W + 2, Ct = a.C + a.Cs;
    const int es = NHWC ? Ct : 1;
    const long long nx = (long long)a.B * a.C * a.h * a.w;
    const long long ns = (long long)a.B * a.Cs * a.H * a.W;
    for (long long idx = (long long)blockIdx.x * kThreads + threadIdx.x; idx < nx + ns;
         idx += (long long)gridDim.x * kThreads) {
        int b, c, i, j;
        if (idx < nx) {
            coords<NHWC>(idx, a.C, a.h, a.w, b, c, i, j);
            const float* g = a.gout + at<NHWC>(b, c, 0, 0, Ct, Hp, Wp);
            float s;
            if (UP) {
                s = fold(g, Wp, a.H, a.W, 2 * i, 2 * j, es) + fold(g, Wp, a.H, a.W, 2 * i, 2 * j + 1, es) +
                    fold(g, Wp, a.H, a.W, 2 * i + 1, 2 * j, es) + fold(g, Wp, a.H, a.W, 2 * i + 1, 2 * j + 1, es);
            } else {
                s = fold(g, Wp, a.H, a.W, i, j, es);
            }
            if (ELU) s *= elu_grad(a.x[idx]);
            a.gx[idx] = s;
        } else {
            const long long k = idx - nx;
            coords<NHWC>(k, a.Cs, a.H, a.W, b, c, i, j);
            a.gskip[k] = fold(a.gout + at<NHWC>(b, a.C + c, 0, 0, Ct, Hp, Wp), Wp, a.H, a.W, i, j, es);
        }
    }
}

// NHWC with C and Cs multiples of 4 (every decoder width): the same passes on float4
// channel quads (a quad never straddles the x / skip boundary).
__device__ __forceinline__ float4 ld4(const float* p) { return *(const float4*)p; }
__device__ __forceinline__ void st4(float* p, float4 v) { *(float4*)p = v; }
__device__ __forceinline__ float4 add4(float4 a, float4 b) { return {a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w}; }

template <typename T, bool ELU, bool UP>
__global__ __launch_bounds__(kThreads) void pad_fwd_v4_kernel(PadArgs a) {
    const int Hp = a.H + 2, Wp = a.W + 2, Ct4 = (a.C + a.Cs) / 4;
    const int total = a.B * Hp * Wp * Ct4;   // < 2^31 (make_args): 32-bit index math
    for (int idx = blockIdx.x * kThreads + threadIdx.x; idx < total; idx += gridDim.x * kThreads) {
        const int c = 4 * (idx % Ct4);
        int t = idx / Ct4;
        const int px = t % Wp;
        t /= Wp;
        const int py = t % Hp;
        const int b = t / Hp;
        const int yy = reflect1(py - 1, a.H), xx = reflect1(px - 1, a.W);
        float4 v;
        if (c < a.C) {
            const int sy = UP ? (yy >> 1) : yy, sx = UP ? (xx >> 1) : xx;
            v = md2::ld4T<T>(a.x, (((size_t)b * a.h + sy) * a.w + sx) * a.C + c);
            if (a.bias) v = add4(v, ld4(a.bias + c));   // the conv's bias, folded in here
            if (ELU) v = {elu(v.x), elu(v.y), elu(v.z), elu(v.w)};
        } else {
            v = md2::ld4T<T>(a.skip, (((size_t)b * a.H + yy) * a.W + xx) * a.Cs + (c - a.C));
        }
        md2::st4T<T>(a.out, 4 * (size_t)idx, v);
    }
}

// fold() on quads: element offset g0 = (b, 0, 0, c) of the NHWC padded gradient
template <typename T>
__device__ __forceinline__ float4 fold4(const float* gout, const float* gout2, size_t g0, int Wp, int H, int W,
                                        int yy, int xx, int Ct) {
    auto G = [&](int y, int x) {
        const size_t o = g0 + ((size_t)y * Wp + x) * Ct;
        float4 v = md2::ld4T<T>(gout, o);
        if (gout2) v = add4(v, md2::ld4T<T>(gout2, o));   // summed per padded element, before the fold
        return v;
    };
    float4 s = G(yy + 1, xx + 1);
    const bool ry = (yy == 1), ry2 = (yy == H - 2), rx = (xx == 1), rx2 = (xx == W - 2);
    if (rx) s = add4(s, G(yy + 1, 0));
    if (rx2) s = add4(s, G(yy + 1, W + 1));
    if (ry) {
        s = add4(s, G(0, xx + 1));
        if (rx) s = add4(s, G(0, 0));
        if (rx2) s = add4(s, G(0, W + 1));
    }
    if (ry2) {
        s = add4(s, G(H + 1, xx + 1));
        if (rx) s = add4(s, G(H + 1, 0));
        if (rx2) s = add4(s, G(H + 1, W + 1));
    }
    return s;
}

// With a bias, every thread also sums the x-gradient of its channel quad (the quad is
// fixed per thread: C/4 divides the block and grid strides), the block folds the
// threads of each quad in a fixed tree and writes one partial per channel; the bias
// gradient is the fixed-order sum of those partials (bias_grad_kernel).
template <typename T, bool ELU, bool UP>
__global__ __launch_bounds__(kThreads) void pad_bwd_v4_kernel(PadArgs a) {
    const int Hp = a.H + 2, Wp = a.W + 2, Ct = a.C + a.Cs, C4 = a.C / 4, Cs4 = a.Cs / 4;
    const int nx = a.B * a.h * a.w * C4;     // nx + ns < 2^31 (make_args)
    const int ns = a.B * a.H * a.W * Cs4;
    float4 bsum = {0.f, 0.f, 0.f, 0.f};
    const float4 bq = a.bias ? ld4(a.bias + 4 * (threadIdx.x % C4)) : float4{0.f, 0.f, 0.f, 0.f};
    for (int idx = blockIdx.x * kThreads + threadIdx.x; idx < nx + ns; idx += gridDim.x * kThreads) {
        if (idx < nx) {
            const int c = 4 * (idx % C4);
            int t = idx / C4;
            const int j = t % a.w;
            t /= a.w;
            const int i = t % a.h;
            const int b = t / a.h;
            const size_t g = (size_t)b * Hp * Wp * Ct + c;
            float4 s;
            if (UP) {
                s = add4(add4(fold4<T>(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i, 2 * j, Ct),
                              fold4<T>(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i, 2 * j + 1, Ct)),
                         add4(fold4<T>(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i + 1, 2 * j, Ct),
                              fold4<T>(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i + 1, 2 * j + 1, Ct)));
            } else {
                s = fold4<T>(a.gout, a.gout2, g, Wp, a.H, a.W, i, j, Ct);
            }
            if (ELU) {
                float4 xv = md2::ld4T<T>(a.x, 4 * (size_t)idx);
                if (a.bias) xv = add4(xv, bq);   // ELU' at the biased pre-activation
                s = {s.x * elu_grad(xv.x), s.y * elu_grad(xv.y), s.z * elu_grad(xv.z), s.w * elu_grad(xv.w)};
            }
            md2::st4T<T>(a.gx, 4 * (size_t)idx, s);
            bsum = add4(bsum, s);
        } else {
            const int k = idx - nx;
            const int c = 4 * (k % Cs4);
            int t = k / Cs4;
            const int xx = t % a.W;
            t /= a.W;
            const int yy = t % a.H;
            const int b = t / a.H;
            md2::st4T<T>(a.gskip, 4 * (size_t)k, fold4<T>(a.gout, a.gout2, (size_t)b * Hp * Wp * Ct + a.C + c, Wp, a.H, a.W, yy, xx, Ct));
        }
    }
    if (!a.gbias_part) return;   // uniform: every thread of the grid returns here together
    __shared__ float4 red[kThreads];
    red[threadIdx.x] = bsum;
    __syncthreads();
    for (int half = kThreads / 2; half >= C4; half >>= 1) {   // threads t and t+half share a quad
        if ((int)threadIdx.x < half) red[threadIdx.x] = add4(red[threadIdx.x], red[threadIdx.x + half]);
        __syncthreads();
    }
    if ((int)threadIdx.x < C4) {
        const float4 v = red[threadIdx.x];
        float* p = a.gbias_part + (size_t)4 * threadIdx.x * gridDim.x + blockIdx.x;
        p[0] = v.x;
        p[gridDim.x] = v.y;
        p[2 * gridDim.x] = v.z;
        p[3 * gridDim.x] = v.w;
    }
}

// bf16 with C and Cs multiples of 8: the same passes on eight channels (one 16-byte
// access) per thread — the quad kernels moved 8 bytes per bf16 access and ran 1.9-2.6x
// their fp32 form's time at C5's batch against ~1.3x in bytes.  x, skip, out, gx and
// gskip are bitwise the quad kernels' (same per-element arithmetic); the bias
// gradient's partial sums group the pixels per thread differently (fixed order, fp32).
__device__ __forceinline__ void ld8(const void* p, size_t off, float (&v)[8]) {
    const uint4 r = *(const uint4*)((const uint16_t*)p + off);
    const uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = md2::bf2f(w[i] & 0xffffu);
        v[2 * i + 1] = md2::bf2f(w[i] >> 16);
    }
}
__device__ __forceinline__ void st8(void* p, size_t off, const float (&v)[8]) {
    *(uint4*)((uint16_t*)p + off) =
        make_uint4(md2::f2bf(v[0]) | (md2::f2bf(v[1]) << 16), md2::f2bf(v[2]) | (md2::f2bf(v[3]) << 16),
                   md2::f2bf(v[4]) | (md2::f2bf(v[5]) << 16), md2::f2bf(v[6]) | (md2::f2bf(v[7]) << 16));
}

template <bool ELU, bool UP>
__global__ __launch_bounds__(kThreads) void pad_fwd_v8_kernel(PadArgs a) {
    const int Hp = a.H + 2, Wp = a.W + 2, Ct8 = (a.C + a.Cs) / 8;
    const int total = a.B * Hp * Wp * Ct8;
    for (int idx = blockIdx.x * kThreads + threadIdx.x; idx < total; idx += gridDim.x * kThreads) {
        const int c = 8 * (idx % Ct8);
        int t = idx / Ct8;
        const int px = t % Wp;
        t /= Wp;
        const int py = t % Hp;
        const int b = t / Hp;
        const int yy = reflect1(py - 1, a.H), xx = reflect1(px - 1, a.W);
        float v[8];
        if (c < a.C) {
            const int sy = UP ? (yy >> 1) : yy, sx = UP ? (xx >> 1) : xx;
            ld8(a.x, (((size_t)b * a.h + sy) * a.w + sx) * a.C + c, v);
            if (a.bias) {
                const float4 b0 = ld4(a.bias + c), b1 = ld4(a.bias + c + 4);
                v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
                v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
            }
            if (ELU) {
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = elu(v[i]);
            }
        } else {
            ld8(a.skip, (((size_t)b * a.H + yy) * a.W + xx) * a.Cs + (c - a.C), v);
        }
        st8(a.out, 8 * (size_t)idx, v);
    }
}

// fold4 on eight channels (same tap order and per-element adds)
__device__ __forceinline__ void fold8(const void* gout, const void* gout2, size_t g0, int Wp, int H, int W, int yy,
                                      int xx, int Ct, float (&s)[8]) {
    auto G = [&](int y, int x, float (&v)[8]) {
        const size_t o = g0 + ((size_t)y * Wp + x) * Ct;
        ld8(gout, o, v);
        if (gout2) {
            float h[8];
            ld8(gout2, o, h);
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] += h[i];
        }
    };
    auto acc = [&](int y, int x) {
        float v[8];
        G(y, x, v);
#pragma unroll
        for (int i = 0; i < 8; ++i) s[i] += v[i];
    };
    G(yy + 1, xx + 1, s);
    const bool ry = (yy == 1), ry2 = (yy == H - 2), rx = (xx == 1), rx2 = (xx == W - 2);
    if (rx) acc(yy + 1, 0);
    if (rx2) acc(yy + 1, W + 1);
    if (ry) {
        acc(0, xx + 1);
        if (rx) acc(0, 0);
        if (rx2) acc(0, W + 1);
    }
    if (ry2) {
        acc(H + 1, xx + 1);
        if (rx) acc(H + 1, 0);
        if (rx2) acc(H + 1, W + 1);
    }
}

template <bool ELU, bool UP>
__global__ __launch_bounds__(kThreads) void pad_bwd_v8_kernel(PadArgs a) {
    const int Hp = a.H + 2, Wp = a.W + 2, Ct = a.C + a.Cs, C8 = a.C / 8, Cs8 = a.Cs / 8;
    const int nx = a.B * a.h * a.w * C8;
    const int ns = a.B * a.H * a.W * Cs8;
    float bsum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float bq[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (a.bias) {
        const float4 b0 = ld4(a.bias + 8 * (threadIdx.x % C8)), b1 = ld4(a.bias + 8 * (threadIdx.x % C8) + 4);
        bq[0] = b0.x; bq[1] = b0.y; bq[2] = b0.z; bq[3] = b0.w;
        bq[4] = b1.x; bq[5] = b1.y; bq[6] = b1.z; bq[7] = b1.w;
    }
    for (int idx = blockIdx.x * kThreads + threadIdx.x; idx < nx + ns; idx += gridDim.x * kThreads) {
        if (idx < nx) {
            const int c = 8 * (idx % C8);
            int t = idx / C8;
            const int j = t % a.w;
            t /= a.w;
            const int i = t % a.h;
            const int b = t / a.h;
            const size_t g = (size_t)b * Hp * Wp * Ct + c;
            float s[8];
            if (UP) {
                float f0[8], f1[8], f2[8], f3[8];
                fold8(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i, 2 * j, Ct, f0);
                fold8(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i, 2 * j + 1, Ct, f1);
                fold8(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i + 1, 2 * j, Ct, f2);
                fold8(a.gout, a.gout2, g, Wp, a.H, a.W, 2 * i + 1, 2 * j + 1, Ct, f3);
#pragma unroll
                for (int e = 0; e < 8; ++e) s[e] = (f0[e] + f1[e]) + (f2[e] + f3[e]);
            } else {
                fold8(a.gout, a.gout2, g, Wp, a.H, a.W, i, j, Ct, s);
            }
            if (ELU) {
                float xv[8];
                ld8(a.x, 8 * (size_t)idx, xv);
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    if (a.bias) xv[e] += bq[e];
                    s[e] *= elu_grad(xv[e]);
                }
            }
            st8(a.gx, 8 * (size_t)idx, s);
#pragma unroll
            for (int e = 0; e < 8; ++e) bsum[e] += s[e];
        } else {
            const int k = idx - nx;
            const int c = 8 * (k % Cs8);
            int t = k / Cs8;
            const int xx = t % a.W;
            t /= a.W;
            const int yy = t % a.H;
            const int b = t / a.H;
            float s[8];
            fold8(a.gout, a.gout2, (size_t)b * Hp * Wp * Ct + a.C + c, Wp, a.H, a.W, yy, xx, Ct, s);
            st8(a.gskip, 8 * (size_t)k, s);
        }
    }
    if (!a.gbias_part) return;   // uniform
    __shared__ float4 red[2][kThreads];
    red[0][threadIdx.x] = make_float4(bsum[0], bsum[1], bsum[2], bsum[3]);
    red[1][threadIdx.x] = make_float4(bsum[4], bsum[5], bsum[6], bsum[7]);
    __syncthreads();
    for (int half = kThreads / 2; half >= C8; half >>= 1) {   // threads t and t+half share an octet
        if ((int)threadIdx.x < half) {
            red[0][threadIdx.x] = add4(red[0][threadIdx.x], red[0][threadIdx.x + half]);
            red[1][threadIdx.x] = add4(red[1][threadIdx.x], red[1][threadIdx.x + half]);
        }
        __syncthreads();
    }
    if ((int)threadIdx.x < C8) {
        const float4 v0 = red[0][threadIdx.x], v1 = red[1][threadIdx.x];
        float* p = a.gbias_part + (size_t)8 * threadIdx.x * gridDim.x + blockIdx.x;
        p[0] = v0.x;
        p[gridDim.x] = v0.y;
        p[2 * gridDim.x] = v0.z;
        p[3 * gridDim.x] = v0.w;
        p[4 * gridDim.x] = v1.x;
        p[5 * gridDim.x] = v1.y;
        p[6 * gridDim.x] = v1.z;
        p[7 * gridDim.x] = v1.w;
    }
}

// bias gradient: one block per channel, fixed-order sum of its G block partials
__global__ __launch_bounds__(kThreads) void bias_grad_kernel(const float* part, int G, float* gbias) {
    const float* p = part + (size_t)blockIdx.x * G;
    float acc = 0.f;
    for (int g = threadIdx.x; g < G; g += kThreads) acc += p[g];
    __shared__ float red[kThreads];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int half = kThreads / 2; half > 0; half >>= 1) {
        if ((int)threadIdx.x < half) red[threadIdx.x] += red[threadIdx.x + half];
        __syncthreads();
    }
    if (threadIdx.x == 0) gbias[blockIdx.x] = red[0];
}

using PadFn = void (*)(PadArgs);

template <bool E, bool U, bool N>
PadFn fwd_of() { return pad_fwd_kernel<E, U, N>; }
template <bool E, bool U, bool N>
PadFn bwd_of() { return pad_bwd_kernel<E, U, N>; }

// the kernel instance for MD2_PAD_* flags (ELU, UPSAMPLE, NHWC)
PadFn fwd_kernel(uint32_t f) {
    static const PadFn t[8] = {fwd_of<false, false, false>(), fwd_of<true, false, false>(),
                               fwd_of<false, true, false>(),  fwd_of<true, true, false>(),
                               fwd_of<false, false, true>(),  fwd_of<true, false, true>(),
                               fwd_of<false, true, true>(),   fwd_of<true, true, true>()};
    return t[f & 7u];
}
PadFn bwd_kernel(uint32_t f) {
    static const PadFn t[8] = {bwd_of<false, false, false>(), bwd_of<true, false, false>(),
                               bwd_of<false, true, false>(),  bwd_of<true, true, false>(),
                               bwd_of<false, false, true>(),  bwd_of<true, false, true>(),
                               bwd_of<false, true, true>(),   bwd_of<true, true, true>()};
    return t[f & 7u];
}

int grid_for(long long n) {
    long long g = (n + kThreads - 1) / kThreads;
    return (int)(g < 8192 ? g : 8192);   // grid-stride beyond 8192 blocks (32 per CU)
}

// float4 channel-quad kernels: NHWC with both channel counts multiples of 4
bool vec4(const md2_pad_desc* d) {
    return (d->flags & MD2_PAD_NHWC) && d->channels % 4 == 0 && d->skip_channels % 4 == 0;
}

// bf16 octet kernels where both channel counts allow (A/B knob MD2_PAD_V8=0: quads)
bool vec8(const md2_pad_desc* d) {
    static const bool on = [] {
        const char* e = getenv("MD2_PAD_V8");
        return !(e && e[0] == '0');
    }();
    return on && (d->flags & MD2_PAD_BF16) && vec4(d) && d->channels % 8 == 0 && d->skip_channels % 8 == 0 &&
           kThreads % (d->channels / 8) == 0;
}
PadFn v8_fwd(bool elu, bool up) {
    return elu ? (up ? pad_fwd_v8_kernel<true, true> : pad_fwd_v8_kernel<true, false>)
               : (up ? pad_fwd_v8_kernel<false, true> : pad_fwd_v8_kernel<false, false>);
}
PadFn v8_bwd(bool elu, bool up) {
    return elu ? (up ? pad_bwd_v8_kernel<true, true> : pad_bwd_v8_kernel<true, false>)
               : (up ? pad_bwd_v8_kernel<false, true> : pad_bwd_v8_kernel<false, false>);
}

template <typename T>
PadFn v4_fwd(bool elu, bool up) {
    return elu ? (up ? pad_fwd_v4_kernel<T, true, true> : pad_fwd_v4_kernel<T, true, false>)
               : (up ? pad_fwd_v4_kernel<T, false, true> : pad_fwd_v4_kernel<T, false, false>);
}
template <typename T>
PadFn v4_bwd(bool elu, bool up) {
    return elu ? (up ? pad_bwd_v4_kernel<T, true, true> : pad_bwd_v4_kernel<T, true, false>)
               : (up ? pad_bwd_v4_kernel<T, false, true> : pad_bwd_v4_kernel<T, false, false>);
}

bool make_args(const md2_pad_desc* d, PadArgs& a) {
    if (!d || d->batch < 1 || d->channels < 1 || d->skip_channels < 0 || d->height < 2 || d->width < 2) return false;
    if ((d->flags & MD2_PAD_BF16) && !vec4(d)) return false;   // bf16: NHWC, channels multiples of 4
    const bool up = (d->flags & MD2_PAD_UPSAMPLE) != 0;
    a.B = d->batch;
    a.C = d->channels;
    a.Cs = d->skip_channels;
    a.h = d->height;
    a.w = d->width;
    a.H = up ? 2 * d->height : d->height;
    a.W = up ? 2 * d->width : d->width;
    // the float4 kernels index element quads in 32 bits
    return (long long)a.B * (a.C + a.Cs) * (a.H + 2) * (a.W + 2) < (1ll << 33);
}

}  // namespace

extern "C" {

size_t md2_decoder_pad_workspace_bytes(const md2_pad_desc* d) {
    PadArgs a = {};
    if (!make_args(d, a) || !vec4(d)) return 0;
    const long long n = (long long)a.B * a.C * a.h * a.w + (long long)a.B * a.Cs * a.H * a.W;
    return sizeof(float) * (size_t)a.C * grid_for(n / 4);
}

int md2_decoder_pad_fwd(const md2_pad_desc* d, const float* x, const float* skip, const float* bias, float* out,
                        void* stream) {
    PadArgs a = {};
    if (!make_args(d, a) || !x || !out || (a.Cs > 0 && !skip)) return MD2_ERR_ARG;
    if (bias && (!vec4(d) || kThreads % (d->channels / 4) != 0)) return MD2_ERR_ARG;   // as the backward
    a.x = x;
    a.skip = skip;
    a.out = out;
    a.bias = bias;
    const long long n = (long long)a.B * (a.C + a.Cs) * (a.H + 2) * (a.W + 2);
    if (vec8(d)) {
        const bool elu = d->flags & MD2_PAD_ELU, up = d->flags & MD2_PAD_UPSAMPLE;
        hipLaunchKernelGGL(v8_fwd(elu, up), dim3(grid_for(n / 8)), dim3(kThreads), 0, (hipStream_t)stream, a);
        return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
    }
    if (vec4(d)) {
        const bool elu = d->flags & MD2_PAD_ELU, up = d->flags & MD2_PAD_UPSAMPLE;
        PadFn k = (d->flags & MD2_PAD_BF16) ? v4_fwd<uint16_t>(elu, up) : v4_fwd<float>(elu, up);
        hipLaunchKernelGGL(k, dim3(grid_for(n / 4)), dim3(kThreads), 0, (hipStream_t)stream, a);
        return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
    }
    hipLaunchKernelGGL(fwd_kernel(d->flags), dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

int md2_decoder_pad_bwd(const md2_pad_desc* d, const float* x, const float* bias, const float* grad_out,
                        float* grad_x, float* grad_skip, float* grad_bias, void* workspace, void* stream) {
    return md2_decoder_pad_bwd2(d, x, bias, grad_out, nullptr, grad_x, grad_skip, grad_bias, workspace, stream);
}

int md2_decoder_pad_bwd2(const md2_pad_desc* d, const float* x, const float* bias, const float* grad_out,
                         const float* grad_out2, float* grad_x, float* grad_skip, float* grad_bias, void* workspace,
                         void* stream) {
    PadArgs a = {};
    if (!make_args(d, a) || !grad_out || !grad_x || (a.Cs > 0 && !grad_skip)) return MD2_ERR_ARG;
    if (grad_out2 && !vec4(d)) return MD2_ERR_ARG;   // only the NHWC quad kernels sum a second gradient
    const bool elu = d->flags & MD2_PAD_ELU, up = d->flags & MD2_PAD_UPSAMPLE;
    if (elu && !x) return MD2_ERR_ARG;
    // bias: the NHWC float4 kernels, with C/4 dividing the block (per-thread channel quad)
    if ((bias || grad_bias) && (!vec4(d) || kThreads % (d->channels / 4) != 0)) return MD2_ERR_ARG;
    if (grad_bias && !workspace) return MD2_ERR_ARG;
    a.x = x;
    a.gout = grad_out;
    a.gout2 = grad_out2;
    a.gx = grad_x;
    a.gskip = grad_skip;
    a.bias = bias;
    a.gbias_part = grad_bias ? (float*)workspace : nullptr;
    const long long n = (long long)a.B * a.C * a.h * a.w + (long long)a.B * a.Cs * a.H * a.W;
    if (vec8(d)) {
        const int G = grid_for(n / 8);
        hipLaunchKernelGGL(v8_bwd(elu, up), dim3(G), dim3(kThreads), 0, (hipStream_t)stream, a);
        if (grad_bias)
            hipLaunchKernelGGL(bias_grad_kernel, dim3(a.C), dim3(kThreads), 0, (hipStream_t)stream,
                               (const float*)workspace, G, grad_bias);
        return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
    }
    if (vec4(d)) {
        PadFn k = (d->flags & MD2_PAD_BF16) ? v4_bwd<uint16_t>(elu, up) : v4_bwd<float>(elu, up);
        const int G = grid_for(n / 4);
        hipLaunchKernelGGL(k, dim3(G), dim3(kThreads), 0, (hipStream_t)stream, a);
        if (grad_bias)
            hipLaunchKernelGGL(bias_grad_kernel, dim3(a.C), dim3(kThreads), 0, (hipStream_t)stream,
                               (const float*)workspace, G, grad_bias);
        return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
    }
    hipLaunchKernelGGL(bwd_kernel(d->flags), dim3(grid_for(n)), dim3(kThreads), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

}  // extern "C"
