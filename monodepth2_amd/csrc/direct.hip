// direct.hip — direct 3x3 stride-1 convolution on the f32 VALU for the DepthDecoder's
// 16-output-channel layers (networks/depth_decoder.py:50-65, upconv(0,0) 32->16 at
// H/2 and upconv(0,1) 16->16 at full resolution on the reflection-padded inputs of
// md2_decoder_pad_fwd, pad 0) and their input gradients (the "full" correlation of the
// output gradient with the flipped, transposed weight: pad 2, channel counts swapped).
//
// Why not a GEMM: with 16 output channels the implicit GEMM is 16 columns wide; its A
// tile (pixels x (tap, channel)) is re-gathered and re-split for every tap while the
// MFMAs have 16 columns to work on — x6 ran these at 36-55 TF/s, MIOpen at 41-50.  Here
// one thread owns one output pixel and all COUT channels: per tap it loads the pixel's
// CIN input channels (float4s, coalesced across lanes; the nine taps re-read them
// from L1/L2), and multiplies them into COUT accumulators with the weights as
// wave-uniform scalar operands (s_load from the [tap][cin][cout] copy, v_fma with an
// SGPR source; packed v_pk_fma_f32).  Measured against two pixels per thread (3 x 4
// column loads shared, weights serving two FMAs): slower (144 vs 108 us on the 16->16
// layer) — to fit registers its kernel rows must run rolled, which serialises the
// loads.  Exact f32 FMA chains (f32-class like MIOpen's direct kernels);
// 2 CIN COUT FMAs per pixel and tap, VALU-bound.
// Layout: x (B, H, W, CIN) NHWC, y (B, Ho, Wo, COUT) NHWC, Ho = H + 2 pad - 2,
// wk [9][CIN][COUT] fp32.

#include <hip/hip_runtime.h>

#include <type_traits>

#include <stdint.h>
#include <stdlib.h>

#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

constexpr int kThreads = 256;

template <int CIN, int COUT>
__global__ __launch_bounds__(kThreads) void conv3_direct_kernel(const float* __restrict__ x,
                                                                const float* __restrict__ wk,
                                                                float* __restrict__ y, int B, int H, int W, int Ho,
                                                                int Wo, int pad) {
    const int m = blockIdx.x * kThreads + threadIdx.x;
    if (m >= B * Ho * Wo) return;
    const int b = m / (Ho * Wo), rem = m - b * Ho * Wo, oh = rem / Wo, ow = rem - oh * Wo;
    float acc[COUT];
#pragma unroll
    for (int o = 0; o < COUT; ++o) acc[o] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
        const int ih = oh + kh - pad;
        const bool rok = (unsigned)ih < (unsigned)H;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int iw = ow + kw - pad;
            const bool ok = rok && (unsigned)iw < (unsigned)W;
            const float4* xp = (const float4*)(x + ((size_t)(b * H + (ok ? ih : 0)) * W + (ok ? iw : 0)) * CIN);
            const float* wt = wk + (kh * 3 + kw) * CIN * COUT;
#pragma unroll
            for (int q = 0; q < CIN / 4; ++q) {
                float4 v = xp[q];
                if (!ok) v = float4{0.f, 0.f, 0.f, 0.f};
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int o = 0; o < COUT; ++o) acc[o] = fmaf(vv[j], wt[(4 * q + j) * COUT + o], acc[o]);
            }
        }
    }
    float4* yp = (float4*)(y + (size_t)m * COUT);
#pragma unroll
    for (int o = 0; o < COUT / 4; ++o) yp[o] = float4{acc[4 * o], acc[4 * o + 1], acc[4 * o + 2], acc[4 * o + 3]};
}


// LDS-tiled form: a block computes a 4 x 64 output tile; its 6 x 66 input patch (all
// CIN channels) is loaded once, coalesced, into LDS, and each thread reads its nine
// taps from there (the global form re-reads every input pixel for nine taps through
// L1/TA).  Quads are rotated by the column so eight consecutive lanes' ds_read_b128
// (64 or 128 B apart) land in distinct bank groups.
constexpr int kTR = 4, kTC = 64;

template <int CIN, int COUT>
__global__ __launch_bounds__(kThreads) void conv3_direct_lds_kernel(const float* __restrict__ x,
                                                                    const float* __restrict__ wk,
                                                                    float* __restrict__ y, int B, int H, int W,
                                                                    int Ho, int Wo, int pad, int tiles_r,
                                                                    int tiles_c) {
    constexpr int QN = CIN / 4, PR = kTR + 2, PC = kTC + 2, SH = QN == 4 ? 2 : (QN == 8 ? 1 : 0);
    static_assert(kTR * kTC == kThreads, "one output pixel per thread");
    __shared__ float4 patch[PR * PC * QN];
    int t = blockIdx.x;
    const int tcb = t % tiles_c;
    t /= tiles_c;
    const int trb = t % tiles_r, b = t / tiles_r;
    const int oh0 = trb * kTR, ow0 = tcb * kTC;
    for (int i = threadIdx.x; i < PR * PC * QN; i += kThreads) {
        const int pix = i / QN, q = i - pix * QN, pr = pix / PC, pc = pix - pr * PC;
        const int ih = oh0 - pad + pr, iw = ow0 - pad + pc;
        float4 v = {0.f, 0.f, 0.f, 0.f};
        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
            v = ((const float4*)x)[((size_t)(b * H + ih) * W + iw) * QN + q];
        patch[pix * QN + ((q + (pc >> SH)) & (QN - 1))] = v;
    }
    __syncthreads();
    const int tr = threadIdx.x / kTC, tc = threadIdx.x - tr * kTC;
    const int oh = oh0 + tr, ow = ow0 + tc;
    if (oh >= Ho || ow >= Wo) return;
    float acc[COUT];
#pragma unroll
    for (int o = 0; o < COUT; ++o) acc[o] = 0.f;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
            const int pc = tc + kw, base = ((tr + kh) * PC + pc) * QN;
            const float* wt = wk + (kh * 3 + kw) * CIN * COUT;
#pragma unroll
            for (int q = 0; q < QN; ++q) {
                const float4 v = patch[base + ((q + (pc >> SH)) & (QN - 1))];
                const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int o = 0; o < COUT; ++o) acc[o] = fmaf(vv[j], wt[(4 * q + j) * COUT + o], acc[o]);
            }
        }
    float4* yp = (float4*)(y + ((size_t)(b * Ho + oh) * Wo + ow) * COUT);
#pragma unroll
    for (int o = 0; o < COUT / 4; ++o) yp[o] = float4{acc[4 * o], acc[4 * o + 1], acc[4 * o + 2], acc[4 * o + 3]};
}

// Split-bf16 MFMA form (MD2_CONV_X6 in the descriptor's flags): the same correlation as
// a GEMM with M = output pixels, N = COUT, K = 9 taps x CIN (k = tap·CIN + ci, padded to
// whole 32-k steps with zero weights), on v_mfma_f32_16x16x32_bf16 with six products of
// three exact bf16 planes per operand (f32-class, conv.hip's x6 scheme).  The GEMM is 16
// or 32 columns wide, so the weights — KS steps x NB column blocks x 3 planes of one
// fragment per lane, 60-120 VGPRs — live in registers for the block's whole life; a
// block walks output tiles (4 rows x 64 columns) persistently: it stages the tile's
// (4+2) x (64+2) x CIN input patch ONCE, split into three bf16 planes in LDS ([row]
// [col][ci], zeros outside the image), and wave w multiplies output row w: per
// 16-pixel group and k step one 16-byte fragment read per plane (eight consecutive
// channels of one tap at the pixel's window position) and 6 x NB MFMAs.  Every input
// element is split once per tile instead of once per tap.
constexpr int kXR = 4, kXC = 64;

__device__ __forceinline__ float x6_trunc16(float x) {
    return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & 0xFFFF0000u);
}
__device__ __forceinline__ uint32_t x6_hi16x2(float lo, float hi) {
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07060302u);
}
// fp32 -> bf16 bits / the bf16 value as fp32, round to nearest even (torch's cast)
__device__ __forceinline__ uint16_t x6_f2bf(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float x6_rne(float v) { return __builtin_bit_cast(float, (uint32_t)x6_f2bf(v) << 16); }
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// BF (MD2_CONV_BF16, config C5): x bf16, the tap-major fp32 weights rounded to bf16 (as
// autocast casts them) into one plane, one MFMA per fragment pair, y written as bf16 (RNE)
template <int CIN, int COUT, bool BF = false>
__global__ __launch_bounds__(kThreads, 2) void conv3_x6_kernel(const float* __restrict__ x,
                                                               const float* __restrict__ wk, float* __restrict__ y,
                                                               int B, int H, int W, int Ho, int Wo, int pad,
                                                               int tiles_r, int tiles_c) {
    constexpr int PR = kXR + 2, PC = kXC + 2, PE = PR * PC * CIN;   // patch elements per plane
    constexpr int KS = (9 * CIN + 31) / 32, NB = COUT / 16;
    constexpr int NQ = PE / 4;                                      // float4s per patch
    static_assert(kThreads == 64 * kXR, "one wave per output row of the tile");
    constexpr int NPL = BF ? 1 : 3;
    __shared__ u32x2 patch[NPL][NQ];                                // 4 bf16 per entry
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int col = lane & 15, g = lane >> 4;
    // the weight fragments: B[k = 32 s + 8 g + j][n = 16 nb + col] = wk[k][n] (k < 9 CIN)
    bf16x8 wf[KS][NB][NPL];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
            float c[3][8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int k = 32 * s + 8 * g + j;
                float v = k < 9 * CIN ? wk[k * COUT + 16 * nb + col] : 0.f;
                if constexpr (BF) v = x6_rne(v);
                const float a0 = x6_trunc16(v), r1 = v - a0, a1 = x6_trunc16(r1);
                c[0][j] = a0;
                c[1][j] = a1;
                c[2][j] = r1 - a1;
            }
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl)
                wf[s][nb][pl] = __builtin_bit_cast(
                    bf16x8, u32x4{x6_hi16x2(c[pl][0], c[pl][1]), x6_hi16x2(c[pl][2], c[pl][3]),
                                  x6_hi16x2(c[pl][4], c[pl][5]), x6_hi16x2(c[pl][6], c[pl][7])});
        }
    const int ntiles = B * tiles_r * tiles_c;
    // the tile's patch is loaded into registers one tile ahead (issued before the current
    // tile's MFMAs, so the loads' latency hides behind them), then split into LDS
    constexpr int NL = (NQ + kThreads - 1) / kThreads;
    using RegT = typename std::conditional<BF, uint2, float4>::type;
    RegT rg[NL];
    auto fetch = [&](int t) {
        const int tcb = t % tiles_c, rest = t / tiles_c, trb = rest % tiles_r, b = rest / tiles_r;
        const int oh0 = trb * kXR, ow0 = tcb * kXC;
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int i = tid + k * kThreads;
            const int pix = i / (CIN / 4), q = i - pix * (CIN / 4), pr = pix / PC, pc = pix - pr * PC;
            const int ih = oh0 - pad + pr, iw = ow0 - pad + pc;
            const bool in = i < NQ && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            const size_t o = ((size_t)(b * H + ih) * W + iw) * (CIN / 4) + q;
            if constexpr (BF) rg[k] = in ? ((const uint2*)x)[o] : uint2{0u, 0u};
            else rg[k] = in ? ((const float4*)x)[o] : float4{0.f, 0.f, 0.f, 0.f};
        }
    };
    if (blockIdx.x < ntiles) fetch(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const int tcb = t % tiles_c, rest = t / tiles_c, trb = rest % tiles_r, b = rest / tiles_r;
        const int oh0 = trb * kXR, ow0 = tcb * kXC;
        // stage the patch: float4 i = (pixel, channel quad), split into three planes
#pragma unroll
        for (int k = 0; k < NL; ++k) {
            const int i = tid + k * kThreads;
            if (NQ % kThreads && i >= NQ) break;
            if constexpr (BF) {
                patch[0][i] = u32x2{rg[k].x, rg[k].y};
            } else {
                const float4 v = rg[k];
                const float e[4] = {v.x, v.y, v.z, v.w};
                float c[3][4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float a0 = x6_trunc16(e[j]), r1 = e[j] - a0, a1 = x6_trunc16(r1);
                    c[0][j] = a0;
                    c[1][j] = a1;
                    c[2][j] = r1 - a1;
                }
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl)
                    patch[pl][i] = u32x2{x6_hi16x2(c[pl][0], c[pl][1]), x6_hi16x2(c[pl][2], c[pl][3])};
            }
        }
        __syncthreads();
        if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x);   // next tile's loads in flight
        const int oh = oh0 + wid;
        const __bf16* P0 = (const __bf16*)patch[0];
        const __bf16* P1 = (const __bf16*)patch[BF ? 0 : 1];
        const __bf16* P2 = (const __bf16*)patch[BF ? 0 : 2];
#pragma unroll
        for (int m = 0; m < kXC / 16; ++m) {
            f32x4 acc[NB];
#pragma unroll
            for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s = 0; s < KS; ++s) {
                // A[m-pixel col][k = 32 s + 8 g + j]: tap, eight channels from ci0 (tap 9 of
                // the padding step reads tap 8's place: finite, zero weights)
                const int k0 = 32 * s + 8 * g, tap = min(k0 / CIN, 8), ci0 = k0 - (k0 / CIN) * CIN;
                const int kh = tap / 3, kw = tap - kh * 3;
                const int e = ((wid + kh) * PC + 16 * m + col + kw) * CIN + ci0;
                bf16x8 fa[NPL];
                fa[0] = *(const bf16x8*)(P0 + e);
                if constexpr (BF) {
#pragma unroll
                    for (int nb = 0; nb < NB; ++nb)
                        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], wf[s][nb][0], acc[nb], 0, 0, 0);
                } else {
                    fa[1] = *(const bf16x8*)(P1 + e);
                    fa[2] = *(const bf16x8*)(P2 + e);
#pragma unroll
                    for (int nb = 0; nb < NB; ++nb) {
                        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], wf[s][nb][0], acc[nb], 0, 0, 0);
                        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], wf[s][nb][1], acc[nb], 0, 0, 0);
                        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], wf[s][nb][2], acc[nb], 0, 0, 0);
                        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], wf[s][nb][0], acc[nb], 0, 0, 0);
                        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], wf[s][nb][1], acc[nb], 0, 0, 0);
                        acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], wf[s][nb][0], acc[nb], 0, 0, 0);
                    }
                }
            }
            // D[row = 4 g + i][col]: pixel ow0 + 16 m + 4 g + i, channel 16 nb + col
            if (oh < Ho) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int ow = ow0 + 16 * m + 4 * g + i;
                    if (ow < Wo) {
                        const size_t o = ((size_t)(b * Ho + oh) * Wo + ow) * COUT + col;
#pragma unroll
                        for (int nb = 0; nb < NB; ++nb) {
                            if constexpr (BF) ((uint16_t*)y)[o + 16 * nb] = x6_f2bf(acc[nb][i]);
                            else y[o + 16 * nb] = acc[nb][i];
                        }
                    }
                }
            }
        }
        __syncthreads();   // the patch is restaged for the next tile
    }
}

// Weight gradient on split-bf16 MFMA (MD2_CONV_X6): per tap a 16 x CIN GEMM over the
// output pixels, D_tap[co][ci] += Σ_p gy[p][co] · x[p + tap][ci] — K runs over pixels, so
// both operands need eight consecutive pixels of ONE channel per lane, the transpose of
// the NHWC layout.  The block stages its tile's gy (4 x 64 pixels x 16) and input patch
// ((4+2) x (64+2) x CIN) as three bf16 planes each, pixel-major as in memory, and reads
// the fragments with ds_read_b64_tr_b16, the hardware transpose read: lane 4q+p of a
// 16-lane group points at pixel q's channels 4p..4p+3, lane i receives channel i of
// the four pixels.  Two reads give a lane its eight pixels; a tap's window shift is a
// different pixel per lane, so the nine taps read the one patch (no shifted copies).
// Pixels are stored XOR-swizzled so the two 16-lane groups of a 32-lane half (pixels
// 8 apart) land on disjoint banks.  A wave owns output row w of the tile and the 9 x
// CIN/16 accumulators of all taps for the block's whole walk; the waves' sums meet in
// LDS in wave order and each block writes one partial row [16][9][CIN], summed in block
// order by conv3_wgrad_reduce_kernel (deterministic, no atomics).
template <int C>
__device__ __forceinline__ int wg_off(int pix, int q4) {   // bf16 offset of channel quad q4 of pixel pix
    if constexpr (C == 16) return ((pix ^ (((pix >> 3) & 1) << 2)) * 16) + 4 * q4;
    else return pix * 32 + 4 * (q4 ^ (((pix >> 3) & 1) << 2));
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ s16x4 tr_read(const __bf16* p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
}

// BF (MD2_CONV_BF16): x and gy bf16, staged as they are into one plane, one MFMA per pair
template <int CIN, int TR, bool BF = false>
__global__ __launch_bounds__(kThreads, 2) void conv3_x6_wgrad_kernel(const float* __restrict__ x,
                                                                     const float* __restrict__ gy,
                                                                     float* __restrict__ part, int B, int H, int W,
                                                                     int Ho, int Wo, int pad, int tiles_r,
                                                                     int tiles_c) {
    // TR tile rows: 4 (wave w: row w, both 32-pixel steps) or 2 (CIN 32, whose patch
    // planes would otherwise leave room for one block per CU: wave w: row w/2, step w%2)
    constexpr int COUT = 16, PR = TR + 2, PC = kXC + 2, CB = CIN / 16, KSW = TR == 4 ? 2 : 1;
    static_assert(TR == 4 || TR == 2, "tile rows");
    // bf16 per plane; the pixel swizzle permutes within aligned groups of 16 pixels, so the
    // patch plane is padded to whole groups (396 -> 400 pixels)
    constexpr int XE = (PR * PC + 15) / 16 * 16 * CIN, GE = TR * kXC * COUT;
    constexpr int NPL = BF ? 1 : 3;
    __shared__ __attribute__((aligned(16))) __bf16 xs[BF ? 2 : 3][XE];   // (the wave reduction reuses 2 planes' worth)
    __shared__ __attribute__((aligned(16))) __bf16 gs[NPL][GE];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int g16 = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
    f32x4 acc[9][CB];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc[t][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto put = [&](__bf16* base, int stride, int off, float4 v) {
        const float e[4] = {v.x, v.y, v.z, v.w};
        float c[3][4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float a0 = x6_trunc16(e[j]), r1 = e[j] - a0, a1 = x6_trunc16(r1);
            c[0][j] = a0;
            c[1][j] = a1;
            c[2][j] = r1 - a1;
        }
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
            *(u32x2*)(base + pl * stride + off) = u32x2{x6_hi16x2(c[pl][0], c[pl][1]), x6_hi16x2(c[pl][2], c[pl][3])};
    };
    auto put_bf = [&](__bf16* base, int off, uint2 u) { *(u32x2*)(base + off) = u32x2{u.x, u.y}; };
    const int ntiles = B * tiles_r * tiles_c;
    // the next tile's input patch and output gradient are loaded into registers while
    // the current tile's MFMAs run (as conv3_x6_kernel), then split / copied into LDS
    constexpr int NX = PR * PC * CIN / 4, NG4 = GE / 4;
    constexpr int LX = (NX + kThreads - 1) / kThreads, LG = (NG4 + kThreads - 1) / kThreads;
    using RegT = typename std::conditional<BF, uint2, float4>::type;
    RegT rx[LX], rgy[LG];
    auto fetch = [&](int t) {
        const int tcb = t % tiles_c, rest = t / tiles_c, trb = rest % tiles_r, b = rest / tiles_r;
        const int oh0 = trb * TR, ow0 = tcb * kXC;
#pragma unroll
        for (int k = 0; k < LX; ++k) {   // input patch, zeros outside the image
            const int i = tid + k * kThreads;
            const int pix = i / (CIN / 4), q4 = i - pix * (CIN / 4), pr = pix / PC, pc = pix - pr * PC;
            const int ih = oh0 - pad + pr, iw = ow0 - pad + pc;
            const bool in = i < NX && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            const size_t o = ((size_t)(b * H + ih) * W + iw) * (CIN / 4) + q4;
            if constexpr (BF) rx[k] = in ? ((const uint2*)x)[o] : uint2{0u, 0u};
            else rx[k] = in ? ((const float4*)x)[o] : float4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int k = 0; k < LG; ++k) {   // output gradient, zeros past the output
            const int i = tid + k * kThreads;
            const int pix = i >> 2, q4 = i & 3, pr = pix / kXC, pc = pix - pr * kXC;
            const int oh = oh0 + pr, ow = ow0 + pc;
            const bool in = i < NG4 && oh < Ho && ow < Wo;
            const size_t o = ((size_t)(b * Ho + oh) * Wo + ow) * 4 + q4;
            if constexpr (BF) rgy[k] = in ? ((const uint2*)gy)[o] : uint2{0u, 0u};
            else rgy[k] = in ? ((const float4*)gy)[o] : float4{0.f, 0.f, 0.f, 0.f};
        }
    };
    if (blockIdx.x < ntiles) fetch(blockIdx.x);
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
#pragma unroll
        for (int k = 0; k < LX; ++k) {
            const int i = tid + k * kThreads;
            if (NX % kThreads && i >= NX) break;
            const int pix = i / (CIN / 4), q4 = i - pix * (CIN / 4);
            if constexpr (BF) put_bf(&xs[0][0], wg_off<CIN>(pix, q4), rx[k]);
            else put(&xs[0][0], XE, wg_off<CIN>(pix, q4), rx[k]);
        }
#pragma unroll
        for (int k = 0; k < LG; ++k) {
            const int i = tid + k * kThreads;
            if (NG4 % kThreads && i >= NG4) break;
            const int pix = i >> 2, q4 = i & 3;
            if constexpr (BF) put_bf(&gs[0][0], wg_off<16>(pix, q4), rgy[k]);
            else put(&gs[0][0], GE, wg_off<16>(pix, q4), rgy[k]);
        }
        __syncthreads();
        if (t + (int)gridDim.x < ntiles) fetch(t + gridDim.x);
        const int wrow = TR == 4 ? wid : wid >> 1, ks0 = TR == 4 ? 0 : wid & 1;
#pragma unroll
        for (int kk = 0; kk < KSW; ++kk) {
            const int ks = ks0 + kk;
            // A = gy^T: row co = lane & 15, k = pixel 8 g16 + j of this 32-pixel step
            bf16x8 fa[NPL];
            const int gp = wrow * kXC + 32 * ks + 8 * g16 + q;
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) {
                const s16x4 lo = tr_read(&gs[pl][wg_off<16>(gp, p4)]), hi = tr_read(&gs[pl][wg_off<16>(gp + 4, p4)]);
                fa[pl] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int kh = tap / 3, kw = tap - kh * 3;
                const int xp = (wrow + kh) * PC + 32 * ks + 8 * g16 + q + kw;
#pragma unroll
                for (int cb = 0; cb < CB; ++cb) {
                    bf16x8 fb[NPL];
#pragma unroll
                    for (int pl = 0; pl < NPL; ++pl) {
                        const s16x4 lo = tr_read(&xs[pl][wg_off<CIN>(xp, 4 * cb + p4)]),
                                    hi = tr_read(&xs[pl][wg_off<CIN>(xp + 4, 4 * cb + p4)]);
                        fb[pl] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
                    }
                    if constexpr (BF) {
                        acc[tap][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[0], acc[tap][cb], 0, 0, 0);
                    } else {
                        f32x4 c = acc[tap][cb];
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fb[0], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[1], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[2], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[0], c, 0, 0, 0);
                        c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[1], c, 0, 0, 0);
                        acc[tap][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[0], c, 0, 0, 0);
                    }
                }
            }
        }
        __syncthreads();   // the planes are restaged for the next tile
    }
    // the four waves' sums in wave order through LDS (the x planes, free now):
    // ((w0 + w1) + w2) + w3, then this block's partial row [co][tap][ci]:
    // D[row = co = 4 g16 + e][col = ci = 16 cb + lane & 15]
    float* red = (float*)&xs[0][0];
    static_assert(9 * CB * 256 * 4 <= (BF ? 2 : 3) * XE * 2, "reduction buffer fits in the patch planes");
    for (int w = 0; w < 4; ++w) {
        if (wid == w) {
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int cb = 0; cb < CB; ++cb)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float* r = &red[(tap * CB + cb) * 256 + e * 64 + lane];
                        *r = w == 0 ? acc[tap][cb][e] : *r + acc[tap][cb][e];
                    }
        }
        __syncthreads();
    }
    float* out = part + (size_t)blockIdx.x * COUT * 9 * CIN;
    for (int i = tid; i < 9 * CB * 256; i += kThreads) {
        const int tc = i >> 8, r = i & 255, e = r >> 6, l = r & 63, tap = tc / CB, cb = tc - tap * CB;
        const int co = 4 * (l >> 4) + e, ci = 16 * cb + (l & 15);
        out[(co * 9 + tap) * CIN + ci] = red[i];
    }
}

bool direct_lds() {   // A/B knob: MD2_DIRECT_LDS=0 selects the global-load form
    static const bool on = [] {
        const char* e = getenv("MD2_DIRECT_LDS");
        return !(e && e[0] == '0');
    }();
    return on;
}

// Weight gradient of the same layers: gw[co][tap][ci] = sum_p gy[p][co] x[p + tap][ci]
// over every output pixel p.  A block walks chunks of 64 consecutive pixels: the chunk's
// gy rows and each pixel's nine tap rows of x (zero outside the image) are staged in
// LDS; a thread owns a (4 co x 4 ci) quad pair over all 9 taps (144 accumulators) and
// a residue class of the chunk's pixels (G = 256 / pairs groups), so per pixel it
// reads one gy quad and nine x quads for 144 FMAs.  The groups' sums are combined in
// LDS in a fixed order, one partial row [COUT][9][CIN] per block; conv3_wgrad_reduce
// adds the blocks' rows in block order (deterministic, no atomics).
constexpr int kWChunk = 64;

template <int CIN, int COUT>
__global__ __launch_bounds__(kThreads) void conv3_wgrad_direct_kernel(const float* __restrict__ x,
                                                                      const float* __restrict__ gy,
                                                                      float* __restrict__ part, int B, int H, int W,
                                                                      int Ho, int Wo, int pad, int chunks_per_block) {
    constexpr int IQ = CIN / 4, OQ = COUT / 4, PAIRS = IQ * OQ, G = kThreads / PAIRS;
    constexpr int NOUT = COUT * 9 * CIN;
    static_assert(kThreads % PAIRS == 0 && kThreads == 4 * kWChunk && IQ % 4 == 0 && OQ <= 4, "thread roles");
    __shared__ float4 sx[kWChunk][9][IQ];
    __shared__ float4 sg[kWChunk][OQ];
    __shared__ float red[G][PAIRS * 16];
    const int tid = threadIdx.x, g = tid / PAIRS, u = tid - g * PAIRS, oq = u / IQ, iq = u - oq * IQ;
    const int P = B * Ho * Wo;
    float acc[9][4][4];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) acc[t][a][c] = 0.f;
    // staging role: chunk pixel t % 64 (one pixel decomposition per chunk) and quads
    // j + 4 k of its [tap][quad] rows, j = t / 64 (tap = 4k / IQ and quad j + 4k % IQ
    // are compile-time in k); the next chunk's loads are issued into registers before
    // this chunk's FMAs, so their latency hides behind them
    constexpr int NK = 9 * IQ / 4;
    const int spp = tid % kWChunk, sj = tid / kWChunk;
    float4 rx[NK], rg;
    const int c0 = blockIdx.x * chunks_per_block;
    const int cend = min(c0 + chunks_per_block, (P + kWChunk - 1) / kWChunk);
    auto fetch = [&](int ch) {
        const int p = ch * kWChunk + spp;
        const bool live = ch < cend && p < P;
        int b = 0, oh = 0, ow = 0;
        if (live) {
            b = p / (Ho * Wo);
            const int rem = p - b * Ho * Wo;
            oh = rem / Wo;
            ow = rem - oh * Wo;
        }
        rg = (live && sj < OQ) ? ((const float4*)gy)[(size_t)p * OQ + sj] : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int tap = 4 * k / IQ, q = sj + (4 * k) % IQ;
            const int ih = oh + tap / 3 - pad, iw = ow + tap % 3 - pad;
            rx[k] = (live && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W)
                        ? ((const float4*)x)[((size_t)(b * H + ih) * W + iw) * IQ + q]
                        : float4{0.f, 0.f, 0.f, 0.f};
        }
    };
    fetch(c0);
    for (int ch = c0; ch < cend; ++ch) {
        if (sj < OQ) sg[spp][sj] = rg;
#pragma unroll
        for (int k = 0; k < NK; ++k) sx[spp][4 * k / IQ][sj + (4 * k) % IQ] = rx[k];
        __syncthreads();
        fetch(ch + 1);
        for (int pp = g; pp < kWChunk; pp += G) {
            const float4 gv = sg[pp][oq];
            const float ga[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const float4 xv = sx[pp][t][iq];
                const float xa[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int c = 0; c < 4; ++c) acc[t][a][c] = fmaf(ga[a], xa[c], acc[t][a][c]);
            }
        }
        __syncthreads();
    }
    // combine the G groups per tap in a fixed order, one partial row per block
    float* out = part + (size_t)blockIdx.x * NOUT;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int c = 0; c < 4; ++c) red[g][u * 16 + a * 4 + c] = acc[t][a][c];
        __syncthreads();
        for (int i = tid; i < PAIRS * 16; i += kThreads) {
            float sum = 0.f;
            for (int k = 0; k < G; ++k) sum += red[k][i];
            const int uu = i / 16, a = (i / 4) % 4, c = i % 4, oo = uu / IQ, ii = uu - oo * IQ;
            out[((4 * oo + a) * 9 + t) * CIN + 4 * ii + c] = sum;
        }
        __syncthreads();
    }
}

// gw[i] = sum over blocks of part[blk][i]: 16 outputs per block, 16 lanes per output
// (lane l sums blocks l, l + 16, ... with four loads in flight), the 16 lane sums then
// added in lane order — deterministic.  (Four lanes per output, 128 dependent loads
// each, took 33 us for 512 rows.)
constexpr int kRedO = 16, kRedL = kThreads / kRedO;
__global__ __launch_bounds__(kThreads) void conv3_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                      float* __restrict__ gw, int n, int nblk) {
    __shared__ float red[kRedL][kRedO];
    const int o = threadIdx.x % kRedO, l = threadIdx.x / kRedO;
    const int i = blockIdx.x * kRedO + o;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (i < n) {
        int k = l;
        for (; k + 3 * kRedL < nblk; k += 4 * kRedL) {
            s0 += part[(size_t)k * n + i];
            s1 += part[(size_t)(k + kRedL) * n + i];
            s2 += part[(size_t)(k + 2 * kRedL) * n + i];
            s3 += part[(size_t)(k + 3 * kRedL) * n + i];
        }
        for (; k < nblk; k += kRedL) s0 += part[(size_t)k * n + i];
    }
    red[l][o] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (l == 0 && i < n) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < kRedL; ++j) s += red[j][o];
        gw[i] = s;
    }
}

}  // namespace

extern "C" {

int md2_conv_direct(const md2_conv_desc* d, const float* x, const float* wk, float* y, void* stream) {
    if (!d || !x || !wk || !y) return md2_report_error(MD2_ERR_ARG, "conv_direct: NULL operand");
    if (d->kernel_h != 3 || d->kernel_w != 3 || d->stride != 1 || d->pad < 0 || d->pad > 2 || d->batch < 1 ||
        d->height < 1 || d->width < 1)
        return md2_report_error(MD2_ERR_ARG, "conv_direct: 3x3, stride 1, pad 0..2");
    const int Ho = d->height + 2 * d->pad - 2, Wo = d->width + 2 * d->pad - 2;
    if (Ho < 1 || Wo < 1) return md2_report_error(MD2_ERR_ARG, "conv_direct: empty output");
    const long long M = (long long)d->batch * Ho * Wo;
    if (M * 32 >= (1ll << 31) || (long long)d->batch * d->height * d->width * 32 >= (1ll << 31))
        return md2_report_error(MD2_ERR_ARG, "conv_direct: tensors of < 2^26 pixels");
    const dim3 grid((unsigned)((M + kThreads - 1) / kThreads));
    const hipStream_t st = (hipStream_t)stream;
    const int ci = d->in_channels, co = d->out_channels;
    if (d->flags & MD2_CONV_X6) {
        const int tr = (Ho + kXR - 1) / kXR, tc = (Wo + kXC - 1) / kXC;
        const long long nt = (long long)d->batch * tr * tc;
        const bool bf = (d->flags & MD2_CONV_BF16) != 0;   // bf16 x / y (config C5)
        // persistent: as many blocks as are resident per CU (the kernels' occupancy with
        // the next tile's patch held in registers: fp32 3 / 2 / 2, bf16 4 / 3 / 4 for
        // 16->16 / 32->16 / 16->32; a fourth fp32 16->16 block would only queue)
        const int per_cu = bf ? ((ci == 32) ? 3 : 4) : ((ci == 16 && co == 16) ? 3 : 2);
        const long long cap = 256ll * per_cu;
        const dim3 g2((unsigned)(nt < cap ? nt : cap));
        void (*k)(const float*, const float*, float*, int, int, int, int, int, int, int, int) =
            (ci == 16 && co == 16)   ? (bf ? conv3_x6_kernel<16, 16, true> : conv3_x6_kernel<16, 16>)
            : (ci == 32 && co == 16) ? (bf ? conv3_x6_kernel<32, 16, true> : conv3_x6_kernel<32, 16>)
            : (ci == 16 && co == 32) ? (bf ? conv3_x6_kernel<16, 32, true> : conv3_x6_kernel<16, 32>)
                                     : nullptr;
        if (k)
            hipLaunchKernelGGL(k, g2, dim3(kThreads), 0, st, x, wk, y, d->batch, d->height, d->width, Ho, Wo, d->pad,
                               tr, tc);
        else
            return md2_report_error(MD2_ERR_ARG, "conv_direct: (in, out) channels (16,16), (32,16) or (16,32)");
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
    }
    // the LDS-tiled form where it measured faster: 16 output channels (16->16 forward /
    // input gradient 95 / 100 vs 104 / 104 us, 32->16 forward 72 vs 83 us); with 32
    // output channels (the 32->16 layer's input gradient) the global form (56 vs 76 us)
    if (direct_lds() && co == 16) {
        const int tr = (Ho + kTR - 1) / kTR, tc = (Wo + kTC - 1) / kTC;
        const dim3 g2((unsigned)((long long)d->batch * tr * tc));
        if (ci == 16 && co == 16)
            hipLaunchKernelGGL((conv3_direct_lds_kernel<16, 16>), g2, dim3(kThreads), 0, st, x, wk, y, d->batch,
                               d->height, d->width, Ho, Wo, d->pad, tr, tc);
        else if (ci == 32 && co == 16)
            hipLaunchKernelGGL((conv3_direct_lds_kernel<32, 16>), g2, dim3(kThreads), 0, st, x, wk, y, d->batch,
                               d->height, d->width, Ho, Wo, d->pad, tr, tc);
        else if (ci == 16 && co == 32)
            hipLaunchKernelGGL((conv3_direct_lds_kernel<16, 32>), g2, dim3(kThreads), 0, st, x, wk, y, d->batch,
                               d->height, d->width, Ho, Wo, d->pad, tr, tc);
        else
            return md2_report_error(MD2_ERR_ARG, "conv_direct: (in, out) channels (16,16), (32,16) or (16,32)");
    } else if (ci == 16 && co == 16)
        hipLaunchKernelGGL((conv3_direct_kernel<16, 16>), grid, dim3(kThreads), 0, st, x, wk, y, d->batch, d->height,
                           d->width, Ho, Wo, d->pad);
    else if (ci == 32 && co == 16)
        hipLaunchKernelGGL((conv3_direct_kernel<32, 16>), grid, dim3(kThreads), 0, st, x, wk, y, d->batch, d->height,
                           d->width, Ho, Wo, d->pad);
    else if (ci == 16 && co == 32)
        hipLaunchKernelGGL((conv3_direct_kernel<16, 32>), grid, dim3(kThreads), 0, st, x, wk, y, d->batch, d->height,
                           d->width, Ho, Wo, d->pad);
    else
        return md2_report_error(MD2_ERR_ARG, "conv_direct: (in, out) channels (16,16), (32,16) or (16,32)");
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}


constexpr int kWBlocks = 512;   // partial rows of the weight gradient

size_t md2_conv_wgrad_direct_workspace_bytes(const md2_conv_desc* d) {
    return d ? sizeof(float) * (size_t)kWBlocks * d->out_channels * 9 * d->in_channels : 0;
}

int md2_conv_wgrad_direct(const md2_conv_desc* d, const float* x, const float* grad_y, float* grad_weight,
                          void* workspace, void* stream) {
    if (!d || !x || !grad_y || !grad_weight || !workspace)
        return md2_report_error(MD2_ERR_ARG, "conv_wgrad_direct: NULL operand or workspace");
    if (d->kernel_h != 3 || d->kernel_w != 3 || d->stride != 1 || d->pad < 0 || d->pad > 2 || d->batch < 1)
        return md2_report_error(MD2_ERR_ARG, "conv_wgrad_direct: 3x3, stride 1, pad 0..2");
    const int Ho = d->height + 2 * d->pad - 2, Wo = d->width + 2 * d->pad - 2;
    if (Ho < 1 || Wo < 1) return md2_report_error(MD2_ERR_ARG, "conv_wgrad_direct: empty output");
    const long long P = (long long)d->batch * Ho * Wo;
    if (P * 32 >= (1ll << 31) || (long long)d->batch * d->height * d->width * 32 >= (1ll << 31))
        return md2_report_error(MD2_ERR_ARG, "conv_wgrad_direct: tensors of < 2^26 pixels");
    const hipStream_t st0 = (hipStream_t)stream;
    if (d->flags & MD2_CONV_X6) {
        if (d->out_channels != 16 || (d->in_channels != 16 && d->in_channels != 32))
            return md2_report_error(MD2_ERR_ARG, "conv_wgrad_direct: (in, out) channels (16,16) or (32,16)");
        static const int tr16 = [] {   // A/B knob: MD2_WGRAD_TR16=2 runs the 16-channel form on 2-row tiles
            const char* e = getenv("MD2_WGRAD_TR16");
            return e && e[0] == '2' ? 2 : 4;
        }();
        const int TRW = d->in_channels == 16 ? tr16 : 2;
        const int tr = (Ho + TRW - 1) / TRW, tc = (Wo + kXC - 1) / kXC;
        const long long nt = (long long)d->batch * tr * tc;
        const int nb = (int)(nt < kWBlocks ? nt : kWBlocks);
        float* part = (float*)workspace;
        const bool bf = (d->flags & MD2_CONV_BF16) != 0;   // bf16 x / grad_y (config C5)
        void (*k)(const float*, const float*, float*, int, int, int, int, int, int, int, int) =
            (d->in_channels == 16 && TRW == 4) ? (bf ? conv3_x6_wgrad_kernel<16, 4, true> : conv3_x6_wgrad_kernel<16, 4>)
            : d->in_channels == 16             ? (bf ? conv3_x6_wgrad_kernel<16, 2, true> : conv3_x6_wgrad_kernel<16, 2>)
                                               : (bf ? conv3_x6_wgrad_kernel<32, 2, true> : conv3_x6_wgrad_kernel<32, 2>);
        hipLaunchKernelGGL(k, dim3(nb), dim3(kThreads), 0, st0, x, grad_y, part, d->batch, d->height, d->width, Ho, Wo,
                           d->pad, tr, tc);
        const int n = 16 * 9 * d->in_channels;
        hipLaunchKernelGGL(conv3_wgrad_reduce_kernel, dim3((n + kRedO - 1) / kRedO), dim3(kThreads), 0, st0, part,
                           grad_weight, n, nb);
        const hipError_t e = hipGetLastError();
        return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
    }
    const int chunks = (int)((P + kWChunk - 1) / kWChunk);
    const int per = (chunks + kWBlocks - 1) / kWBlocks;
    const int nblk = (chunks + per - 1) / per;
    const hipStream_t st = (hipStream_t)stream;
    float* part = (float*)workspace;
    const int ci = d->in_channels, co = d->out_channels, n = co * 9 * ci;
    if (ci == 16 && co == 16)
        hipLaunchKernelGGL((conv3_wgrad_direct_kernel<16, 16>), dim3(nblk), dim3(kThreads), 0, st, x, grad_y, part,
                           d->batch, d->height, d->width, Ho, Wo, d->pad, per);
    else if (ci == 32 && co == 16)
        hipLaunchKernelGGL((conv3_wgrad_direct_kernel<32, 16>), dim3(nblk), dim3(kThreads), 0, st, x, grad_y, part,
                           d->batch, d->height, d->width, Ho, Wo, d->pad, per);
    else
        return md2_report_error(MD2_ERR_ARG, "conv_wgrad_direct: (in, out) channels (16,16) or (32,16)");
    hipLaunchKernelGGL(conv3_wgrad_reduce_kernel, dim3((n + kRedO - 1) / kRedO), dim3(kThreads), 0, st, part,
                       grad_weight, n, nblk);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
