// conv.hip — fp32 convolutions of the ResNet encoders and the DepthDecoder as implicit
// GEMMs on gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32: exact f32 fma chains, the same
// 157 TFLOP/s as the f32 vector peak), NHWC activations, weights in PyTorch's
// channels_last layout [co][kh][kw][ci].
//
// Callers: networks/resnet_encoder.py (torchvision BasicBlock / Bottleneck 3x3 and 1x1
// convs) and networks/depth_decoder.py:50-65 (Conv3x3 = ReflectionPad2d(1) +
// Conv2d(.., 3); the padding is done by csrc/decoder.hip, so the conv is "valid").
//
//   forward      y[p][n]   = Σ_{tap,c} x[p's tap][c] · w[n][tap][c]     M = pixels, N = Co, K = taps·Ci
//   input grad   gx[p][ci] = Σ_{tap,co} gy[p's flipped tap][co] · w[co][tap][ci]   (stride 1: a
//                "full" convolution of gy, padding k-1-p, the weight read transposed)
//   weight grad  gw[co][tap][ci] = Σ_p x[p's tap][ci] · gy[p][co]       M = taps·Ci, N = Co, K = pixels
//                (written transposed: [co][tap][ci] = the channels_last weight)
//
// One kernel template: block = 4 waves, tile 128 x BN (BN = 32/64/128), K in chunks of
// 32.  The next-but-one chunk is loaded into registers (row-coalesced dwordx4 buffer
// loads; an offset past the buffer end reads zeros = the zero padding outside the
// image, so no branch surrounds a load) while the MFMAs consume the current chunk from
// LDS; one barrier per chunk.  Each operand is staged in the orientation it has in
// HBM: "row-k" tiles (a row of 32 contiguous k values: im2col rows, forward weights)
// with XOR-swizzled 16-byte quads, read 4 k-values per ds_read_b128; "k-row" tiles (a
// row per k value: gy and x in the weight gradient, the weight in the input gradient)
// read with one ds_read_b32 per MFMA.  Lane l feeds k = 16·(l/32) + j of the chunk to
// MFMA j, A and B alike.  Deterministic: a K split writes partials that a second
// launch sums in split order.

#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <stdint.h>

#include <algorithm>
#include <type_traits>

#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kThreads = 256;
constexpr int BM = 128;         // tile rows (M)
constexpr int BK = 32;          // K per chunk

enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

// physical quad of logical quad q in a row-k LDS row r (32 floats): conflict-free
// ds_read_b128 of the MFMA operand pattern (16 lanes = 16 rows at one logical quad)
// and of the staging writes (8 lanes = one row)
__device__ __forceinline__ int swz(int r, int q) { return (q ^ (r >> 1)) & 7; }

struct ConvArgs {
    int B, H, W, C;          // input of the GEMM's pixel side (NHWC): x (fwd), gy (dgrad), x (wgrad)
    int Ho, Wo;              // output spatial (fwd / dgrad: the y / gx pixels; wgrad: gy pixels)
    int N;                   // fwd: Co; dgrad: Ci; wgrad: taps·Ci
    int M;                   // fwd / dgrad: pixels; wgrad: Co
    int P;                   // wgrad: pixels (K)
    int Cg;                  // wgrad: channels of gy (= N)
    int KH, KW, stride, pad;
    int mblocks, nblocks, splits, chunks_per_split, nchunks;
    int a_elems, b_elems;    // sizes of the two operands (the buffer-descriptor bounds)
    int bn;                  // tile width chosen by plan()
    int bm;                  // x6 tile height (128 or 256)
    // x6 stride-2 input gradient, one output parity class (py, px) per launch: the
    // GEMM pixels are gx(2 oh + py, 2 ow + px) on the Ho x Wo class grid, the taps
    // kh = kh0 + 2 th (th < nth), kw = kw0 + 2 tw (tw < ntw) read gy(oh + dy0 - th,
    // ow + dx0 - tw); outputs scatter into the oHf x oWf image
    int par, py, px, kh0, kw0, ntw, dy0, dx0, oHf, oWf;
    int flatk;               // x6 fwd / dgrad with C < 32: K chunks run over the flattened
                             // (tap, channel) index, several taps per chunk
    int ptr, ptc;            // patch kernel (conv_x6p_kernel): output tiles per image, rows / columns
    // conv_x6_kernel over several stride-2 parity classes in one launch (ncls > 0): the
    // blocks of class c start at cls_blk[c]; per class the fields above it replaces
    int ncls;
    int cls_blk[4], cls_py[4], cls_px[4], cls_kh0[4], cls_kw0[4], cls_ntw[4], cls_dy0[4], cls_dx0[4], cls_Ho[4],
        cls_Wo[4], cls_nchunks[4];
    const float* a;          // fwd: x; dgrad: gy; wgrad: x
    const float* b;          // fwd / dgrad: weight; wgrad: gy
    float* y;                // output [M][N], or partials [splits][M][N]
    // MD2_CONV_BF16 (ABI 22): bf16 activations / one bf16 weight plane; the output is
    // written as bf16 (ybf16 = 1, fwd / dgrad) or as fp32 rounded to bf16 values (ybf16 =
    // 2, wgrad) when there is no K split (else the reduction does it)
    int ybf16;
};

__device__ __forceinline__ int xcd_contiguous_block(int bid, int n) {
    const int q = n >> 3, r = n & 7;
    const int xcd = bid & 7, idx = bid >> 3;
    return xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
}

__device__ __forceinline__ float4 bload(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

constexpr int kBad = 0x7fffffff;   // a byte offset past every buffer: the load returns zeros

// 8 bytes (four bf16) from a buffer
__device__ __forceinline__ uint2 bload8(__amdgpu_buffer_rsrc_t r, int byte_off) {
    return __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(r, byte_off, 0, 0));
}
// fp32 -> bf16 bits, round to nearest even (finite values; NaN stays a NaN)
__device__ __forceinline__ uint16_t f2bf16(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_round(float v) {
    return __builtin_bit_cast(float, (uint32_t)f2bf16(v) << 16);
}

// n / d for 0 <= n < 2^24, d >= 1, from a float reciprocal (rd = 1.0f / d) and one
// correction step each way: ~6 VALU instead of the ~30 of an integer division
__device__ __forceinline__ int fdiv(int n, int d, float rd) {
    int q = (int)((float)n * rd);
    const int r = n - q * d;
    q += (r >= d) - (r < 0);
    return q;
}

template <int BN, int MODE>
struct Cfg {
    static constexpr int WAVES_M = BN == 32 ? 4 : 2;
    static constexpr int WAVES_N = 4 / WAVES_M;
    static constexpr int TM = BM / WAVES_M / 32;   // 32x32 MFMA tiles per wave
    static constexpr int TN = BN / WAVES_N / 32;
    static constexpr bool A_ROWK = MODE != MODE_WGRAD;   // else k-row
    static constexpr bool B_ROWK = MODE == MODE_FWD;
    static constexpr int AQ = BM * BK / 4 / kThreads;    // 16-byte quads per thread per chunk
    static constexpr int BQ = BN * BK / 4 / kThreads;
    static constexpr int A_FLOATS = BM * BK, B_FLOATS = BN * BK;
};

template <int BN, int MODE>
__global__ __launch_bounds__(kThreads, BN == 128 ? 2 : (BN == 64 ? 3 : 4)) void conv_gemm_kernel(ConvArgs a) {
    using G = Cfg<BN, MODE>;
    constexpr int TM = G::TM, TN = G::TN, AQ = G::AQ, BQ = G::BQ;
    __shared__ float lds[2][G::A_FLOATS + G::B_FLOATS];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / G::WAVES_N, wn = wid % G::WAVES_N;
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int nb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int m0 = mb * BM, n0 = nb * BN;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);
    const int KT = a.KH * a.KW;

    // ---------------------------------------------------------------- A side
    // row-k (fwd / dgrad): thread rows r = tid/8 + 32 j of the 128-pixel tile, quad tid%8
    // k-row (wgrad): quad i = tid + 256 j of the [32 pixels][128 (tap, ci)] tile
    const int qa = tid & 7, ra = tid >> 3;
    int aih[AQ], aiw[AQ], apb[AQ];
    const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc(
        (void*)a.a, 0, a.a_elems * 4, 0x00020000);
    if (MODE != MODE_WGRAD) {
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const int m = m0 + ra + 32 * j;
            if (m < a.M) {
                const int b = m / (a.Ho * a.Wo), rem = m - b * a.Ho * a.Wo;
                const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
                aih[j] = oh * a.stride - a.pad;
                aiw[j] = ow * a.stride - a.pad;
                apb[j] = ((b * a.H + aih[j]) * a.W + aiw[j]) * a.C + 4 * qa;
            } else {
                aih[j] = -(1 << 20);
                aiw[j] = 0;
                apb[j] = 0;
            }
        }
    }
    // wgrad A side (x): per quad its (tap, ci); every quad of this thread sits in k row
    // tid/32 + 8 j of the chunk, whose pixel (b, oh, ow) is tracked incrementally
    int wkh[AQ], wkw[AQ], wci[AQ];
    int pb_b = 0, pb_oh = 0, pb_ow = 0;
    if (MODE == MODE_WGRAD) {
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const int m = m0 + 4 * (tid % (BM / 4));
            const int tap = m / a.C, ci = m - tap * a.C;
            wkh[j] = m < a.M ? tap / a.KW : -(1 << 20);
            wkw[j] = tap - (tap / a.KW) * a.KW;
            wci[j] = ci;
        }
        const int pk = t0 * BK + tid / (BM / 4);
        pb_b = pk / (a.Ho * a.Wo);
        const int rem = pk - pb_b * a.Ho * a.Wo;
        pb_oh = rem / a.Wo;
        pb_ow = rem - pb_oh * a.Wo;
    }
    // ---------------------------------------------------------------- B side
    const int qb = tid & 7, rb = tid >> 3;
    int bofs[BQ];
    const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * 4, 0x00020000);
    if (MODE == MODE_FWD) {
#pragma unroll
        for (int j = 0; j < BQ; ++j) {
            const int n = n0 + rb + 32 * j;
            bofs[j] = n < a.N ? (n * KT * a.C + 4 * qb) : -1;
        }
    } else {
        // k-row tiles [32][BN]: quad i = tid + 256 j covers columns n0 + 4 (i % (BN/4))
#pragma unroll
        for (int j = 0; j < BQ; ++j) {
            const int i = tid + kThreads * j, nq = i % (BN / 4);
            const int n = n0 + 4 * nq;
            bofs[j] = n < a.N ? n : -1;
        }
    }
    const int cchunks = (a.C + BK - 1) / BK;   // fwd / dgrad: chunks per tap

    f32x16 acc[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

    float4 ra0[AQ], rb0[BQ], ra1[AQ], rb1[BQ];

    // load chunk (t0 + t) into registers RA, RB
#define CONV_LOAD(t, RA, RB)                                                                                 \
    {                                                                                                        \
        const int tt_ = t0 + (t);                                                                            \
        if (MODE != MODE_WGRAD) {                                                                            \
            const int tap_ = tt_ / cchunks, c0_ = (tt_ - tap_ * cchunks) * BK;                               \
            const int kh_ = tap_ / a.KW, kw_ = tap_ - kh_ * a.KW;                                            \
            const int off_ = (kh_ * a.W + kw_) * a.C + c0_;                                                  \
            const bool cok_ = c0_ + 4 * qa < a.C;                                                            \
            _Pragma("unroll") for (int j = 0; j < AQ; ++j) {                                                 \
                const bool ok = cok_ && (unsigned)(aih[j] + kh_) < (unsigned)a.H &&                          \
                                (unsigned)(aiw[j] + kw_) < (unsigned)a.W;                                    \
                RA[j] = bload(ar, ok ? (apb[j] + off_) * 4 : kBad);                                          \
            }                                                                                                \
            if (MODE == MODE_FWD) {                                                                          \
                const int woff_ = tap_ * a.C + c0_;                                                          \
                const bool bok_ = c0_ + 4 * qb < a.C;                                                        \
                _Pragma("unroll") for (int j = 0; j < BQ; ++j)                                               \
                    RB[j] = bload(br, (bofs[j] >= 0 && bok_) ? (bofs[j] + woff_) * 4 : kBad);                \
            } else {                                                                                         \
                /* w[co = c0 + k][flipped tap][ci = n]: k row of BN contiguous ci */                         \
                const int ftap_ = KT - 1 - tap_;                                                             \
                _Pragma("unroll") for (int j = 0; j < BQ; ++j) {                                             \
                    const int k_ = (tid + kThreads * j) / (BN / 4);                                          \
                    const bool ok = bofs[j] >= 0 && c0_ + k_ < a.C;                                          \
                    RB[j] = bload(br, ok ? (((c0_ + k_) * KT + ftap_) * a.N + bofs[j]) * 4 : kBad);          \
                }                                                                                            \
            }                                                                                                \
        } else {                                                                                             \
            /* A: x at pixel (k row) shifted by the quad's tap; B: gy[pixel][co] */                          \
            _Pragma("unroll") for (int j = 0; j < AQ; ++j) {                                                 \
                int b_ = pb_b, oh_ = pb_oh, ow_ = pb_ow + j * (kThreads / (BM / 4));                         \
                while (ow_ >= a.Wo) { ow_ -= a.Wo; if (++oh_ == a.Ho) { oh_ = 0; ++b_; } }                    \
                const int ih_ = oh_ * a.stride - a.pad + wkh[j], iw_ = ow_ * a.stride - a.pad + wkw[j];      \
                const bool ok = b_ < a.B && (unsigned)ih_ < (unsigned)a.H && (unsigned)iw_ < (unsigned)a.W;  \
                RA[j] = bload(ar, ok ? (((b_ * a.H + ih_) * a.W + iw_) * a.C + wci[j]) * 4 : kBad);          \
            }                                                                                                \
            pb_ow += BK;                                                                                     \
            while (pb_ow >= a.Wo) { pb_ow -= a.Wo; if (++pb_oh == a.Ho) { pb_oh = 0; ++pb_b; } }             \
            const int p0_ = tt_ * BK;                                                                        \
            _Pragma("unroll") for (int j = 0; j < BQ; ++j) {                                                 \
                const int p_ = p0_ + (tid + kThreads * j) / (BN / 4);                                        \
                RB[j] = bload(br, (p_ < a.P && bofs[j] >= 0) ? (p_ * a.Cg + bofs[j]) * 4 : kBad);            \
            }                                                                                                \
        }                                                                                                    \
    }

    // registers -> LDS buffer `buf`
#define CONV_STORE(buf, RA, RB)                                                                              \
    {                                                                                                        \
        float* As_ = lds[buf];                                                                               \
        float* Bs_ = lds[buf] + G::A_FLOATS;                                                                 \
        _Pragma("unroll") for (int j = 0; j < AQ; ++j) {                                                     \
            if (G::A_ROWK) {                                                                                 \
                const int r_ = ra + 32 * j;                                                                  \
                *(float4*)(As_ + r_ * BK + 4 * swz(r_, qa)) = RA[j];                                         \
            } else {                                                                                         \
                *(float4*)(As_ + 4 * (tid + kThreads * j)) = RA[j];                                          \
            }                                                                                                \
        }                                                                                                    \
        _Pragma("unroll") for (int j = 0; j < BQ; ++j) {                                                     \
            if (G::B_ROWK) {                                                                                 \
                const int r_ = rb + 32 * j;                                                                  \
                *(float4*)(Bs_ + r_ * BK + 4 * swz(r_, qb)) = RB[j];                                         \
            } else {                                                                                         \
                *(float4*)(Bs_ + 4 * (tid + kThreads * j)) = RB[j];                                          \
            }                                                                                                \
        }                                                                                                    \
    }

    const int arow = wm * (TM * 32) + (lane & 31), brow = wn * (TN * 32) + (lane & 31);
    const int h = lane >> 5;
    // multiply the chunk in LDS buffer `buf`: MFMA j (j = 4 kq + e) takes k = 16 h + j
#define CONV_MMA(buf)                                                                                        \
    {                                                                                                        \
        const float* As_ = lds[buf];                                                                         \
        const float* Bs_ = lds[buf] + G::A_FLOATS;                                                           \
        _Pragma("unroll") for (int kq = 0; kq < 4; ++kq) {                                                   \
            float fa[TM][4], fb[TN][4];                                                                      \
            _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                                 \
                if (G::A_ROWK) {                                                                             \
                    const float4 v = *(const float4*)(As_ + (arow + 32 * i) * BK + 4 * swz(arow + 32 * i, 4 * h + kq)); \
                    fa[i][0] = v.x; fa[i][1] = v.y; fa[i][2] = v.z; fa[i][3] = v.w;                          \
                } else {                                                                                     \
                    _Pragma("unroll") for (int e = 0; e < 4; ++e)                                            \
                        fa[i][e] = As_[(16 * h + 4 * kq + e) * BM + arow + 32 * i];                          \
                }                                                                                            \
            }                                                                                                \
            _Pragma("unroll") for (int j = 0; j < TN; ++j) {                                                 \
                if (G::B_ROWK) {                                                                             \
                    const float4 v = *(const float4*)(Bs_ + (brow + 32 * j) * BK + 4 * swz(brow + 32 * j, 4 * h + kq)); \
                    fb[j][0] = v.x; fb[j][1] = v.y; fb[j][2] = v.z; fb[j][3] = v.w;                          \
                } else {                                                                                     \
                    _Pragma("unroll") for (int e = 0; e < 4; ++e)                                            \
                        fb[j][e] = Bs_[(16 * h + 4 * kq + e) * BN + brow + 32 * j];                          \
                }                                                                                            \
            }                                                                                                \
            _Pragma("unroll") for (int e = 0; e < 4; ++e)                                                    \
                _Pragma("unroll") for (int i = 0; i < TM; ++i)                                               \
                    _Pragma("unroll") for (int j = 0; j < TN; ++j)                                           \
                        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i][e], fb[j][e], acc[i][j], 0, 0, 0); \
        }                                                                                                    \
        asm volatile("" ::: "memory"); /* keep the next LDS writes behind these reads */                   \
    }

    CONV_LOAD(0, ra0, rb0);
    if (nchunks > 1) CONV_LOAD(1, ra1, rb1);
    CONV_STORE(0, ra0, rb0);
    __syncthreads();
    // iteration t: load t+2, multiply t (buffer t&1), store t+1, barrier
    int t = 0;
    for (; t + 1 < nchunks; t += 2) {
        if (t + 2 < nchunks) CONV_LOAD(t + 2, ra0, rb0);
        CONV_MMA(0);
        CONV_STORE(1, ra1, rb1);
        __syncthreads();
        if (t + 3 < nchunks) CONV_LOAD(t + 3, ra1, rb1);
        CONV_MMA(1);
        if (t + 2 < nchunks) CONV_STORE(0, ra0, rb0);
        __syncthreads();
    }
    if (t < nchunks) CONV_MMA(0);
#undef CONV_LOAD
#undef CONV_STORE
#undef CONV_MMA

    // C/D map of 32x32: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 (lane >> 5)
    float* out = a.y + (size_t)ks * a.M * a.N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
            const int n = n0 + wn * (TN * 32) + 32 * j + (lane & 31);
            if (n < a.N) {
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int m = m0 + wm * (TM * 32) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (m < a.M) out[MODE == MODE_WGRAD ? n * a.M + m : m * a.N + n] = acc[i][j][e];
                }
            }
        }
}

// ----------------------------------------------------------------------------
// Split-bf16 ("x6") forward: f32 operands split exactly into three bf16 planes
// (x = x0 + x1 + x2: 8 + 8 + 8 significand bits = all 24 of an f32; see split3), products by v_mfma_f32_32x32x16_bf16 keeping the six terms xi*yj with
// i + j <= 2 (the three dropped ones are below 2^-24 relative), f32 accumulation.
// Error per product <= ~3 * 2^-24 relative: f32-class accuracy (tests compare it
// with the exact-f32 MFMA path against an fp64 reference) at 6 bf16 MFMAs of 32
// cycles per 16 k instead of 8 f32 MFMAs of 64 cycles: 2.7x the MFMA rate.
// Block 128 x BN, 4 waves as 2 x 2 (wave tile 64 x BN/2), K chunks of 32 staged
// from f32 registers (split on the way) into LDS planes [row][32 k] bf16 whose 16-byte
// quads are XOR-swizzled by (row >> 2) & 3 (conflict-free ds_read_b128 fragments).
// ----------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
constexpr int XBK = 32;

// Exact three-way split by truncation: x0 = x with the low 16 bits cleared (the top 8
// significand bits), r1 = x - x0 exact (<= 16 significant bits), x1 = r1 truncated the
// same way, x2 = r1 - x1 exact with <= 8 significant bits, so its bf16 (the high half)
// is exact too: x == x0 + x1 + x2.  Pairs of elements are packed with one v_perm per
// plane (the high halves of two dwords).
__device__ __forceinline__ uint32_t hi16x2(float lo, float hi) {
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07060302u);
}
__device__ __forceinline__ float trunc16(float x) {
    return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & 0xFFFF0000u);
}
__device__ __forceinline__ void split3(float4 v, bf16x4& p0, bf16x4& p1, bf16x4& p2) {
    const float x[4] = {v.x, v.y, v.z, v.w};
    float a[4], b[4], c[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        a[i] = trunc16(x[i]);
        const float r1 = x[i] - a[i];
        b[i] = trunc16(r1);
        c[i] = r1 - b[i];
    }
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 q0, q1, q2;
    q0.x = hi16x2(a[0], a[1]), q0.y = hi16x2(a[2], a[3]);
    q1.x = hi16x2(b[0], b[1]), q1.y = hi16x2(b[2], b[3]);
    q2.x = hi16x2(c[0], c[1]), q2.y = hi16x2(c[2], c[3]);
    p0 = __builtin_bit_cast(bf16x4, q0);
    p1 = __builtin_bit_cast(bf16x4, q1);
    p2 = __builtin_bit_cast(bf16x4, q2);
}

// element index of (row r, k) in a [rows][32] bf16 plane, 16-byte quads swizzled
__device__ __forceinline__ int xidx(int r, int k) { return r * XBK + ((((k >> 3) ^ (r >> 2)) & 3) << 3) + (k & 7); }
// xidx with rows r and r ^ 1 swapped in every odd row quad: the same ds_read_b128
// banks as xidx (a fragment group's rows map onto the same row set), and an 8-byte
// store of row 4 q + j by the 16 lanes of two quads (q, q + 1) then lands on both
// 16-bank halves (row parity differs) instead of two-way on one
__device__ __forceinline__ int xidx2(int r, int k) { return xidx(r ^ ((r >> 2) & 1), k); }
// The 16x16x32 MFMA path's operand layout: k-octet slot kq ^ (row >> 2 & 2).  Its
// ds_read_b128 lane groups ({0-3, 12-15, 20-27}, ...) read rows c, 12 + c at one octet
// and 4 + c, 8 + c at the next, which xidx's kq ^ (row >> 2) puts on the same 16-byte
// bank slot (two-way on every fragment read); this slot function keeps all four apart.
template <int MT>
__device__ __forceinline__ int xsw(int r, int k) {
    if constexpr (MT == 32) return xidx(r, k);
    return r * XBK + ((((k >> 3) ^ ((r >> 2) & 2)) & 3) << 3) + (k & 7);
}

// Weights split once per call into three bf16 planes [3][R][KT][Ck] in row-k order:
// forward R = Co, Ck = Ci (w as is); input gradient R = Ci, Ck = Co with the taps
// flipped (the "full" convolution's operand), so both GEMMs read B as row-k.
__global__ __launch_bounds__(256) void conv_wsplit_kernel(const float* w, __bf16* out, int Co, int KT, int Ci,
                                                          int dgrad) {
    const int n = Co * KT * Ci;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float v;
    if (!dgrad) {
        v = w[i];
    } else {
        const int co = i % Co, rest = i / Co, t = rest % KT, ci = rest / KT;   // out [ci][t][co]
        v = w[((size_t)co * KT + (KT - 1 - t)) * Ci + ci];
    }
    const float a = trunc16(v), r1 = v - a, b = trunc16(r1), c = r1 - b;
    out[i] = __builtin_bit_cast(__bf16, (uint16_t)(__builtin_bit_cast(uint32_t, a) >> 16));
    out[n + i] = __builtin_bit_cast(__bf16, (uint16_t)(__builtin_bit_cast(uint32_t, b) >> 16));
    out[2 * n + i] = __builtin_bit_cast(__bf16, (uint16_t)(__builtin_bit_cast(uint32_t, c) >> 16));
}

// Both layouts in one launch (md2_conv_split_weights): one block per (tap, 32 co,
// 32 ci) tile.  The tile is read once, coalesced along ci, split into the forward
// planes [3][Co][KT][Ci] (same element order), and — if `dg` is non-null — transposed
// through LDS into the input gradient's [3][Ci][KT][Co] with the tap flipped, so
// those 2-byte stores coalesce along co as well.
__device__ __forceinline__ void split_store(__bf16* out, int n, int i, float v) {
    const float a = trunc16(v), r1 = v - a, b = trunc16(r1), c = r1 - b;
    out[i] = __builtin_bit_cast(__bf16, (uint16_t)(__builtin_bit_cast(uint32_t, a) >> 16));
    out[n + i] = __builtin_bit_cast(__bf16, (uint16_t)(__builtin_bit_cast(uint32_t, b) >> 16));
    out[2 * n + i] = __builtin_bit_cast(__bf16, (uint16_t)(__builtin_bit_cast(uint32_t, c) >> 16));
}
// A 32 (co) x 32 (ci) tile of one tap, split into the three bf16 planes of the
// forward layout [co][tap][ci] and (through LDS) of the input-gradient layout
// [ci][flipped tap][co] / the col layout [tap][ci][co].  With Ci and Co multiples of 4
// (every x6 convolution) a thread handles 4 consecutive elements along the contiguous
// index of each layout: one 16-byte load, and per plane one 8-byte store instead of
// four 2-byte ones (the step's one split launch ran at ~60 % of HBM bandwidth on 2-byte
// stores).  Same split (split3 = split_store's arithmetic), same bits.
// bf (MD2_CONV_BF16, md2_conv_bf16_weights): ONE plane per layout, the weight rounded to
// bf16 (nearest even) — the operand a bf16 autocast convolution multiplies
__device__ __forceinline__ bf16x4 rne4(float4 v) {
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    u32x2 q;
    q.x = (uint32_t)f2bf16(v.x) | ((uint32_t)f2bf16(v.y) << 16);
    q.y = (uint32_t)f2bf16(v.z) | ((uint32_t)f2bf16(v.w) << 16);
    return __builtin_bit_cast(bf16x4, q);
}
__device__ __forceinline__ void planes_store4(__bf16* out, int n, int i, float4 v, bool bf) {
    if (bf) {
        *(bf16x4*)(out + i) = rne4(v);
        return;
    }
    bf16x4 p0, p1, p2;
    split3(v, p0, p1, p2);
    *(bf16x4*)(out + i) = p0;
    *(bf16x4*)(out + n + i) = p1;
    *(bf16x4*)(out + 2 * n + i) = p2;
}
__device__ __forceinline__ void wsplit_tile(const float* w, __bf16* fw, __bf16* dg, __bf16* cl, int Co, int KT,
                                            int Ci, int tap, int co0, int ci0, float (*tile)[33], bool bf = false) {
    const int n = Co * KT * Ci;
    if ((Ci & 3) == 0 && (Co & 3) == 0) {   // block-uniform
        const int q = threadIdx.x & 7, r = threadIdx.x >> 3;   // 8 quads x 32 rows
        {
            const int co = co0 + r, ci = ci0 + 4 * q;
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            if (co < Co && ci < Ci) {   // Ci % 4 == 0: the whole quad is in range
                const int i = (co * KT + tap) * Ci + ci;
                v = *(const float4*)(w + i);
                planes_store4(fw, n, i, v, bf);
            }
            tile[r][4 * q] = v.x;
            tile[r][4 * q + 1] = v.y;
            tile[r][4 * q + 2] = v.z;
            tile[r][4 * q + 3] = v.w;
        }
        if (!dg && !cl) return;   // block-uniform
        __syncthreads();
        const int ci = ci0 + r, co = co0 + 4 * q;
        if (ci < Ci && co < Co) {
            const float4 v = make_float4(tile[4 * q][r], tile[4 * q + 1][r], tile[4 * q + 2][r], tile[4 * q + 3][r]);
            if (dg) planes_store4(dg, n, (ci * KT + (KT - 1 - tap)) * Co + co, v, bf);
            if (cl) planes_store4(cl, n, (tap * Ci + ci) * Co + co, v, bf);   // [(tap, ci)][co], not flipped
        }
        return;
    }
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int r = ty; r < 32; r += 8) {
        const int co = co0 + r, ci = ci0 + tx;
        float v = 0.f;
        if (co < Co && ci < Ci) {
            const int i = (co * KT + tap) * Ci + ci;
            v = w[i];
            split_store(fw, n, i, v);
        }
        tile[r][tx] = v;
    }
    if (!dg && !cl) return;   // block-uniform
    __syncthreads();
#pragma unroll
    for (int r = ty; r < 32; r += 8) {
        const int ci = ci0 + r, co = co0 + tx;
        if (ci < Ci && co < Co) {
            if (dg) split_store(dg, n, (ci * KT + (KT - 1 - tap)) * Co + co, tile[tx][r]);
            if (cl) split_store(cl, n, (tap * Ci + ci) * Co + co, tile[tx][r]);   // [(tap, ci)][co], not flipped
        }
    }
}

// md2_conv_split_weights_multi: the tile kernel's work for every weight of the step in
// one grid.  Block b belongs to the last entry whose block0 <= b (entries ascending;
// a binary search over <= a few hundred entries held in the kernel's scalar path).
__global__ __launch_bounds__(256) void conv_wsplit_multi_kernel(const md2_wsplit_entry* tab, int n, int bf = 0) {
    __shared__ float tile[32][33];
    const int b = blockIdx.x;
    int lo = 0, hi = n - 1;
    while (lo < hi) {   // largest e with tab[e].block0 <= b
        const int mid = (lo + hi + 1) >> 1;
        if (tab[mid].block0 <= b) lo = mid;
        else hi = mid - 1;
    }
    const md2_wsplit_entry e = tab[lo];
    const int nx = (e.ci + 31) / 32, ny = (e.co + 31) / 32;
    int t = b - e.block0;
    const int bx = t % nx;
    t /= nx;
    const int by = t % ny, tap = t / ny;
    wsplit_tile(e.weight, (__bf16*)e.planes_fwd, (__bf16*)e.planes_dgrad, (__bf16*)e.planes_col, e.co, e.kt, e.ci,
                tap, by * 32, bx * 32, tile, bf != 0);
}

__global__ __launch_bounds__(256) void conv_wsplit_tile_kernel(const float* w, __bf16* fw, __bf16* dg, int Co,
                                                               int KT, int Ci, int bf = 0) {
    __shared__ float tile[32][33];
    wsplit_tile(w, fw, dg, nullptr, Co, KT, Ci, blockIdx.z, blockIdx.y * 32, blockIdx.x * 32, tile, bf != 0);
}

// Tiles BMX x BN.  NT threads: 8 waves (2 x 4 / 4 x 2 / 2 x 4, wave tiles 64/128 x 32)
// whenever BN = 128 or BMX = 256, so that two waves share each SIMD and one's split
// VALU overlaps the other's MFMAs; 128 x 64 and 128 x 32 (the decoder's 16/32-channel
// convolutions, which waste 3/4 or 1/2 of a 64-wide tile) run 4 waves at two blocks
// per CU; 128 x 16 (16 output channels) multiplies with 16x16x32 MFMAs.  The 256-row tile loads 1.5x the bytes of the 128-row one for 2x the MFMA
// work.
template <int BN, int BMX>
struct X6Geo {
    static constexpr int NT = (BN == 128 || BMX == 256) ? 512 : 256;
    static constexpr int MT = BN == 16 ? 16 : 32;   // MFMA tile: 16x16x32 for 16 columns, else 32x32x16
    static constexpr int WN = BN / MT;            // waves along N (wave tile MT wide)
    static constexpr int WM = NT / 64 / WN;       // waves along M
    static constexpr int TM = BMX / MT / WM;      // MFMA row blocks per wave
    static constexpr int MINB = (BN <= 64 && BMX == 128) ? 2 : 1;
};

// Workgroup barrier that leaves LDS-DMA loads in flight: __syncthreads()'s fence
// would wait for every outstanding vector-memory op (vmcnt(0)) once LDS-DMA is in
// the kernel, draining the register prefetch of A; the DMA is ordered by explicit
// wait_vm<> calls instead.  The "memory" clobber keeps LDS accesses on their side.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }
template <int VM>
__device__ __forceinline__ void wait_vm() {
    static_assert(VM >= 0 && VM < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((VM & 0xF) | ((VM >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}
// 16 bytes per lane from the buffer at byte offset `voff` into LDS at lds + 16·lane
// (lds wave-uniform; an offset past the buffer writes zeros)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, void* lds, int voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}

// A (activations, NHWC f32, im2col rows) is split while staged; B comes pre-split
// (conv_wsplit_kernel) and goes straight from memory into the LDS tile by LDS-DMA
// (buffer_load_dwordx4 ... lds: no VGPRs, no ds_write), one chunk ahead.  Forward
// and stride-1 input gradient alike (ConvArgs as the f32 path builds them; b = the
// planes).
// BF (MD2_CONV_BF16): A holds bf16 activations and B ONE bf16 weight plane (the
// operands of a bf16 autocast convolution, config C5): A quads are 8-byte bf16 loads
// stored to LDS as they are (no split), one MFMA per fragment pair, f32 accumulation,
// the output rounded to bf16 (RNE) — the same tiles, pipeline and swizzles.
template <int BN, int BMX, bool BF = false>
__global__ __launch_bounds__((X6Geo<BN, BMX>::NT), (X6Geo<BN, BMX>::MINB)) void conv_x6_kernel(ConvArgs a_) {
    using G = X6Geo<BN, BMX>;
    constexpr int NT = G::NT, TM = G::TM;
    constexpr int NP = BF ? 1 : 3;                 // bf16 planes per operand
    constexpr int AQ = BMX * XBK / 4 / NT;         // 4-element quads of A per thread
    constexpr int NW = NT / 64, PIECES = NP * BN / 16;   // B: 1 KiB DMA pieces per chunk
    constexpr int BQ = (PIECES + NW - 1) / NW;          // pieces per wave (the last j partial)
    constexpr int PA = BMX * XBK, PB = BN * XBK;   // bf16 elements per plane
    static_assert(AQ * NT * 4 == BMX * XBK, "A staging must tile the chunk");
    __shared__ __bf16 lds[2][NP * (PA + PB)];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / G::WN, wn = wid % G::WN;
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    ConvArgs a = a_;
    if (a.ncls > 0) {   // this block's parity class (constant-index selects: no scratch array)
        int c = 0;
#pragma unroll
        for (int i = 1; i < 4; ++i) c += (i < a.ncls && blk >= a.cls_blk[i]) ? 1 : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (i == c) {
                blk -= a.cls_blk[i];
                a.py = a.cls_py[i];
                a.px = a.cls_px[i];
                a.kh0 = a.cls_kh0[i];
                a.kw0 = a.cls_kw0[i];
                a.ntw = a.cls_ntw[i];
                a.dy0 = a.cls_dy0[i];
                a.dx0 = a.cls_dx0[i];
                a.Ho = a.cls_Ho[i];
                a.Wo = a.cls_Wo[i];
                a.nchunks = a.cls_nchunks[i];
            }
        a.M = a.B * a.Ho * a.Wo;
        a.mblocks = (a.M + BMX - 1) / BMX;
        a.chunks_per_split = a.nchunks;
    }
    const int nb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int m0 = mb * BMX, n0 = nb * BN;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);
    const int KT = a.KH * a.KW;
    const int cchunks = (a.C + XBK - 1) / XBK;

    // A staging: rows ra + (NT/8) j of the tile, f32 quad qa (k = 4 qa .. 4 qa + 3)
    const int qa = tid & 7, ra = tid >> 3;
    int aih[AQ], aiw[AQ], apb[AQ];
    const __amdgpu_buffer_rsrc_t ar =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, a.a_elems * (BF ? 2 : 4), 0x00020000);
#pragma unroll
    for (int j = 0; j < AQ; ++j) {
        const int m = m0 + ra + (NT / 8) * j;
        if (m < a.M) {
            const int b = m / (a.Ho * a.Wo), rem = m - b * a.Ho * a.Wo;
            const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
            aih[j] = oh * a.stride - a.pad;
            aiw[j] = ow * a.stride - a.pad;
            apb[j] = ((b * a.H + aih[j]) * a.W + aiw[j]) * a.C + 4 * qa;
        } else {
            aih[j] = -(1 << 20);
            aiw[j] = 0;
            apb[j] = 0;
        }
    }
    // B staging by LDS-DMA: BQ pieces per wave and chunk, each 1 KiB = 16 rows of one
    // plane (64 B per row).  Lane l fills row 16 rb + l/4, quad slot l&3 — the slot
    // that xsw() gives k-quad (slot ^ (row >> 2)) & 3, or (slot ^ (row >> 2 & 2)) & 3 on
    // the 16x16 path — so the DMA's linear lane order writes the swizzled layout.
    constexpr int RB16 = BN / 16;
    int bsrc[BQ], bk8[BQ], bdst[BQ];
    const __amdgpu_buffer_rsrc_t br =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * 2, 0x00020000);
#pragma unroll
    for (int j = 0; j < BQ; ++j) {
        const int piece = wid + NW * j, pl = piece / RB16, rb = piece - pl * RB16;
        const int r = rb * 16 + (lane >> 2), q = ((lane & 3) ^ (G::MT == 16 ? (r >> 2) & 2 : r >> 2)) & 3;
        const int n = n0 + r;
        bk8[j] = 8 * q;
        bsrc[j] = n < a.N ? ((pl * a.N + n) * KT) * a.C + 8 * q : -1;
        bdst[j] = (NP * PA + pl * PB + rb * 16 * XBK) * 2;   // bytes into the buffer (wave-uniform)
    }

    constexpr int NACC = G::MT == 16 ? 4 : 16;
    typedef float accv __attribute__((ext_vector_type(NACC)));
    accv acc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < NACC; ++e) acc[i][e] = 0.f;

    using AReg = typename std::conditional<BF, uint2, float4>::type;   // one quad of A
    AReg fa0[AQ], fa1[AQ];
    auto load = [&](int t, AReg (&RA)[AQ]) {
        const int tt = t0 + t;
        const bool live = t < nchunks;
        int kh, kw, off;
        bool cok;
        if (a.par) {
            const int tc = tt / cchunks, c0 = (tt - tc * cchunks) * XBK;
            const int th = tc / a.ntw, tw = tc - th * a.ntw;
            kh = a.dy0 - th;   // gy row / column offsets of this tap (stride 1, pad 0 grid)
            kw = a.dx0 - tw;
            off = (kh * a.W + kw) * a.C + c0;
            cok = live && c0 + 4 * qa < a.C;
        } else if (a.flatk) {
            // this thread's 4 k of the chunk: one tap (C % 4 == 0), channels ci .. ci+3
            const int k = tt * XBK + 4 * qa, tap = k / a.C, ci = k - tap * a.C;
            kh = tap / a.KW;
            kw = tap - kh * a.KW;
            off = (kh * a.W + kw) * a.C + ci - 4 * qa;   // apb[] holds the + 4 qa
            cok = live && tap < KT;
        } else {
            const int tap = tt / cchunks, c0 = (tt - tap * cchunks) * XBK;
            kh = tap / a.KW;
            kw = tap - kh * a.KW;
            off = (kh * a.W + kw) * a.C + c0;
            cok = live && c0 + 4 * qa < a.C;
        }
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const bool ok = cok && (unsigned)(aih[j] + kh) < (unsigned)a.H && (unsigned)(aiw[j] + kw) < (unsigned)a.W;
            if constexpr (BF) RA[j] = bload8(ar, ok ? (apb[j] + off) * 2 : kBad);
            else RA[j] = bload(ar, ok ? (apb[j] + off) * 4 : kBad);
        }
    };
    // B of chunk t into LDS buffer `buf` (wave-uniform skip past the last chunk)
    auto dma = [&](int t, int buf) {
        if (t >= nchunks) return;
        const int tt = t0 + t;
        int tap = tt / cchunks;
        const int c0 = (tt - tap * cchunks) * XBK;
        if (a.par) {   // the class tap's index in the flipped [Ci][KT][Co] planes
            const int th = tap / a.ntw, tw = tap - th * a.ntw;
            tap = (a.KH - 1 - (a.kh0 + 2 * th)) * a.KW + (a.KW - 1 - (a.kw0 + 2 * tw));
        }
        // B rows are [tap][channel] contiguous: the chunk starts at k = tap C + c0, or
        // at 32 tt of the flattened index
        const int kofs = a.flatk ? tt * XBK : tap * a.C + c0;
        const int klim = a.flatk ? KT * a.C : tap * a.C + a.C;
        char* base = (char*)lds[buf];
#pragma unroll
        for (int j = 0; j < BQ; ++j) {
            if (PIECES % NW && wid + NW * j >= PIECES) break;   // wave-uniform
            const bool ok = bsrc[j] >= 0 && kofs + bk8[j] < klim;
            dma16(br, base + bdst[j], ok ? (bsrc[j] + kofs) * 2 : kBad);
        }
    };
    bf16x4 sa[AQ][NP];
    auto split = [&](const AReg (&RA)[AQ]) {
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            if constexpr (BF) sa[j][0] = __builtin_bit_cast(bf16x4, RA[j]);
            else split3(RA[j], sa[j][0], sa[j][1], sa[j][2]);
        }
    };
    auto store = [&](int buf) {
        __bf16* L = lds[buf];
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const int e = xsw<G::MT>(ra + (NT / 8) * j, 4 * qa);
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) *(bf16x4*)(L + pl * PA + e) = sa[j][pl];
        }
    };
    const int lr = lane & 31, h = lane >> 5;
    auto mma = [&](int buf) {
        const __bf16* L = lds[buf];
        if constexpr (G::MT == 16) {
            // 16x16x32: lane l holds row / column l & 15, k = 8 (l >> 4) .. + 7
            const int l16 = lane & 15, kq = lane >> 4;
            bf16x8 fb[NP];
            const int eb = xsw<16>(wn * 16 + l16, 8 * kq);
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) fb[pl] = *(const bf16x8*)(L + NP * PA + pl * PB + eb);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                bf16x8 fa[NP];
                const int e = xsw<16>(wm * (TM * 16) + 16 * i + l16, 8 * kq);
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) fa[pl] = *(const bf16x8*)(L + pl * PA + e);
                if constexpr (BF) {
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                } else {
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fb[0], acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[1], acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[2], acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[0], acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[1], acc[i], 0, 0, 0);
                    acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                }
            }
        } else {
#pragma unroll
            for (int s = 0; s < XBK / 16; ++s) {
                bf16x8 fb[NP];
                const int eb = xidx(wn * 32 + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) fb[pl] = *(const bf16x8*)(L + NP * PA + pl * PB + eb);
#pragma unroll
                for (int i = 0; i < TM; ++i) {
                    bf16x8 fa[NP];
                    const int e = xidx(wm * (TM * 32) + 32 * i + lr, 16 * s + 8 * h);
#pragma unroll
                    for (int pl = 0; pl < NP; ++pl) fa[pl] = *(const bf16x8*)(L + pl * PA + e);
                    if constexpr (BF) {
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                    } else {
                        // small terms first: x2y0, x1y1, x0y2, x1y0, x0y1, x0y0
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc[i], 0, 0, 0);
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc[i], 0, 0, 0);
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc[i], 0, 0, 0);
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc[i], 0, 0, 0);
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc[i], 0, 0, 0);
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                    }
                }
            }
        }
    };

    // A of chunk t+2 is fetched into registers while chunk t is multiplied; chunk t+1
    // (fetched one iteration earlier) is split beside the MFMAs and stored to the other
    // LDS buffer afterwards, where its B is DMA'd at the start of the iteration (that
    // buffer was released by the previous barrier); one barrier per chunk.  The DMA is
    // issued before the A loads, so vmcnt(AQ) before the barrier waits for the DMA
    // alone (vector-memory loads complete in order).  A loads past the last chunk read
    // zeros.
    // 8-wave blocks: the second-dispatched half (waves 4-7, each sharing a SIMD with
    // one of waves 0-3) loses every VALU arbitration at equal priority; one static
    // s_setprio for it (MI355X_MICROARCH.md, two waves per SIMD, item 4)
    if (NT == 512 && wid >= 4) __builtin_amdgcn_s_setprio(1);
    load(0, fa0);
    load(1, fa1);
    dma(0, 0);
    split(fa0);
    store(0);
    wait_vm<0>();
    lds_sync();
    for (int t = 0; t < nchunks; t += 2) {
        dma(t + 1, 1);
        load(t + 2, fa0);
        split(fa1);
        mma(0);
        asm volatile("" ::: "memory");
        store(1);
        wait_vm<AQ>();
        lds_sync();
        if (t + 1 >= nchunks) break;
        dma(t + 2, 0);
        load(t + 3, fa1);
        split(fa0);
        mma(1);
        asm volatile("" ::: "memory");
        store(0);
        wait_vm<AQ>();
        lds_sync();
    }

    float* out = a.y + (size_t)ks * a.M * a.N;
    // output row of GEMM pixel m: m itself, or its gx pixel for a stride-2 parity class
    // written in place (split partials stay class-ordered; the scatter reduce places them)
    auto orow = [&](int m) {
        if (!a.par || a.splits > 1) return m;
        const int hw = a.Ho * a.Wo, b = m / hw, rem = m - b * hw, oh = rem / a.Wo, ow = rem - oh * a.Wo;
        return (b * a.oHf + 2 * oh + a.py) * a.oWf + 2 * ow + a.px;
    };
    // BF without a K split: the bf16 output itself (round to nearest even)
    const bool obf = BF && a.ybf16 == 1 && a.splits == 1;
    auto put = [&](int m, int n, float v) {
        if (obf) ((uint16_t*)a.y)[orow(m) * a.N + n] = f2bf16(v);
        else out[orow(m) * a.N + n] = v;
    };
    if constexpr (G::MT == 16) {
        // 16x16 D: lane l holds column l & 15, rows 4 (l >> 4) .. + 3
        const int n = n0 + wn * 16 + (lane & 15);
        if (n < a.N) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int m = m0 + wm * (TM * 16) + 16 * i + 4 * (lane >> 4) + e;
                    if (m < a.M) put(m, n, acc[i][e]);
                }
        }
    } else {
        const int n = n0 + wn * 32 + lr;
        if (n < a.N) {
#pragma unroll
            for (int i = 0; i < TM; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int m = m0 + wm * (TM * 32) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (m < a.M) put(m, n, acc[i][e]);
                }
        }
    }
}

// Warp-specialised split-bf16 GEMM for the forward / stride-1 input gradient with a
// 128-wide tile (MD2_CONV_WS): the 8-wave block is 4 MFMA waves and 4 staging waves,
// one of each per SIMD (waves are dealt to the SIMDs round-robin: wave w and w + 4 share
// SIMD w).  conv_x6_kernel's 8 waves all stage and all multiply, in lockstep between
// two barriers per chunk pair, so a SIMD's split VALU, LDS stores and address math sit
// between its own MFMAs (its MFMA pipe measured 0.19-0.21 busy on the 12x40 / 6x20
// layers).  Here the MFMA wave of a SIMD only reads fragments and multiplies while the
// staging wave beside it fetches chunk t+2, splits and stores chunk t+1 and DMAs its
// weights — on the VALU, LDS and memory pipes, beside the matrix pipe.  One barrier per
// chunk hands the double-buffered LDS over.  MFMA wave tile (BMX/2) x 64: per 16 k,
// BMX/64 + 2 fragment triples for 6 (BMX/32) MFMAs (0.375 reads per MFMA at BMX = 256
// instead of 0.625).  Same operands, same products in the same order per output as
// conv_x6_kernel: bitwise equal results (tests/test_conv_gpu.py).
template <int BMX>
__global__ __launch_bounds__(512, 1) void conv_x6ws_kernel(ConvArgs a) {
    constexpr int BN = 128, NP = 256;              // tile width, staging threads
    constexpr int TMc = BMX / 64, TNc = 2;         // MFMA row / column blocks per MFMA wave
    constexpr int AQ = BMX * XBK / 4 / NP;         // f32 quads of A per staging thread
    constexpr int PIECES = 3 * BN / 16, BQ = PIECES / 4;   // B: 1 KiB DMA pieces per chunk / per staging wave
    constexpr int PA = BMX * XBK, PB = BN * XBK;
    static_assert(AQ * NP * 4 == BMX * XBK && BQ * 4 == PIECES, "staging must tile the chunk");
    __shared__ __bf16 lds[2][3 * (PA + PB)];

    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool mfma_wave = wid < 4;   // wave-uniform: scalar branches between the roles
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int nb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int m0 = mb * BMX, n0 = nb * BN;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);
    const int KT = a.KH * a.KW;
    const int cchunks = (a.C + XBK - 1) / XBK;

    // ---- staging waves: A rows ra + 32 j, f32 quad qa; B pieces sw + 4 j ----
    const int st = tid - 256, sw = wid - 4;
    const int qa = st & 7, ra = st >> 3;
    int aih[AQ], aiw[AQ], apb[AQ];
    int bsrc[BQ], bk8[BQ], bdst[BQ];
    const __amdgpu_buffer_rsrc_t ar = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, a.a_elems * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * 2, 0x00020000);
    if (!mfma_wave) {
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const int m = m0 + ra + (NP / 8) * j;
            if (m < a.M) {
                const int b = m / (a.Ho * a.Wo), rem = m - b * a.Ho * a.Wo;
                const int oh = rem / a.Wo, ow = rem - oh * a.Wo;
                aih[j] = oh * a.stride - a.pad;
                aiw[j] = ow * a.stride - a.pad;
                apb[j] = ((b * a.H + aih[j]) * a.W + aiw[j]) * a.C + 4 * qa;
            } else {
                aih[j] = -(1 << 20);
                aiw[j] = 0;
                apb[j] = 0;
            }
        }
#pragma unroll
        for (int j = 0; j < BQ; ++j) {
            const int piece = sw + 4 * j, pl = piece / (BN / 16), rb = piece - pl * (BN / 16);
            const int r = rb * 16 + (lane >> 2), q = ((lane & 3) ^ (r >> 2)) & 3;
            const int n = n0 + r;
            bk8[j] = 8 * q;
            bsrc[j] = n < a.N ? ((pl * a.N + n) * KT) * a.C + 8 * q : -1;
            bdst[j] = (3 * PA + pl * PB + rb * 16 * XBK) * 2;
        }
    }
    float4 RA[AQ];
    auto load = [&](int t) {
        const int tt = t0 + t;
        const int tap = tt / cchunks, c0 = (tt - tap * cchunks) * XBK;
        const int kh = tap / a.KW, kw = tap - kh * a.KW;
        const int off = (kh * a.W + kw) * a.C + c0;
        const bool cok = t < nchunks && c0 + 4 * qa < a.C;
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            const bool ok = cok && (unsigned)(aih[j] + kh) < (unsigned)a.H && (unsigned)(aiw[j] + kw) < (unsigned)a.W;
            RA[j] = bload(ar, ok ? (apb[j] + off) * 4 : kBad);
        }
    };
    auto dma = [&](int t, int buf) {   // every staging wave issues BQ pieces (zeros past the last chunk)
        const int tt = t0 + t;
        const int tap = tt / cchunks, c0 = (tt - tap * cchunks) * XBK;
        const int kofs = tap * a.C + c0, klim = tap * a.C + a.C;
        char* base = (char*)lds[buf];
#pragma unroll
        for (int j = 0; j < BQ; ++j) {
            const bool ok = t < nchunks && bsrc[j] >= 0 && kofs + bk8[j] < klim;
            dma16(br, base + bdst[j], ok ? (bsrc[j] + kofs) * 2 : kBad);
        }
    };
    auto split_store = [&](int buf) {
        __bf16* L = lds[buf];
#pragma unroll
        for (int j = 0; j < AQ; ++j) {
            bf16x4 p0, p1, p2;
            split3(RA[j], p0, p1, p2);
            const int e = xidx(ra + (NP / 8) * j, 4 * qa);
            *(bf16x4*)(L + e) = p0;
            *(bf16x4*)(L + PA + e) = p1;
            *(bf16x4*)(L + 2 * PA + e) = p2;
        }
    };

    // ---- MFMA waves: 2 x 2, wave tile (BMX/2) x 64 ----
    const int wm = wid >> 1, wn = wid & 1;
    const int lr = lane & 31, h = lane >> 5;
    f32x16 acc[TMc][TNc];
#pragma unroll
    for (int i = 0; i < TMc; ++i)
#pragma unroll
        for (int jn = 0; jn < TNc; ++jn)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][jn][e] = 0.f;
    auto mma = [&](int buf) {
        const __bf16* L = lds[buf];
#pragma unroll
        for (int s2 = 0; s2 < XBK / 16; ++s2) {
            bf16x8 fb[TNc][3];
#pragma unroll
            for (int jn = 0; jn < TNc; ++jn) {
                const int eb = xidx(wn * 64 + 32 * jn + lr, 16 * s2 + 8 * h);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) fb[jn][pl] = *(const bf16x8*)(L + 3 * PA + pl * PB + eb);
            }
#pragma unroll
            for (int i = 0; i < TMc; ++i) {
                bf16x8 fa[3];
                const int e = xidx(wm * (BMX / 2) + 32 * i + lr, 16 * s2 + 8 * h);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) fa[pl] = *(const bf16x8*)(L + pl * PA + e);
#pragma unroll
                for (int jn = 0; jn < TNc; ++jn) {
                    // small terms first: x2y0, x1y1, x0y2, x1y0, x0y1, x0y0 (conv_x6_kernel's order)
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[jn][0], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[jn][1], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[jn][2], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[jn][0], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[jn][1], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[jn][0], acc[i][jn], 0, 0, 0);
                }
            }
        }
    };

    // prologue: chunk 0 staged, chunk 1's A in registers
    if (!mfma_wave) {
        load(0);
        dma(0, 0);
        wait_vm<BQ>();   // A(0) landed (the DMA pieces were issued after it)
        split_store(0);
        load(1);
        wait_vm<AQ>();   // DMA(0) landed
    }
    lds_sync();
    for (int t = 0; t < nchunks; ++t) {
        if (mfma_wave) {
            mma(t & 1);
        } else if (t + 1 < nchunks) {
            // the other buffer was released by the last barrier: chunk t+1 into it
            dma(t + 1, (t + 1) & 1);
            wait_vm<BQ>();   // A(t+1), loaded during the previous chunk
            split_store((t + 1) & 1);
            load(t + 2);
            wait_vm<AQ>();   // DMA(t+1)
        }
        lds_sync();
    }
    if (!mfma_wave) return;

    float* out = a.y + (size_t)ks * a.M * a.N;
#pragma unroll
    for (int jn = 0; jn < TNc; ++jn) {
        const int n = n0 + wn * 64 + 32 * jn + lr;
        if (n >= a.N) continue;
#pragma unroll
        for (int i = 0; i < TMc; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + wm * (BMX / 2) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (m < a.M) out[(size_t)m * a.N + n] = acc[i][jn][e];
            }
    }
}

// Patch layout of the 16-column tiles (TC = 16): patch pixel pix = (pr, pc) at LDS row
// pix, k-octet slot kq ^ (pr & 1) ^ (pc >> 2 & 1) << 1.  A 32-lane fragment there spans
// two output rows (16 + 16 pixels, patch pitch 18), so a ds_read_b128 lane group reads
// columns x .. x+3, x+12 .. x+15 of one patch row and x+4 .. x+11 of the next, which
// xidx's kq ^ (pix >> 2) maps two-way onto the same bank slots; with this slot function
// the 16 lanes of every group hit 16 distinct slots at every tap offset (an exhaustive
// check over the row parities and tap columns chose it).  The 8-byte patch stores (two
// consecutive pixels per 16 lanes) stay conflict-free under any per-pixel permutation.
__device__ __forceinline__ int pidx16(int pix, int pr, int pc, int k) {
    const int sw = (pr & 1) ^ (((pc >> 2) & 1) << 1);
    return pix * XBK + ((((k >> 3) ^ sw) & 3) << 3) + (k & 7);
}

// Patch-staged split-bf16 3x3 stride-1 convolution (forward, and the stride-1 input
// gradient as the "full" convolution of gy with the flipped planes).  conv_x6_kernel
// stages its A tile per (tap, 32 channels) chunk: every activation is fetched, split and
// written to LDS nine times, once per tap.  Here a block owns a TR x TC rectangle of
// output pixels of one image; for every 32-channel chunk it stages the (TR+2) x (TC+2)
// input patch ONCE (one global fetch, one split, one LDS write per activation), and the
// nine taps read it at row / column offsets — the A fragment of tap (kh, kw) for output
// pixel (r, c) is patch pixel (r + kh, c + kw), the same [pixel][32 k] swizzled rows as
// conv_x6_kernel's tile, conflict-free at any offset (16-lane groups hit 16 distinct
// bank quads).  B (the weight planes of one tap) goes in by LDS-DMA, double-buffered
// across taps; one barrier per tap.  The next chunk's patch is fetched into registers
// behind tap 0's MFMAs and split / stored after tap 8.  A tiles of 128 or 256 pixels
// as TR x TC with TC in {16, 32, 64} chosen per shape (the least padding); outputs
// outside the image are not stored.  K splits run over channel chunks.
// BF (MD2_CONV_BF16): bf16 activations staged as they are (8-byte quads, one plane), one
// bf16 weight plane, one MFMA per fragment pair, the output rounded to bf16.
template <int BN, int BMX, int TC, bool BF = false>
__global__ __launch_bounds__((X6Geo<BN, BMX>::NT), 1) void conv_x6p_kernel(ConvArgs a) {
    using G = X6Geo<BN, BMX>;
    static_assert(G::MT == 32, "patch kernel: 32x32x16 MFMA tiles");
    constexpr int NT = G::NT, TM = G::TM;
    constexpr int NP = BF ? 1 : 3;
    constexpr int TR = BMX / TC, PW = TC + 2, PH = TR + 2, PP = PH * PW;
    constexpr int AQP = (PP * 8 + NT - 1) / NT;          // 4-channel quads of the patch per thread
    constexpr int NW = NT / 64, PIECES = NP * BN / 16;
    constexpr int BQ = (PIECES + NW - 1) / NW;
    constexpr int PA = PP * XBK, PB = BN * XBK;          // bf16 elements per plane
    // taps per barrier: the bf16 form (one MFMA per fragment pair) multiplies three taps'
    // weight tiles per LDS hand-over (a tap alone is ~128 MFMA cycles per wave, less
    // than the barrier and DMA round trip around it); the three-plane form one
    constexpr int TPS = BF ? 3 : 1, NGR = 9 / TPS;
    __shared__ __bf16 lds[NP * PA + 2 * TPS * NP * PB];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / G::WN, wn = wid % G::WN;
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int nb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int per_img = a.ptr * a.ptc;
    const int b = mb / per_img, trc = mb - b * per_img, tr = trc / a.ptc, tc = trc - tr * a.ptc;
    const int oh0 = tr * TR, ow0 = tc * TC, n0 = nb * BN;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);   // 32-channel chunks
    constexpr int KT = 9;

    // A: patch float4 f = tid + NT j -> pixel f / 8 (row-major PH x PW), channel quad f % 8
    int aofs[AQP];
    const __amdgpu_buffer_rsrc_t ar =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, a.a_elems * (BF ? 2 : 4), 0x00020000);
#pragma unroll
    for (int j = 0; j < AQP; ++j) {
        const int f = tid + NT * j, pix = f >> 3, q = f & 7;
        const int pr = pix / PW, pc = pix - pr * PW;
        const int ih = oh0 + pr - a.pad, iw = ow0 + pc - a.pad;
        const bool ok = f < PP * 8 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        aofs[j] = ok ? ((b * a.H + ih) * a.W + iw) * a.C + 4 * q : -1;
    }
    // B: as conv_x6_kernel (1 KiB LDS-DMA pieces, swizzle-ordered lanes)
    constexpr int RB16 = BN / 16;
    int bsrc[BQ], bk8[BQ], bdst[BQ];
    const __amdgpu_buffer_rsrc_t br = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * 2, 0x00020000);
#pragma unroll
    for (int j = 0; j < BQ; ++j) {
        const int piece = wid + NW * j, pl = piece / RB16, rb = piece - pl * RB16;
        const int r = rb * 16 + (lane >> 2), q = ((lane & 3) ^ (r >> 2)) & 3;
        const int n = n0 + r;
        bk8[j] = 8 * q;
        bsrc[j] = n < a.N ? ((pl * a.N + n) * KT) * a.C + 8 * q : -1;
        bdst[j] = (NP * PA + pl * PB + rb * 16 * XBK) * 2;
    }
    f32x16 acc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;

    using AReg = typename std::conditional<BF, uint2, float4>::type;
    AReg RA[AQP];
    auto load = [&](int t) {   // the patch of channel chunk t (zeros outside the image)
        const int c0 = (t0 + t) * XBK;
#pragma unroll
        for (int j = 0; j < AQP; ++j) {
            if constexpr (BF) RA[j] = bload8(ar, aofs[j] >= 0 ? (aofs[j] + c0) * 2 : kBad);
            else RA[j] = bload(ar, aofs[j] >= 0 ? (aofs[j] + c0) * 4 : kBad);
        }
    };
    auto store_patch = [&]() {
#pragma unroll
        for (int j = 0; j < AQP; ++j) {
            const int f = tid + NT * j;
            if (PP * 8 % NT && f >= PP * 8) break;
            bf16x4 p0, p1, p2;
            if constexpr (BF) p0 = __builtin_bit_cast(bf16x4, RA[j]);
            else split3(RA[j], p0, p1, p2);
            int e;
            if constexpr (TC == 16) {
                const int pix = f >> 3, pr = pix / PW;
                e = pidx16(pix, pr, pix - pr * PW, 4 * (f & 7));
            } else {
                e = xidx(f >> 3, 4 * (f & 7));
            }
            *(bf16x4*)(lds + e) = p0;
            if constexpr (!BF) {
                *(bf16x4*)(lds + PA + e) = p1;
                *(bf16x4*)(lds + 2 * PA + e) = p2;
            }
        }
    };
    auto dma = [&](int t, int tap, int slot) {   // B of (chunk t, tap) into B slot `slot`
        const int kofs = tap * a.C + (t0 + t) * XBK, klim = tap * a.C + a.C;
        char* base = (char*)lds + slot * NP * PB * 2;
#pragma unroll
        for (int j = 0; j < BQ; ++j) {
            if (PIECES % NW && wid + NW * j >= PIECES) break;   // wave-uniform
            const bool ok = bsrc[j] >= 0 && kofs + bk8[j] < klim;
            dma16(br, base + bdst[j], ok ? (bsrc[j] + kofs) * 2 : kBad);
        }
    };
    const int lr = lane & 31, h = lane >> 5;
    int abase[TM], arow[TM], acol[TM];   // this lane's patch pixel at tap (0, 0), per row fragment
#pragma unroll
    for (int i = 0; i < TM; ++i) {
        const int ml = wm * (TM * 32) + 32 * i + lr, r = ml / TC, c = ml - r * TC;
        abase[i] = r * PW + c;
        arow[i] = r;
        acol[i] = c;
    }
    // the TPS taps of group g of chunk t into buffer buf (slots buf TPS ..)
    auto dma_group = [&](int t, int g, int buf) {
#pragma unroll
        for (int u = 0; u < TPS; ++u) dma(t, g * TPS + u, buf * TPS + u);
    };
    auto mma = [&](int slot, int tap) {
        const __bf16* LB = lds + NP * PA + slot * NP * PB;
        const int th = tap / 3, tw = tap - 3 * th, toff = th * PW + tw;
#pragma unroll
        for (int s = 0; s < XBK / 16; ++s) {
            bf16x8 fb[NP];
            const int eb = xidx(wn * 32 + lr, 16 * s + 8 * h);
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) fb[pl] = *(const bf16x8*)(LB + pl * PB + eb);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                bf16x8 fa[NP];
                const int e = TC == 16 ? pidx16(abase[i] + toff, arow[i] + th, acol[i] + tw, 16 * s + 8 * h)
                                       : xidx(abase[i] + toff, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) fa[pl] = *(const bf16x8*)(lds + pl * PA + e);
                if constexpr (BF) {
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                    continue;
                } else {
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                }
            }
        }
    };

    if (NT == 512 && wid >= 4) __builtin_amdgcn_s_setprio(1);   // as conv_x6_kernel
    if (nchunks > 0) {
        load(0);
        dma_group(0, 0, 0);
        store_patch();
        wait_vm<0>();
        lds_sync();
    }
    int buf = 0;
    for (int t = 0; t < nchunks; ++t) {
        for (int g = 0; g < NGR; ++g) {
            const bool more = g + 1 < NGR || t + 1 < nchunks;
            if (more) dma_group(g + 1 < NGR ? t : t + 1, g + 1 < NGR ? g + 1 : 0, buf ^ 1);
            // the next patch behind group 0 (issued after the DMA: waiting for the DMA at the
            // end of this group leaves these loads in flight)
            if (g == 0 && t + 1 < nchunks) load(t + 1);
#pragma unroll
            for (int u = 0; u < TPS; ++u) mma(buf * TPS + u, g * TPS + u);
            asm volatile("" ::: "memory");
            if (g == 0 && t + 1 < nchunks) wait_vm<AQP>();
            else wait_vm<0>();
            lds_sync();
            buf ^= 1;
        }
        if (t + 1 < nchunks) {   // every wave is past tap 8: the patch can be replaced
            store_patch();
            lds_sync();
        }
    }

    float* out = a.y + (size_t)ks * a.M * a.N;
    const int n = n0 + wn * 32 + lr;
    if (n < a.N) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int ml = wm * (TM * 32) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                const int r = ml / TC, c = ml - r * TC, oh = oh0 + r, ow = ow0 + c;
                if (oh < a.Ho && ow < a.Wo) {
                    const size_t o = ((size_t)(b * a.Ho + oh) * a.Wo + ow) * a.N + n;
                    if (BF && a.ybf16 == 1 && a.splits == 1) ((uint16_t*)a.y)[o] = f2bf16(acc[i][e]);
                    else out[o] = acc[i][e];
                }
            }
    }
}

// Split-bf16 weight gradient: gw[co][tap][ci] = Σ_p gy[p][co] · x[p + tap][ci] as a
// GEMM with rows m = co, columns n = (tap, ci), K = output pixels.  Both operands are
// stored k-row in HBM (channels contiguous per pixel), the MFMA wants 8 consecutive k
// per lane: each staging thread loads a 4-pixel x 4-channel micro-tile (four 16-byte
// loads), splits it, and writes it transposed — per plane and channel one 8-byte run of
// 4 consecutive k — into the same swizzled [row][32 k] planes as the forward.
// 512 threads: waves 0-3 stage gy (A), waves 4-7 stage x (B); all 8 multiply (2 x 4,
// wave tile BMW/2 x 32).  BMW = 128 rows (co) per tile, or 64 for the 64-channel
// layers (half the MFMA work of a 128 tile there; only waves 0-1 stage gy, and two
// blocks fit a CU).  ConvArgs: M = Co, N = KT*Ci, P = pixels, C = Ci, Cg = Co.
// BF (MD2_CONV_BF16): x and gy are bf16 — a micro-tile is four 8-byte loads, repacked
// (not split) into one plane; one MFMA per fragment pair; the weight gradient (fp32
// accumulation, two-level as above) leaves as fp32 values rounded to bf16 (a bf16
// autocast convolution's weight gradient) — here without a K split, else in the
// reduction.
template <int BMW, bool XFAST, bool BF = false>
__global__ __launch_bounds__(512, (BMW == 64 ? 2 : 1)) void conv_x6_wgrad_kernel(ConvArgs a) {
    constexpr int NT = 512, BNW = 128, TM = BMW / 64;
    constexpr int NP = BF ? 1 : 3;
    constexpr int PA = BMW * XBK, PB = BNW * XBK;
    static_assert(BMW == 64 || BMW == 128, "wgrad row tile");
    __shared__ __bf16 lds[2][NP * (PA + PB)];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid >> 2, wn = wid & 3;
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int nb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int m0 = mb * BMW, n0 = nb * BNW;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);
    const int HoWo = a.Ho * a.Wo;
    const float rHoWo = 1.0f / (float)HoWo, rWo = 1.0f / (float)a.Wo;

    // staging role: side 0 (gy, rows co) or 1 (x, rows (tap, ci)); micro-tile
    // rows 4 mq .. 4 mq + 3, pixels 4 kq .. 4 kq + 3 of the chunk.  With BMW = 64 the
    // gy tile needs only threads 0-127: waves 2-3 stage nothing (wave-uniform)
    const int side = tid >> 8, u = tid & 255, kq = u & 7, mq = u >> 3;
    const int row = 4 * mq;
    const bool stager = side == 1 || u < 2 * BMW;
    int ci = 0, kh = 0, kw = 0;
    bool rok;
    if (side == 0) {
        rok = stager && m0 + row < a.M;
    } else {
        const int n = n0 + row;
        rok = n < a.N;
        const int tap = n / a.C;
        ci = n - tap * a.C;
        kh = tap / a.KW;
        kw = tap - kh * a.KW;
    }
    constexpr int ES = BF ? 2 : 4;   // operand element bytes
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, a.a_elems * ES, 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * ES, 0x00020000);

    // two-level accumulation: the MFMAs sum one chunk (32 pixels x 6 products) into
    // `acc`, which is then added into `tot` with rounded f32 adds — K here runs over
    // up to millions of pixels, and one MFMA accumulator over all of them drifts
    // (measured 1e-5 relative at 1.5 M pixels vs 4e-7 with this)
    f32x16 acc[TM], tot[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) tot[i][e] = 0.f;

    // x side with Wo % 4 == 0 (every encoder layer): a micro-tile's 4 output pixels
    // (p0 % 4 == 0) lie in one output row, so they share (b, oh) and their input
    // offsets step by stride·C.  (b, oh, ow) of p0 is walked XBK pixels per chunk
    // (load() is called for t = 0, 1, 2, ... in order) instead of two divisions and
    // three 32-bit multiplies per pixel (quarter-rate v_mul_lo_u32 / v_mad_u64_u32: the
    // x-staging waves issued ~1.6x the VALU of the gy-staging ones).
    constexpr bool xfast = XFAST;   // the host checks Wo % 4 == 0
    int wb = 0, woh = 0, wow = 0;
    if (side == 1 && xfast) {
        const int p = t0 * XBK + 4 * kq;
        wb = fdiv(p, HoWo, rHoWo);
        const int rem = p - wb * HoWo;
        woh = fdiv(rem, a.Wo, rWo);
        wow = rem - woh * a.Wo;
    }
    const int sC = a.stride * a.C;
    using VReg = typename std::conditional<BF, uint2, float4>::type;   // 4 channels of one pixel
    auto ld = [&](__amdgpu_buffer_rsrc_t r, int elem) -> VReg {
        if constexpr (BF) return bload8(r, elem == kBad ? kBad : elem * 2);
        else return bload(r, elem == kBad ? kBad : elem * 4);
    };
    auto load = [&](auto side_c, int t, VReg (&V)[4]) {
        constexpr int SIDE = decltype(side_c)::value;
        const int p0 = (t0 + t) * XBK + 4 * kq;
        const bool live = t < nchunks && rok;
        if constexpr (SIDE == 0) {
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int p = p0 + i;
                V[i] = ld(gr, (live && p < a.P) ? p * a.Cg + m0 + row : kBad);
            }
        } else if constexpr (xfast) {
            const int ih = woh * a.stride - a.pad + kh, iw0 = wow * a.stride - a.pad + kw;
            const bool rowok = live && p0 < a.P && (unsigned)ih < (unsigned)a.H;
            const int base = ((wb * a.H + ih) * a.W + iw0) * a.C + ci;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const bool ok = rowok && (unsigned)(iw0 + i * a.stride) < (unsigned)a.W;
                V[i] = ld(xr, ok ? base + i * sC : kBad);
            }
            wow += XBK;
            while (wow >= a.Wo) {
                wow -= a.Wo;
                if (++woh == a.Ho) {
                    woh = 0;
                    ++wb;
                }
            }
        } else {
            int b = fdiv(p0, HoWo, rHoWo);
            const int rem = p0 - b * HoWo;
            int oh = fdiv(rem, a.Wo, rWo), ow = rem - oh * a.Wo;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ih = oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
                const bool ok = live && p0 + i < a.P && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
                V[i] = ld(xr, ok ? ((b * a.H + ih) * a.W + iw) * a.C + ci : kBad);
                if (++ow == a.Wo) {
                    ow = 0;
                    if (++oh == a.Ho) {
                        oh = 0;
                        ++b;
                    }
                }
            }
        }
    };
    uint32_t pk[NP][4][2];   // plane, channel j, (k0k1, k2k3) packed bf16 pairs
    auto split = [&](const VReg (&V)[4]) {
        if constexpr (BF) {
            // channel j of pixels (0, 1) and (2, 3): the low / high halves of dword j / 2
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;
                const uint32_t d0 = (j < 2) ? V[0].x : V[0].y, d1 = (j < 2) ? V[1].x : V[1].y;
                const uint32_t d2 = (j < 2) ? V[2].x : V[2].y, d3 = (j < 2) ? V[3].x : V[3].y;
                pk[0][j][0] = __builtin_amdgcn_perm(d1, d0, sel);
                pk[0][j][1] = __builtin_amdgcn_perm(d3, d2, sel);
            }
            return;
        } else {
        float c[3][4][4];   // plane, pixel i, channel j
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float x[4] = {V[i].x, V[i].y, V[i].z, V[i].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a0 = trunc16(x[j]), r1 = x[j] - a0, a1 = trunc16(r1);
                c[0][i][j] = a0;
                c[1][i][j] = a1;
                c[2][i][j] = r1 - a1;
            }
        }
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                pk[pl][j][0] = hi16x2(c[pl][0][j], c[pl][1][j]);
                pk[pl][j][1] = hi16x2(c[pl][2][j], c[pl][3][j]);
            }
        }
    };
    auto store = [&](auto side_c, int buf) {
        constexpr int SIDE = decltype(side_c)::value;
        __bf16* L = lds[buf] + (SIDE ? NP * PA : 0);
        constexpr int P = SIDE ? PB : PA;
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
#pragma unroll
        for (int pl = 0; pl < NP; ++pl)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                u32x2 q;
                q.x = pk[pl][j][0];
                q.y = pk[pl][j][1];
                *(u32x2*)(L + pl * P + xidx2(row + j, 4 * kq)) = q;
            }
    };
    const int lr = lane & 31, h = lane >> 5;
    auto zero_acc = [&]() {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    };
    auto fold = [&]() {
#pragma unroll
        for (int i = 0; i < TM; ++i) tot[i] += acc[i];
    };
    auto mma = [&](int buf) {
        const __bf16* L = lds[buf];
#pragma unroll
        for (int s = 0; s < XBK / 16; ++s) {
            bf16x8 fa[TM][NP], fb[NP];
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                const int e = xidx2(wm * (TM * 32) + 32 * i + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) fa[i][pl] = *(const bf16x8*)(L + pl * PA + e);
            }
            const int eb = xidx2(wn * 32 + lr, 16 * s + 8 * h);
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) fb[pl] = *(const bf16x8*)(L + NP * PA + pl * PB + eb);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                if constexpr (BF) {
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[0], acc[i], 0, 0, 0);
                    continue;
                } else {
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[2], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[0], acc[i], 0, 0, 0);
                }
            }
        }
    };

    if (wid >= 4) __builtin_amdgcn_s_setprio(1);   // as in conv_x6_kernel
    // one loop per staging side (wave-uniform, compile-time inside): the step — fetch
    // chunk t+2, split chunk t+1, multiply chunk t, store chunk t+1 — is one basic block
    // the scheduler can interleave (the MFMA shadows hide the split VALU), as in
    // conv_x6pw_kernel's per-role loops
    auto run = [&](auto side_c) {
        VReg v0[4], v1[4];
        load(side_c, 0, v0);
        load(side_c, 1, v1);
        split(v0);
        store(side_c, 0);
        __syncthreads();
        for (int t = 0; t < nchunks; t += 2) {
            load(side_c, t + 2, v0);
            split(v1);
            zero_acc();
            mma(0);
            fold();
            asm volatile("" ::: "memory");
            store(side_c, 1);
            __syncthreads();
            if (t + 1 >= nchunks) break;
            load(side_c, t + 3, v1);
            split(v0);
            zero_acc();
            mma(1);
            fold();
            asm volatile("" ::: "memory");
            store(side_c, 0);
            __syncthreads();
        }
    };
    if (!stager) {
        // waves 2-3 at BMW = 64: multiply only
        __syncthreads();
        for (int t = 0; t < nchunks; t += 2) {
            zero_acc();
            mma(0);
            fold();
            __syncthreads();
            if (t + 1 >= nchunks) break;
            zero_acc();
            mma(1);
            fold();
            __syncthreads();
        }
    } else if (side == 0) {
        run(std::integral_constant<int, 0>());
    } else {
        run(std::integral_constant<int, 1>());
    }

    float* out = a.y + (size_t)ks * a.M * a.N;
    const int n = n0 + wn * 32 + lr;
    if (n < a.N) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + wm * (TM * 32) + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (m < a.M) out[m * a.N + n] = (BF && a.splits == 1) ? bf16_round(tot[i][e]) : tot[i][e];
            }
    }
}

// Warp-specialised split-bf16 weight gradient (MD2_CONV_X6 | MD2_CONV_WS, 128-row tiles).
// conv_x6_wgrad_kernel<128> has all 8 waves stage AND multiply between two barriers, so a
// SIMD's two waves split, store and wait on their loads in the same window as their MFMAs
// (profiles/r06: MFMA busy 0.35, a third of its wave cycles waiting).  Here waves 0-3
// only multiply (2 x 2, wave tile 64 x 64: per 16 k, 4 fragment triples for 24 MFMAs —
// 0.5 reads per MFMA instead of 0.75) and waves 4-7 (one per SIMD) stage both operands:
// each thread the gy AND the x micro-tile of conv_x6_wgrad_kernel's two staging sides.
// The staging waves keep two register sets: chunk t+2's loads are issued before chunk
// t+1 is split and stored (a whole chunk of MFMAs between a load and its use; three sets,
// loads two chunks ahead, measured 2-10 % slower per shape); one barrier per chunk hands
// the double-buffered LDS over.  Same tiles, swizzle, products,
// product order and two-level accumulation per output as conv_x6_wgrad_kernel<128>:
// bitwise equal results (tests/test_conv_gpu.py).
template <bool XFAST>
__global__ __launch_bounds__(512, 1) void conv_x6wws_kernel(ConvArgs a) {
    constexpr int BMW = 128, BNW = 128;
    constexpr int PA = BMW * XBK, PB = BNW * XBK;
    __shared__ __bf16 lds[2][3 * (PA + PB)];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool mfma_wave = wid < 4;
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int nb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int m0 = mb * BMW, n0 = nb * BNW;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);
    const int HoWo = a.Ho * a.Wo;
    const float rHoWo = 1.0f / (float)HoWo, rWo = 1.0f / (float)a.Wo;

    // ---- staging waves: micro-tile rows 4 mq .. 4 mq + 3 of both operands, pixels 4 kq .. ----
    const int st = tid - 256, kq = st & 7, mq = st >> 3, row = 4 * mq;
    const bool rokA = m0 + row < a.M;
    const int nrow = n0 + row;
    const bool rokB = nrow < a.N;
    const int tap = nrow / a.C, ci = nrow - tap * a.C;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, a.a_elems * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * 4, 0x00020000);
    int wb = 0, woh = 0, wow = 0;   // (b, oh, ow) of this thread's first pixel of the next x load
    if (XFAST && !mfma_wave) {
        const int p = t0 * XBK + 4 * kq;
        wb = fdiv(p, HoWo, rHoWo);
        const int rem = p - wb * HoWo;
        woh = fdiv(rem, a.Wo, rWo);
        wow = rem - woh * a.Wo;
    }
    const int sC = a.stride * a.C;
    // chunk t's gy quads (G) and x quads (X); called for t = 0, 1, 2, ... in order
    auto load = [&](int t, float4 (&G)[4], float4 (&X)[4]) {
        const int p0 = (t0 + t) * XBK + 4 * kq;
        const bool live = t < nchunks;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = p0 + i;
            G[i] = bload(gr, (live && rokA && p < a.P) ? (p * a.Cg + m0 + row) * 4 : kBad);
        }
        if constexpr (XFAST) {
            const int ih = woh * a.stride - a.pad + kh, iw0 = wow * a.stride - a.pad + kw;
            const bool rowok = live && rokB && p0 < a.P && (unsigned)ih < (unsigned)a.H;
            const int base = ((wb * a.H + ih) * a.W + iw0) * a.C + ci;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const bool ok = rowok && (unsigned)(iw0 + i * a.stride) < (unsigned)a.W;
                X[i] = bload(xr, ok ? (base + i * sC) * 4 : kBad);
            }
            wow += XBK;
            while (wow >= a.Wo) {
                wow -= a.Wo;
                if (++woh == a.Ho) {
                    woh = 0;
                    ++wb;
                }
            }
        } else {
            int b = fdiv(p0, HoWo, rHoWo);
            const int rem = p0 - b * HoWo;
            int oh = fdiv(rem, a.Wo, rWo), ow = rem - oh * a.Wo;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int ih = oh * a.stride - a.pad + kh, iw = ow * a.stride - a.pad + kw;
                const bool ok = live && rokB && p0 + i < a.P && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
                X[i] = bload(xr, ok ? (((b * a.H + ih) * a.W + iw) * a.C + ci) * 4 : kBad);
                if (++ow == a.Wo) {
                    ow = 0;
                    if (++oh == a.Ho) {
                        oh = 0;
                        ++b;
                    }
                }
            }
        }
    };
    // split a 4-pixel x 4-channel micro-tile into 3 planes and store it transposed (per
    // plane and channel one 8-byte run of 4 consecutive k) — conv_x6_wgrad_kernel's split
    auto split_store = [&](const float4 (&V)[4], __bf16* L, int P) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        float c[3][4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float x[4] = {V[i].x, V[i].y, V[i].z, V[i].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a0 = trunc16(x[j]), r1 = x[j] - a0, a1 = trunc16(r1);
                c[0][i][j] = a0;
                c[1][i][j] = a1;
                c[2][i][j] = r1 - a1;
            }
        }
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                u32x2 q;
                q.x = hi16x2(c[pl][0][j], c[pl][1][j]);
                q.y = hi16x2(c[pl][2][j], c[pl][3][j]);
                *(u32x2*)(L + pl * P + xidx2(row + j, 4 * kq)) = q;
            }
    };
    auto stage = [&](int buf, const float4 (&G)[4], const float4 (&X)[4]) {
        split_store(G, lds[buf], PA);
        split_store(X, lds[buf] + 3 * PA, PB);
    };

    // ---- MFMA waves: 2 x 2, wave tile 64 x 64 ----
    const int wm = wid >> 1, wn = wid & 1, lr = lane & 31, h = lane >> 5;
    f32x16 acc[2][2], tot[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jn = 0; jn < 2; ++jn)
#pragma unroll
            for (int e = 0; e < 16; ++e) tot[i][jn][e] = 0.f;
    auto mma = [&](int buf) {
        const __bf16* L = lds[buf];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jn = 0; jn < 2; ++jn)
#pragma unroll
                for (int e = 0; e < 16; ++e) acc[i][jn][e] = 0.f;
#pragma unroll
        for (int s = 0; s < XBK / 16; ++s) {
            bf16x8 fb[2][3];
#pragma unroll
            for (int jn = 0; jn < 2; ++jn) {
                const int eb = xidx2(wn * 64 + 32 * jn + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) fb[jn][pl] = *(const bf16x8*)(L + 3 * PA + pl * PB + eb);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                bf16x8 fa[3];
                const int e = xidx2(wm * 64 + 32 * i + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) fa[pl] = *(const bf16x8*)(L + pl * PA + e);
#pragma unroll
                for (int jn = 0; jn < 2; ++jn) {
                    // conv_x6_wgrad_kernel's order: x2y0, x1y1, x0y2, x1y0, x0y1, x0y0
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[jn][0], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[jn][1], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[jn][2], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[jn][0], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[jn][1], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[jn][0], acc[i][jn], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int jn = 0; jn < 2; ++jn) tot[i][jn] += acc[i][jn];
    };

    if (mfma_wave) {
        lds_sync();   // chunk 0 staged
        for (int t = 0; t < nchunks; ++t) {
            mma(t & 1);
            lds_sync();
        }
        float* out = a.y + (size_t)ks * a.M * a.N;
#pragma unroll
        for (int jn = 0; jn < 2; ++jn) {
            const int n = n0 + wn * 64 + 32 * jn + lr;
            if (n >= a.N) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int m = m0 + wm * 64 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (m < a.M) out[(size_t)m * a.N + n] = tot[i][jn][e];
                }
        }
        return;
    }
    // staging: register set c & 1 holds chunk c; the loop body is unrolled by two so the
    // sets are static
    float4 g0[4], x0[4], g1[4], x1[4];
    load(0, g0, x0);
    load(1, g1, x1);
    stage(0, g0, x0);
    lds_sync();
    for (int t = 0; t < nchunks; t += 2) {
        // MFMA waves on chunk t (buffer 0); chunk t+1 into buffer 1, chunk t+2's loads first
        if (t + 1 < nchunks) {
            load(t + 2, g0, x0);
            stage(1, g1, x1);
        }
        lds_sync();
        if (t + 1 >= nchunks) break;
        // chunk t+1 (buffer 1) being multiplied; chunk t+2 into buffer 0
        if (t + 2 < nchunks) {
            load(t + 3, g1, x1);
            stage(0, g0, x0);
        }
        lds_sync();
    }
}

// Warp-specialised weight gradient with a 256-wide tile (MD2_CONV_X6 | MD2_CONV_WS |
// MD2_CONV_BM256; more than 64 output channels): a block covers 128 output channels x 256
// (tap, ci) columns — two taps of a 128-channel layer — so each gy micro-tile staged
// feeds twice the MFMAs (48 KB fetched per 384 MFMAs instead of 32 KB per 192) and each
// barrier / pipe drain twice the work.  4 MFMA waves, wave tile 64 x 128 (per 16 k, 6
// fragment triples for 48 MFMAs: 0.375 reads per MFMA); 4 staging waves, each thread one
// gy and two x micro-tiles per chunk.  The wave tile's 8 accumulators fill 128 VGPRs, so
// there is no second accumulation level: the MFMAs sum a whole K split, which the host
// caps at 64 chunks (2,048 pixels, 128 MFMA k-steps; plan_x6w256) — f32-class against
// fp64 like the others (tests/test_conv_gpu.py), deterministic, not bitwise the
// two-level kernels.  LDS: 2 x 72 KB.  BF (MD2_CONV_BF16, config C5): bf16 x / gy
// repacked into one plane, one MFMA per fragment pair, the output rounded to bf16
// values (as conv_x6_wgrad_kernel's BF form; tests/test_conv_bf16_gpu.py).
template <bool XFAST, bool BF = false>
__global__ __launch_bounds__(512, 1) void conv_x6wws256_kernel(ConvArgs a) {
    constexpr int BMW = 128, BNW = 256;
    constexpr int NP = BF ? 1 : 3;   // bf16 planes per operand
    constexpr int PA = BMW * XBK, PB = BNW * XBK;
    // chunks per barrier (KS = 2 for bf16 measured 0-8 % slower: the bf16 form is bound
    // by its LDS traffic — one MFMA per fragment pair — not by the barriers)
    constexpr int KS = 1, SUB = NP * (PA + PB);
    __shared__ __bf16 lds[2][KS * SUB];
    const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool mfma_wave = wid < 4;
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int nb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int m0 = mb * BMW, n0 = nb * BNW;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);
    const int HoWo = a.Ho * a.Wo;
    const float rHoWo = 1.0f / (float)HoWo, rWo = 1.0f / (float)a.Wo;

    // ---- staging waves: gy rows 4 mq .., x rows 4 mq .. and 128 + 4 mq .., pixels 4 kq .. ----
    const int st = tid - 256, kq = st & 7, mq = st >> 3, row = 4 * mq;
    const bool rokA = m0 + row < a.M;
    bool rokB[2];
    int ci[2], kh[2], kw[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
        const int nrow = n0 + row + 128 * u;
        rokB[u] = nrow < a.N;
        const int tap = nrow / a.C;
        ci[u] = nrow - tap * a.C;
        kh[u] = tap / a.KW;
        kw[u] = tap - kh[u] * a.KW;
    }
    constexpr int ES = BF ? 2 : 4;   // operand element bytes
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, a.a_elems * ES, 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * ES, 0x00020000);
    using VReg = typename std::conditional<BF, uint2, float4>::type;   // 4 channels of one pixel
    auto ld = [&](__amdgpu_buffer_rsrc_t r, bool ok, int elem) -> VReg {
        if constexpr (BF) return bload8(r, ok ? elem * 2 : kBad);
        else return bload(r, ok ? elem * 4 : kBad);
    };
    int wb = 0, woh = 0, wow = 0;
    if (XFAST && !mfma_wave) {
        const int p = t0 * XBK + 4 * kq;
        wb = fdiv(p, HoWo, rHoWo);
        const int rem = p - wb * HoWo;
        woh = fdiv(rem, a.Wo, rWo);
        wow = rem - woh * a.Wo;
    }
    const int sC = a.stride * a.C;
    auto load = [&](int t, VReg (&G)[4], VReg (&X)[2][4]) {
        const int p0 = (t0 + t) * XBK + 4 * kq;
        const bool live = t < nchunks;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int p = p0 + i;
            G[i] = ld(gr, live && rokA && p < a.P, p * a.Cg + m0 + row);
        }
        if constexpr (XFAST) {
            const int oh_s = woh * a.stride - a.pad, ow_s = wow * a.stride - a.pad;
            const bool pok = live && p0 < a.P;
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int ih = oh_s + kh[u], iw0 = ow_s + kw[u];
                const bool rowok = pok && rokB[u] && (unsigned)ih < (unsigned)a.H;
                const int base = ((wb * a.H + ih) * a.W + iw0) * a.C + ci[u];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const bool ok = rowok && (unsigned)(iw0 + i * a.stride) < (unsigned)a.W;
                    X[u][i] = ld(xr, ok, base + i * sC);
                }
            }
            wow += XBK;
            while (wow >= a.Wo) {
                wow -= a.Wo;
                if (++woh == a.Ho) {
                    woh = 0;
                    ++wb;
                }
            }
        } else {
            int b = fdiv(p0, HoWo, rHoWo);
            const int rem = p0 - b * HoWo;
            int oh = fdiv(rem, a.Wo, rWo), ow = rem - oh * a.Wo;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
#pragma unroll
                for (int u = 0; u < 2; ++u) {
                    const int ih = oh * a.stride - a.pad + kh[u], iw = ow * a.stride - a.pad + kw[u];
                    const bool ok = live && rokB[u] && p0 + i < a.P && (unsigned)ih < (unsigned)a.H &&
                                    (unsigned)iw < (unsigned)a.W;
                    X[u][i] = ld(xr, ok, ((b * a.H + ih) * a.W + iw) * a.C + ci[u]);
                }
                if (++ow == a.Wo) {
                    ow = 0;
                    if (++oh == a.Ho) {
                        oh = 0;
                        ++b;
                    }
                }
            }
        }
    };
    auto split_store = [&](const VReg (&V)[4], __bf16* L, int P, int r0) {
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        if constexpr (BF) {
            // channel j of pixels (0, 1) and (2, 3): the low / high halves of dword j / 2
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t sel = (j & 1) ? 0x07060302u : 0x05040100u;
                const uint32_t d0 = (j < 2) ? V[0].x : V[0].y, d1 = (j < 2) ? V[1].x : V[1].y;
                const uint32_t d2 = (j < 2) ? V[2].x : V[2].y, d3 = (j < 2) ? V[3].x : V[3].y;
                u32x2 q;
                q.x = __builtin_amdgcn_perm(d1, d0, sel);
                q.y = __builtin_amdgcn_perm(d3, d2, sel);
                *(u32x2*)(L + xidx2(r0 + j, 4 * kq)) = q;
            }
            return;
        } else {
        float c[3][4][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float x[4] = {V[i].x, V[i].y, V[i].z, V[i].w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a0 = trunc16(x[j]), r1 = x[j] - a0, a1 = trunc16(r1);
                c[0][i][j] = a0;
                c[1][i][j] = a1;
                c[2][i][j] = r1 - a1;
            }
        }
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                u32x2 q;
                q.x = hi16x2(c[pl][0][j], c[pl][1][j]);
                q.y = hi16x2(c[pl][2][j], c[pl][3][j]);
                *(u32x2*)(L + pl * P + xidx2(r0 + j, 4 * kq)) = q;
            }
        }
    };
    // step j = chunks KS j .. KS j + KS - 1 (zeros past the split's last chunk)
    auto load_step = [&](int j, VReg (&G)[KS][4], VReg (&X)[KS][2][4]) {
#pragma unroll
        for (int u = 0; u < KS; ++u) load(KS * j + u, G[u], X[u]);
    };
    auto stage = [&](int buf, const VReg (&G)[KS][4], const VReg (&X)[KS][2][4]) {
#pragma unroll
        for (int u = 0; u < KS; ++u) {
            __bf16* L = lds[buf] + u * SUB;
            split_store(G[u], L, PA, row);
            split_store(X[u][0], L + NP * PA, PB, row);
            split_store(X[u][1], L + NP * PA, PB, row + 128);
        }
    };

    // ---- MFMA waves: 2 x 2, wave tile 64 x 128, one accumulation level ----
    const int wm = wid >> 1, wn = wid & 1, lr = lane & 31, h = lane >> 5;
    f32x16 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jn = 0; jn < 4; ++jn)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[i][jn][e] = 0.f;
    auto mma = [&](int buf) {
#pragma unroll
        for (int su = 0; su < KS * XBK / 16; ++su) {
            const __bf16* L = lds[buf] + (su / (XBK / 16)) * SUB;
            const int s = su % (XBK / 16);
            bf16x8 fa[2][NP];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int e = xidx2(wm * 64 + 32 * i + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) fa[i][pl] = *(const bf16x8*)(L + pl * PA + e);
            }
#pragma unroll
            for (int jn = 0; jn < 4; ++jn) {
                bf16x8 fb[NP];
                const int eb = xidx2(wn * 128 + 32 * jn + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) fb[pl] = *(const bf16x8*)(L + NP * PA + pl * PB + eb);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if constexpr (BF) {
                        acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[0], acc[i][jn], 0, 0, 0);
                        continue;
                    } else {
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][2], fb[0], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[1], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[2], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][1], fb[0], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[1], acc[i][jn], 0, 0, 0);
                    acc[i][jn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i][0], fb[0], acc[i][jn], 0, 0, 0);
                    }
                }
            }
        }
    };

    const int nsteps = (nchunks + KS - 1) / KS;
    if (mfma_wave) {
        lds_sync();   // step 0 staged
        for (int t = 0; t < nsteps; ++t) {
            mma(t & 1);
            lds_sync();
        }
        float* out = a.y + (size_t)ks * a.M * a.N;
#pragma unroll
        for (int jn = 0; jn < 4; ++jn) {
            const int n = n0 + wn * 128 + 32 * jn + lr;
            if (n >= a.N) continue;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int e = 0; e < 16; ++e) {
                    const int m = m0 + wm * 64 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                    if (m < a.M) out[(size_t)m * a.N + n] = (BF && a.splits == 1) ? bf16_round(acc[i][jn][e]) : acc[i][jn][e];
                }
        }
        return;
    }
    VReg g0[KS][4], x0[KS][2][4], g1[KS][4], x1[KS][2][4];
    load_step(0, g0, x0);
    load_step(1, g1, x1);
    stage(0, g0, x0);
    lds_sync();
    for (int t = 0; t < nsteps; t += 2) {
        if (t + 1 < nsteps) {
            load_step(t + 2, g0, x0);
            stage(1, g1, x1);
        }
        lds_sync();
        if (t + 1 >= nsteps) break;
        if (t + 2 < nsteps) {
            load_step(t + 3, g1, x1);
            stage(0, g0, x0);
        }
        lds_sync();
    }
}

// Patch-staged split-bf16 weight gradient (MD2_CONV_X6 | MD2_CONV_PATCH; 3x3, stride 1).
// conv_x6_wgrad_kernel stages x once per (tap, ci) column, so every activation is
// fetched and split nine times.  Here a K chunk is one 32-pixel segment of one output
// row: its three input rows x 34 columns x 32 channels are fetched and split ONCE and
// written as nine [32 ci][32 k] tiles — input row kh, columns shifted by kw, i.e. the B
// operand of tap (kh, kw), 16-byte aligned for the fragment reads.  Block tile: BMW
// output channels (rows, A = gy) x 9 taps x 32 input channels; nine waves, wave w
// multiplies tap w (TM = BMW / 32 row fragments).  Staging: waves 0-2 the x rows (a
// lane loads 6 pixels x 4 channels to fill the three shifted copies of 4 positions),
// waves 3-4 (3 at BMW = 32) the gy tile; LDS double-buffered, one barrier per chunk.
// K splits run over the chunks; output and partials as conv_x6_wgrad_kernel.
// ConvArgs: M = Co, N = 9 Ci, C = Ci, Cg = Co, nblocks = 32-channel groups of Ci,
// ptc = 32-column segments per output row, nchunks = B Ho ptc.
// BF (MD2_CONV_BF16): bf16 x / gy, one plane (repacked, not split), one MFMA per
// fragment pair, the output rounded to bf16 values (as conv_x6_wgrad_kernel's BF form).
template <int BMW, bool BF = false>
__global__ __launch_bounds__(576, 1) void conv_x6pw_kernel(ConvArgs a) {
    constexpr int TM = BMW / 32;
    constexpr int NP = BF ? 1 : 3;
    constexpr int PA = BMW * XBK, PT = 32 * XBK;   // bf16 per A plane / per B tile plane
    constexpr int BUF = NP * PA + 9 * NP * PT;
    static_assert(BMW == 32 || BMW == 64, "wgrad patch row tile");
    __shared__ __bf16 lds[2 * BUF];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    int blk = xcd_contiguous_block(blockIdx.x, gridDim.x);
    const int cb = blk % a.nblocks;
    blk /= a.nblocks;
    const int mb = blk % a.mblocks, ks = blk / a.mblocks;
    const int m0 = mb * BMW, c0 = cb * XBK;
    const int t0 = ks * a.chunks_per_split;
    const int nchunks = min(a.chunks_per_split, a.nchunks - t0);
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

    // staging roles by wave (the x rows on waves 0-2, the gy tile on 3-4; measured 4 %
    // faster than keeping the three waves that share a SIMD, 0 / 4 / 8, free of staging)
    const int rr = wid, g = lane & 7, q = lane >> 3;        // x: input row rr, columns 4g .., channels 4q ..
    const int u = tid - 192, kq = u & 7, mq = u >> 3;       // gy: pixels 4kq .., channels 4mq ..
    constexpr int ES = BF ? 2 : 4;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)a.a, 0, a.a_elems * ES, 0x00020000);
    const __amdgpu_buffer_rsrc_t gr = __builtin_amdgcn_make_buffer_rsrc((void*)a.b, 0, a.b_elems * ES, 0x00020000);

    // the loader's chunk position (b, oh, seg), advanced one chunk at a time
    int pc = t0, pseg, poh, pb;
    {
        const int r = pc / a.ptc;
        pseg = pc - r * a.ptc;
        pb = r / a.Ho;
        poh = r - pb * a.Ho;
    }
    auto advance = [&]() {
        ++pc;
        if (++pseg == a.ptc) {
            pseg = 0;
            if (++poh == a.Ho) {
                poh = 0;
                ++pb;
            }
        }
    };
    using VReg = typename std::conditional<BF, uint2, float4>::type;   // 4 channels of one pixel
    VReg V[6];
    auto ld = [&](__amdgpu_buffer_rsrc_t r, bool ok, int elem) -> VReg {
        if constexpr (BF) return bload8(r, ok ? elem * 2 : kBad);
        else return bload(r, ok ? elem * 4 : kBad);
    };
    // channel j of pixels i and i + 1 as one bf16 pair (BF)
    auto pair16 = [&](int j, int i) -> uint32_t {
        if constexpr (BF) {
            const uint32_t d0 = (j < 2) ? V[i].x : V[i].y, d1 = (j < 2) ? V[i + 1].x : V[i + 1].y;
            return __builtin_amdgcn_perm(d1, d0, (j & 1) ? 0x07060302u : 0x05040100u);
        } else {
            return 0u;
        }
    };
    // loads of the loader's chunk (zeros past the split's last chunk: no branch)
    auto load_x = [&]() {
        const int ih = poh - a.pad + rr, iw0 = pseg * 32 - a.pad + 4 * g;
        const bool rok = pc < t0 + nchunks && c0 + 4 * q < a.C && (unsigned)ih < (unsigned)a.H;
        const int base = ((pb * a.H + ih) * a.W) * a.C + c0 + 4 * q;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int iw = iw0 + i;
            V[i] = ld(xr, rok && (unsigned)iw < (unsigned)a.W, base + iw * a.C);
        }
    };
    auto load_g = [&]() {
        const int ow0 = pseg * 32 + 4 * kq;
        const bool ok = pc < t0 + nchunks && m0 + 4 * mq < a.M;
        const int base = ((pb * a.Ho + poh) * a.Wo) * a.Cg + m0 + 4 * mq;
#pragma unroll
        for (int i = 0; i < 4; ++i) V[i] = ld(gr, ok && ow0 + i < a.Wo, base + (ow0 + i) * a.Cg);
    };
    auto store_x = [&](__bf16* L) {
        if constexpr (BF) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                uint32_t w[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) w[k] = pair16(j, k);
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    u32x2 v;
                    v.x = w[kw];
                    v.y = w[kw + 2];
                    *(u32x2*)(L + PA + (kw * 3 + rr) * PT + xidx2(4 * q + j, 4 * g)) = v;
                }
            }
            return;
        } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float c[3][6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const float x = j == 0 ? V[i].x : (j == 1 ? V[i].y : (j == 2 ? V[i].z : V[i].w));
                const float a0 = trunc16(x), r1 = x - a0, a1 = trunc16(r1);
                c[0][i] = a0;
                c[1][i] = a1;
                c[2][i] = r1 - a1;
            }
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                uint32_t w[5];
#pragma unroll
                for (int k = 0; k < 5; ++k) w[k] = hi16x2(c[pl][k], c[pl][k + 1]);
#pragma unroll
                for (int kw = 0; kw < 3; ++kw) {
                    u32x2 v;
                    v.x = w[kw];
                    v.y = w[kw + 2];
                    *(u32x2*)(L + 3 * PA + ((kw * 3 + rr) * 3 + pl) * PT + xidx2(4 * q + j, 4 * g)) = v;
                }
            }
        }
        }
    };
    auto store_g = [&](__bf16* L) {
        if constexpr (BF) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                u32x2 v;
                v.x = pair16(j, 0);
                v.y = pair16(j, 2);
                *(u32x2*)(L + xidx2(4 * mq + j, 4 * kq)) = v;
            }
            return;
        } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float c[3][4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float x = j == 0 ? V[i].x : (j == 1 ? V[i].y : (j == 2 ? V[i].z : V[i].w));
                const float a0 = trunc16(x), r1 = x - a0, a1 = trunc16(r1);
                c[0][i] = a0;
                c[1][i] = a1;
                c[2][i] = r1 - a1;
            }
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                u32x2 v;
                v.x = hi16x2(c[pl][0], c[pl][1]);
                v.y = hi16x2(c[pl][2], c[pl][3]);
                *(u32x2*)(L + pl * PA + xidx2(4 * mq + j, 4 * kq)) = v;
            }
        }
        }
    };

    const int lr = lane & 31, h = lane >> 5;
    const int kh = wid / 3, kw = wid - 3 * kh;
    // one accumulator per row fragment over the whole split: plan_x6pw caps a split at
    // kX6pwMaxChunks chunks (2048 pixels), short enough for the MFMA's f32 accumulation
    f32x16 acc[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    const int boff = NP * PA + (kw * 3 + kh) * NP * PT;
    auto mma = [&](const __bf16* L) {
#pragma unroll
        for (int s = 0; s < XBK / 16; ++s) {
            bf16x8 fb[NP];
            const int eb = boff + xidx2(lr, 16 * s + 8 * h);
#pragma unroll
            for (int pl = 0; pl < NP; ++pl) fb[pl] = *(const bf16x8*)(L + pl * PT + eb);
#pragma unroll
            for (int i = 0; i < TM; ++i) {
                bf16x8 fa[NP];
                const int e = xidx2(32 * i + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < NP; ++pl) fa[pl] = *(const bf16x8*)(L + pl * PA + e);
                if constexpr (BF) {
                    acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                    continue;
                } else {
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
                }
            }
        }
    };

    // One loop per staging role (wave-uniform), so that a step — multiply the chunk in
    // one buffer, split / store the next one (in registers) into the other, fetch the
    // one after — is one basic block the scheduler can interleave (MFMA shadows hide
    // the split VALU).  Every role runs the same number of barriers.
    auto run = [&](auto role_c) {
        constexpr int ROLE = decltype(role_c)::value;   // 0: x rows, 1: gy, 2: multiply only
        auto load = [&]() {
            if constexpr (ROLE == 0) load_x();
            else if constexpr (ROLE == 1) load_g();
        };
        auto store = [&](__bf16* L) {
            if constexpr (ROLE == 0) store_x(L);
            else if constexpr (ROLE == 1) store_g(L);
        };
        load();                 // chunk 0
        store(lds);
        advance();
        load();                 // chunk 1
        lds_sync();
        int t = 0;
        for (; t + 2 < nchunks; t += 2) {
            mma(lds);
            store(lds + BUF);   // chunk t + 1
            advance();
            load();             // chunk t + 2
            lds_sync();
            mma(lds + BUF);
            store(lds);         // chunk t + 2
            advance();
            load();             // chunk t + 3 (zeros past the end)
            lds_sync();
        }
        if (t + 1 < nchunks) {
            mma(lds);
            store(lds + BUF);
            lds_sync();
            mma(lds + BUF);
        } else if (t < nchunks) {
            mma(lds);
        }
    };
    if (wid < 3) run(std::integral_constant<int, 0>());
    else if (tid < 192 + 2 * BMW) run(std::integral_constant<int, 1>());
    else run(std::integral_constant<int, 2>());

    float* out = a.y + (size_t)ks * a.M * a.N;
    const int ci = c0 + lr;
    if (ci < a.C) {
        const int n = (kh * 3 + kw) * a.C + ci;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int m = m0 + 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (m < a.M) out[m * a.N + n] = (BF && a.splits == 1) ? bf16_round(acc[i][e]) : acc[i][e];
            }
    }
}

// y = Σ_split partial[split], deterministic: 64 float4 outputs per block, four lanes
// per output summing every 4th split, then the four lane sums added in lane order.
// (One thread per output walked all splits — up to ~60 in the weight gradients — as
// one serial chain over a few dozen blocks.)
constexpr int kRedOut = 64, kRedLanes = 256 / kRedOut;
// OUT outputs per block, 256 / OUT lanes each: 64 for wide partials with few splits,
// 16 (sixteen lanes, each every 16th split) for the weight gradients' narrow ones with
// many splits, which at 64 per block ran a few dozen blocks of long serial chains
// OM: the output as fp32 (0), as bf16 bits (1: a bf16 convolution's activations, RNE)
// or as fp32 rounded to bf16 values (2: a bf16 convolution's weight gradient)
template <int OUT, int OM = 0>
__global__ __launch_bounds__(256) void conv_reduce_kernel(const float4* part, float4* y, int n4, int splits) {
    constexpr int LANES = 256 / OUT;
    __shared__ float4 red[LANES][OUT];
    const int o = threadIdx.x % OUT, l = threadIdx.x / OUT;
    const int i = blockIdx.x * OUT + o;
    float4 s = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
#pragma unroll 4
        for (int k = l; k < splits; k += LANES) {
            const float4 v = part[(size_t)k * n4 + i];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
    }
    red[l][o] = s;
    __syncthreads();
    if (l == 0 && i < n4) {
#pragma unroll
        for (int j = 1; j < LANES; ++j) {
            const float4 v = red[j][o];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        if constexpr (OM == 1) {
            ((uint2*)y)[i] = make_uint2((uint32_t)f2bf16(s.x) | ((uint32_t)f2bf16(s.y) << 16),
                                        (uint32_t)f2bf16(s.z) | ((uint32_t)f2bf16(s.w) << 16));
        } else if constexpr (OM == 2) {
            y[i] = make_float4(bf16_round(s.x), bf16_round(s.y), bf16_round(s.z), bf16_round(s.w));
        } else {
            y[i] = s;
        }
    }
}

template <int OM>
void launch_reduce_om(const float4* part, float4* y, int n4, int splits, hipStream_t st) {
    if (splits >= 16 && (n4 + kRedOut - 1) / kRedOut < 512)
        hipLaunchKernelGGL((conv_reduce_kernel<16, OM>), dim3((n4 + 15) / 16), dim3(256), 0, st, part, y, n4, splits);
    else
        hipLaunchKernelGGL((conv_reduce_kernel<kRedOut, OM>), dim3((n4 + kRedOut - 1) / kRedOut), dim3(256), 0, st,
                           part, y, n4, splits);
}
void launch_reduce(const float4* part, float4* y, int n4, int splits, hipStream_t st, int om = 0) {
    if (om == 1) launch_reduce_om<1>(part, y, n4, splits, st);
    else if (om == 2) launch_reduce_om<2>(part, y, n4, splits, st);
    else launch_reduce_om<0>(part, y, n4, splits, st);
}

// conv_reduce_kernel for a stride-2 parity class: class-ordered partials [splits][M][N]
// summed the same way, each output quad written to its gx pixel
template <int OM = 0>   // OM 1: bf16 output (MD2_CONV_BF16)
__global__ __launch_bounds__(256) void conv_reduce_scatter_kernel(const float4* part, float4* y, int n4, int splits,
                                                                   int N4, int Hc, int Wc, int oHf, int oWf, int py,
                                                                   int px) {
    __shared__ float4 red[kRedLanes][kRedOut];
    const int o = threadIdx.x % kRedOut, l = threadIdx.x / kRedOut;
    const int i = blockIdx.x * kRedOut + o;
    float4 s = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
        for (int k = l; k < splits; k += kRedLanes) {
            const float4 v = part[(size_t)k * n4 + i];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
    }
    red[l][o] = s;
    __syncthreads();
    if (l == 0 && i < n4) {
#pragma unroll
        for (int j = 1; j < kRedLanes; ++j) {
            const float4 v = red[j][o];
            s.x += v.x;
            s.y += v.y;
            s.z += v.z;
            s.w += v.w;
        }
        const int m = i / N4, q = i - m * N4, hw = Hc * Wc, b = m / hw, rem = m - b * hw, oh = rem / Wc,
                  ow = rem - oh * Wc;
        const size_t o = ((size_t)(b * oHf + 2 * oh + py) * oWf + 2 * ow + px) * N4 + q;
        if constexpr (OM == 1)
            ((uint2*)y)[o] = make_uint2((uint32_t)f2bf16(s.x) | ((uint32_t)f2bf16(s.y) << 16),
                                        (uint32_t)f2bf16(s.z) | ((uint32_t)f2bf16(s.w) << 16));
        else
            y[o] = s;
    }
}

bool valid(const md2_conv_desc* d) {
    if (!d) return false;
    if (d->batch < 1 || d->height < 1 || d->width < 1) return false;
    if (d->in_channels < 4 || d->in_channels % 4 || d->out_channels < 4 || d->out_channels % 4) return false;
    if (d->kernel_h < 1 || d->kernel_w < 1 || d->stride < 1 || d->pad < 0) return false;
    if (d->pad >= d->kernel_h || d->pad >= d->kernel_w) return false;
    const long long ho = (d->height + 2ll * d->pad - d->kernel_h) / d->stride + 1;
    const long long wo = (d->width + 2ll * d->pad - d->kernel_w) / d->stride + 1;
    if (ho < 1 || wo < 1) return false;
    if ((long long)d->batch * d->height * d->width * d->in_channels >= (1ll << 29)) return false;
    if ((long long)d->batch * ho * wo * d->out_channels >= (1ll << 29)) return false;
    if ((long long)d->out_channels * d->kernel_h * d->kernel_w * d->in_channels >= (1ll << 29)) return false;
    return true;
}

struct Shape {
    int B, H, W, C, N, KH, KW, s, p, Ho, Wo;
};

Shape shape_of(const md2_conv_desc* d) {
    Shape s;
    s.B = d->batch;
    s.H = d->height;
    s.W = d->width;
    s.C = d->in_channels;
    s.N = d->out_channels;
    s.KH = d->kernel_h;
    s.KW = d->kernel_w;
    s.s = d->stride;
    s.p = d->pad;
    s.Ho = (s.H + 2 * s.p - s.KH) / s.s + 1;
    s.Wo = (s.W + 2 * s.p - s.KW) / s.s + 1;
    return s;
}

int resident_blocks(int BN) { return 256 * (BN == 128 ? 2 : (BN == 64 ? 3 : 4)); }   // 256 CUs

// Tile width and K split from a wave-quantisation model: time ~ rounds of resident
// blocks x chunks per block x tile width, plus a small charge per split for the
// partials' round trip.  Forced by MD2_CONV_TILE_* / MD2_CONV_NO_SPLIT.
void plan(ConvArgs& a, uint32_t flags, int min_chunks) {
    int best_bn = 64, best_s = 1;
    double best_t = 1e30;
    for (int BN = 32; BN <= 128; BN *= 2) {
        if ((flags & MD2_CONV_TILE_N32) && BN != 32) continue;
        if ((flags & MD2_CONV_TILE_N64) && BN != 64) continue;
        if ((flags & MD2_CONV_TILE_N128) && BN != 128) continue;
        if (BN > 32 && a.N <= BN / 2 && !(flags & (MD2_CONV_TILE_N64 | MD2_CONV_TILE_N128))) continue;
        const int mblocks = (a.M + BM - 1) / BM, nblocks = (a.N + BN - 1) / BN;
        const int base = mblocks * nblocks, res = resident_blocks(BN);
        const int smax = (flags & MD2_CONV_NO_SPLIT) ? 1 : (a.nchunks / min_chunks > 1 ? a.nchunks / min_chunks : 1);
        for (int sp = 1; sp <= smax && sp <= 64; ++sp) {
            const int per = (a.nchunks + sp - 1) / sp;
            const int splits = (a.nchunks + per - 1) / per;
            const int rounds = (base * splits + res - 1) / res;
            const double t = (double)rounds * per * BN + (splits > 1 ? 8.0 * splits : 0.0);
            if (t < best_t - 1e-9) {
                best_t = t;
                best_bn = BN;
                best_s = splits;
            }
        }
    }
    a.bn = best_bn;
    a.mblocks = (a.M + BM - 1) / BM;
    a.nblocks = (a.N + best_bn - 1) / best_bn;
    a.chunks_per_split = (a.nchunks + best_s - 1) / best_s;
    a.splits = (a.nchunks + a.chunks_per_split - 1) / a.chunks_per_split;
}

ConvArgs args_of(const md2_conv_desc* d, int mode) {
    const Shape s = shape_of(d);
    ConvArgs a = {};
    a.KH = s.KH;
    a.KW = s.KW;
    if (mode == MODE_FWD) {
        a.B = s.B; a.H = s.H; a.W = s.W; a.C = s.C;
        a.Ho = s.Ho; a.Wo = s.Wo; a.stride = s.s; a.pad = s.p;
        a.N = s.N;
        a.M = s.B * s.Ho * s.Wo;
        a.nchunks = s.KH * s.KW * ((s.C + BK - 1) / BK);
        a.a_elems = s.B * s.H * s.W * s.C;            // x
        a.b_elems = s.N * s.KH * s.KW * s.C;          // weight
    } else if (mode == MODE_DGRAD) {
        // full convolution of gy (B, Ho, Wo, N) -> gx (B, H, W, C), stride 1
        a.B = s.B; a.H = s.Ho; a.W = s.Wo; a.C = s.N;
        a.Ho = s.H; a.Wo = s.W; a.stride = 1; a.pad = s.KH - 1 - s.p;
        a.N = s.C;
        a.Cg = s.N;
        a.M = s.B * s.H * s.W;
        a.nchunks = s.KH * s.KW * ((s.N + BK - 1) / BK);
        a.a_elems = s.B * s.Ho * s.Wo * s.N;          // gy
        a.b_elems = s.N * s.KH * s.KW * s.C;          // weight
    } else {
        a.B = s.B; a.H = s.H; a.W = s.W; a.C = s.C;
        a.Ho = s.Ho; a.Wo = s.Wo; a.stride = s.s; a.pad = s.p;
        a.M = s.KH * s.KW * s.C;   // (tap, ci): the output is written transposed, [co][tap][ci]
        a.Cg = s.N;
        a.N = s.N;
        a.P = s.B * s.Ho * s.Wo;
        a.nchunks = (a.P + BK - 1) / BK;
        a.a_elems = s.B * s.H * s.W * s.C;            // x
        a.b_elems = s.B * s.Ho * s.Wo * s.N;          // gy
    }
    return a;
}

int resident_blocks_x6(int BN, int BMX) { return 256 * ((BN <= 64 && BMX == 128) || BMX == 64 ? 2 : 1); }

// fixed cost of a K split's reduction launch in chunk-rounds (A/B knob MD2_X6_SPLIT_COST)
double split_launch_cost() {
    static const double c = [] {
        const char* e = getenv("MD2_X6_SPLIT_COST");
        return e ? atof(e) : 0.0;
    }();
    return c;
}

// x6 plan: BN = 16 / 32 / 64 for N <= 16 / 32 / 64, else 128; BMX = 256 with MD2_CONV_BM256 (the caller's
// autotune tries both); K split by the wave-quantisation model.  The weight-gradient
// kernel is 128 wide, 64 or 128 rows (co) tall.
void plan_x6(ConvArgs& a, uint32_t flags, bool wgrad = false) {
    // the weight gradient's 256-wide warp-specialised tile (conv_x6wws256_kernel): one
    // accumulation level, so at most 64 chunks per K split
    const bool w256 = wgrad && a.M > 64 && (flags & MD2_CONV_WS) && (flags & MD2_CONV_BM256);
    const int BN = wgrad ? (w256 ? 256 : 128) : (a.N <= 16 ? 16 : (a.N <= 32 ? 32 : (a.N <= 64 ? 64 : 128)));
    const int BMX = wgrad ? (a.M <= 64 ? 64 : 128) : ((BN == 128 && (flags & MD2_CONV_BM256)) ? 256 : 128);
    const int mblocks = (a.M + BMX - 1) / BMX, nblocks = (a.N + BN - 1) / BN;
    const int base = mblocks * nblocks, res = resident_blocks_x6(BN, BMX);
    int best_s = 1;
    double best_t = 1e30;
    const int smin = w256 ? (a.nchunks + 63) / 64 : 1;
    const int smax = std::max(smin, (flags & MD2_CONV_NO_SPLIT) ? 1 : (a.nchunks / 6 > 1 ? a.nchunks / 6 : 1));
    for (int sp = smin; sp <= smax && sp <= std::max(64, smin); ++sp) {
        const int per = (a.nchunks + sp - 1) / sp;
        const int splits = (a.nchunks + per - 1) / per;
        const int rounds = (base * splits + res - 1) / res;
        // a chunk-round of blocks ~1.5k cycles (x BMX/128); the split reduction moves
        // (splits + 1) M x N floats at ~2.4 KB/cycle chip-wide
        const double red = splits > 1 ? (double)(splits + 1) * a.M * a.N * 4.0 / 2400.0 / 1536.0 + split_launch_cost()
                                      : 0.0;
        const double t = (double)rounds * per * (BMX / 128.0) * (BN / 128 > 1 ? BN / 128 : 1) + red;
        if (t < best_t - 1e-9) {
            best_t = t;
            best_s = splits;
        }
    }
    a.bm = BMX;
    a.bn = BN;
    a.mblocks = mblocks;
    a.nblocks = nblocks;
    a.chunks_per_split = (a.nchunks + best_s - 1) / best_s;
    a.splits = (a.nchunks + a.chunks_per_split - 1) / a.chunks_per_split;
}

template <int MODE>
void launch(const ConvArgs& a, int BN, hipStream_t st) {
    const dim3 grid(a.mblocks * a.nblocks * a.splits);
    if (BN == 128)
        hipLaunchKernelGGL((conv_gemm_kernel<128, MODE>), grid, dim3(kThreads), 0, st, a);
    else if (BN == 64)
        hipLaunchKernelGGL((conv_gemm_kernel<64, MODE>), grid, dim3(kThreads), 0, st, a);
    else
        hipLaunchKernelGGL((conv_gemm_kernel<32, MODE>), grid, dim3(kThreads), 0, st, a);
}

int min_chunks_of(int mode) { return mode == MODE_WGRAD ? 8 : 6; }

bool use_x6(const md2_conv_desc* d, int mode) {
    if (d->flags & MD2_CONV_BF16) return false;
    if (!((d->flags & MD2_CONV_X6) && d->in_channels % 8 == 0 && d->out_channels % 8 == 0)) return false;
    if (mode == MODE_WGRAD) {   // fdiv() of the pixel index needs it below 2^24
        const Shape s = shape_of(d);
        if ((long long)s.B * s.Ho * s.Wo + 64 >= (1ll << 24)) return false;
    }
    return true;
}

// MD2_CONV_BF16 (ABI 22): the per-tap GEMMs on bf16 operands.  The forward's B rows
// run along in_channels and the input gradient's along out_channels (16-byte LDS-DMA
// pieces: multiples of 8); the A quads are 4 channels (multiples of 4); the input
// gradient is stride 1 only; the weight gradient walks its pixels with fdiv (< 2^24).
bool use_bf(const md2_conv_desc* d, int mode) {
    if (!(d->flags & MD2_CONV_BF16)) return false;
    if (mode == MODE_FWD) return d->in_channels % 8 == 0;
    if (mode == MODE_DGRAD) return d->stride == 1 && d->out_channels % 8 == 0;
    const Shape s = shape_of(d);
    return (long long)s.B * s.Ho * s.Wo + 64 < (1ll << 24);
}

// the patch-staged forward / stride-1 input gradient on bf16 operands (MD2_CONV_BF16 |
// MD2_CONV_PATCH): 3x3, GEMM channels % 32, more than 16 GEMM columns (as use_x6p)
bool use_bfp(const md2_conv_desc* d, int mode, const ConvArgs& a) {
    return (d->flags & MD2_CONV_PATCH) && use_bf(d, mode) && mode != MODE_WGRAD && a.KH == 3 && a.KW == 3 &&
           a.stride == 1 && a.C % XBK == 0 && a.N > 16 && !a.flatk;
}

// the patch-staged weight gradient on bf16 operands (MD2_CONV_BF16 | MD2_CONV_PATCH): 3x3 stride 1
bool use_bfpw(const md2_conv_desc* d) {
    return (d->flags & MD2_CONV_PATCH) && use_bf(d, MODE_WGRAD) && d->kernel_h == 3 && d->kernel_w == 3 &&
           d->stride == 1;
}

// the weight gradient's x6 GEMM: rows co, columns (tap, ci), K = output pixels
ConvArgs args_x6_wgrad(const md2_conv_desc* d) {
    const Shape s = shape_of(d);
    ConvArgs a = {};
    a.KH = s.KH;
    a.KW = s.KW;
    a.B = s.B; a.H = s.H; a.W = s.W; a.C = s.C;
    a.Ho = s.Ho; a.Wo = s.Wo; a.stride = s.s; a.pad = s.p;
    a.M = s.N;
    a.N = s.KH * s.KW * s.C;
    a.Cg = s.N;
    a.P = s.B * s.Ho * s.Wo;
    a.nchunks = (a.P + XBK - 1) / XBK;
    a.a_elems = s.B * s.H * s.W * s.C;    // x
    a.b_elems = s.B * s.Ho * s.Wo * s.N;  // gy
    return a;
}

size_t x6_planes_bytes(const md2_conv_desc* d) {
    return (3 * sizeof(uint16_t) * (size_t)d->out_channels * d->kernel_h * d->kernel_w * d->in_channels + 255) &
           ~(size_t)255;
}

// x6 fwd / dgrad on fewer than 32 GEMM channels: chunks over the flattened (tap, channel)
// index (a 16-channel 3x3 convolution is 4.5 full chunks instead of 9 half-empty ones)
void flat_k(ConvArgs& a, int mode) {
    if (mode != MODE_WGRAD && a.C < XBK) {
        a.flatk = 1;
        a.nchunks = (a.KH * a.KW * a.C + XBK - 1) / XBK;
    }
}

void launch_bf(const ConvArgs& a, hipStream_t st) {
    const dim3 grid(a.mblocks * a.nblocks * a.splits);
    if (a.bm == 256) hipLaunchKernelGGL((conv_x6_kernel<128, 256, true>), grid, dim3(X6Geo<128, 256>::NT), 0, st, a);
    else if (a.bn == 128)
        hipLaunchKernelGGL((conv_x6_kernel<128, 128, true>), grid, dim3(X6Geo<128, 128>::NT), 0, st, a);
    else if (a.bn == 64) hipLaunchKernelGGL((conv_x6_kernel<64, 128, true>), grid, dim3(X6Geo<64, 128>::NT), 0, st, a);
    else if (a.bn == 32) hipLaunchKernelGGL((conv_x6_kernel<32, 128, true>), grid, dim3(X6Geo<32, 128>::NT), 0, st, a);
    else hipLaunchKernelGGL((conv_x6_kernel<16, 128, true>), grid, dim3(X6Geo<16, 128>::NT), 0, st, a);
}

void launch_x6(const ConvArgs& a, hipStream_t st, bool ws = false) {
    const dim3 grid(a.mblocks * a.nblocks * a.splits);
    if (ws && a.bn == 128 && !a.flatk && !a.par) {   // warp-specialised (MD2_CONV_WS)
        if (a.bm == 256) hipLaunchKernelGGL((conv_x6ws_kernel<256>), grid, dim3(512), 0, st, a);
        else hipLaunchKernelGGL((conv_x6ws_kernel<128>), grid, dim3(512), 0, st, a);
        return;
    }
    if (a.bm == 256) hipLaunchKernelGGL((conv_x6_kernel<128, 256>), grid, dim3(X6Geo<128, 256>::NT), 0, st, a);
    else if (a.bn == 128) hipLaunchKernelGGL((conv_x6_kernel<128, 128>), grid, dim3(X6Geo<128, 128>::NT), 0, st, a);
    else if (a.bn == 64) hipLaunchKernelGGL((conv_x6_kernel<64, 128>), grid, dim3(X6Geo<64, 128>::NT), 0, st, a);
    else if (a.bn == 32) hipLaunchKernelGGL((conv_x6_kernel<32, 128>), grid, dim3(X6Geo<32, 128>::NT), 0, st, a);
    else hipLaunchKernelGGL((conv_x6_kernel<16, 128>), grid, dim3(X6Geo<16, 128>::NT), 0, st, a);
}

// Patch kernel (MD2_CONV_X6 | MD2_CONV_PATCH): 3x3 stride-1 forward / input gradient with
// the GEMM's channel count a multiple of 32 and more than 16 output channels
bool use_x6p(const md2_conv_desc* d, int mode, const ConvArgs& a) {
    return (d->flags & MD2_CONV_PATCH) && use_x6(d, mode) && mode != MODE_WGRAD && a.KH == 3 && a.KW == 3 &&
           a.stride == 1 && a.C % XBK == 0 && a.N > 16 && !a.flatk;
}

// TC (tile columns) with the least padded area; K split over 32-channel chunks by the
// wave-quantisation model of plan_x6 (a chunk here is nine taps)
void plan_x6p(ConvArgs& a, uint32_t flags) {
    const int BN = a.N <= 32 ? 32 : (a.N <= 64 ? 64 : 128);
    const int BMX = (BN == 128 && (flags & MD2_CONV_BM256)) ? 256 : 128;
    // least padded output area; among equals the smallest patch (the least halo per tile)
    int best_tc = 64;
    long long best_cost = -1;
    for (int TC = 64; TC >= 16; TC /= 2) {
        const int TR = BMX / TC;
        const long long area = (long long)((a.Ho + TR - 1) / TR) * TR * ((a.Wo + TC - 1) / TC) * TC;
        const long long cost = area * 4096 + (TR + 2) * (TC + 2);
        if (best_cost < 0 || cost < best_cost) {
            best_cost = cost;
            best_tc = TC;
        }
    }
    const int TR = BMX / best_tc;
    a.ptr = (a.Ho + TR - 1) / TR;
    a.ptc = (a.Wo + best_tc - 1) / best_tc;
    a.nchunks = a.C / XBK;
    const int mblocks = a.B * a.ptr * a.ptc, nblocks = (a.N + BN - 1) / BN;
    const int base = mblocks * nblocks, res = BN == 128 ? 256 : 512;   // blocks per CU: 1 (BN 128) / 2
    int best_s = 1;
    double best_t = 1e30;
    const int smax = (flags & MD2_CONV_NO_SPLIT) ? 1 : a.nchunks;
    for (int sp = 1; sp <= smax && sp <= 64; ++sp) {
        const int per = (a.nchunks + sp - 1) / sp;
        const int splits = (a.nchunks + per - 1) / per;
        const int rounds = (base * splits + res - 1) / res;
        const double red = splits > 1 ? (double)(splits + 1) * a.M * a.N * 4.0 / 2400.0 / 1536.0 + split_launch_cost()
                                      : 0.0;
        const double t = (double)rounds * per * 9.0 * (BMX / 128.0) + red;
        if (t < best_t - 1e-9) {
            best_t = t;
            best_s = splits;
        }
    }
    a.bm = BMX;
    a.bn = BN;
    a.mblocks = mblocks;
    a.nblocks = nblocks;
    a.chunks_per_split = (a.nchunks + best_s - 1) / best_s;
    a.splits = (a.nchunks + a.chunks_per_split - 1) / a.chunks_per_split;
    a.flatk = best_tc;   // carried to launch_x6p (the kernel itself does not read flatk)
}

template <int BN, int BMX, bool BF = false>
void launch_x6p_tc(const ConvArgs& a, hipStream_t st) {
    const dim3 grid(a.mblocks * a.nblocks * a.splits), block(X6Geo<BN, BMX>::NT);
    ConvArgs b = a;
    b.flatk = 0;
    if (a.flatk == 64) hipLaunchKernelGGL((conv_x6p_kernel<BN, BMX, 64, BF>), grid, block, 0, st, b);
    else if (a.flatk == 32) hipLaunchKernelGGL((conv_x6p_kernel<BN, BMX, 32, BF>), grid, block, 0, st, b);
    else hipLaunchKernelGGL((conv_x6p_kernel<BN, BMX, 16, BF>), grid, block, 0, st, b);
}

template <bool BF = false>
void launch_x6p(const ConvArgs& a, hipStream_t st) {
    if (a.bm == 256) launch_x6p_tc<128, 256, BF>(a, st);
    else if (a.bn == 128) launch_x6p_tc<128, 128, BF>(a, st);
    else if (a.bn == 64) launch_x6p_tc<64, 128, BF>(a, st);
    else launch_x6p_tc<32, 128, BF>(a, st);
}

// Patch weight gradient (MD2_CONV_X6 | MD2_CONV_PATCH): 3x3 stride 1, any Ci % 8 (the
// last 32-channel group zero-filled), Co % 8
bool use_x6pw(const md2_conv_desc* d) {
    return (d->flags & MD2_CONV_PATCH) && use_x6(d, MODE_WGRAD) && d->kernel_h == 3 && d->kernel_w == 3 &&
           d->stride == 1;
}

// rows BMW = 32 for Co <= 32 else 64; one block per CU (135 KB LDS); K split by the
// wave-quantisation model of plan_x6 (a chunk-round ~1.7k cycles)
constexpr int kX6pwMaxChunks = 64;

void plan_x6pw(ConvArgs& a, uint32_t flags) {
    const int BMW = a.M <= 32 ? 32 : 64;
    a.ptc = (a.Wo + 31) / 32;
    a.nchunks = a.B * a.Ho * a.ptc;
    const int smin = (a.nchunks + kX6pwMaxChunks - 1) / kX6pwMaxChunks;
    const int mblocks = (a.M + BMW - 1) / BMW, nblocks = (a.C + XBK - 1) / XBK;
    const int base = mblocks * nblocks, res = 256;
    int best_s = 1;
    double best_t = 1e30;
    const int smax = std::max(1, a.nchunks / 4);
    // candidates: no split, and the largest split count that fills k rounds of CUs
    for (int k = 0; k <= 8; ++k) {
        const int sp = std::max(smin, std::min(smax, k == 0 ? 1 : std::max(1, k * res / base)));
        const int per = (a.nchunks + sp - 1) / sp;
        const int splits = (a.nchunks + per - 1) / per;
        const int rounds = (base * splits + res - 1) / res;
        const double red = splits > 1 ? (double)(splits + 1) * a.M * a.N * 4.0 / 2400.0 / 1700.0 + split_launch_cost()
                                      : 0.0;
        const double t = (double)rounds * per + red;
        if (t < best_t - 1e-9) {
            best_t = t;
            best_s = splits;
        }
    }
    a.bm = BMW;
    a.mblocks = mblocks;
    a.nblocks = nblocks;
    a.chunks_per_split = (a.nchunks + best_s - 1) / best_s;
    a.splits = (a.nchunks + a.chunks_per_split - 1) / a.chunks_per_split;
}

// Stride-2 input gradient on x6 (MD2_CONV_X6, at least 32 output channels): gx pixels
// of one parity (py, px) receive only the taps kh ≡ py + pad, kw ≡ px + pad (mod 2),
// each from one gy pixel — a stride-1 GEMM over that class's Ho x Wo grid, scattered
// into gx.  Four launches (a 1x1 stride-2 convolution's odd classes have no taps: they
// run with no chunks and write zeros).  false: the class is empty.
bool dgrad_s2_class(const md2_conv_desc* d, int py, int px, ConvArgs& a, uint32_t extra_flags = 0) {
    const Shape s = shape_of(d);
    a = ConvArgs{};
    a.KH = s.KH;
    a.KW = s.KW;
    a.B = s.B; a.H = s.Ho; a.W = s.Wo; a.C = s.N;   // GEMM input: gy
    a.Ho = (s.H - py + 1) / 2;
    a.Wo = (s.W - px + 1) / 2;
    if (a.Ho < 1 || a.Wo < 1) return false;
    a.stride = 1;
    a.pad = 0;
    a.N = s.C;
    a.Cg = s.N;
    a.M = s.B * a.Ho * a.Wo;
    a.par = 1;
    a.py = py;
    a.px = px;
    a.oHf = s.H;
    a.oWf = s.W;
    a.kh0 = (py + s.p) & 1;
    a.kw0 = (px + s.p) & 1;
    const int nth = a.kh0 < s.KH ? (s.KH - a.kh0 + 1) / 2 : 0, ntw = a.kw0 < s.KW ? (s.KW - a.kw0 + 1) / 2 : 0;
    a.ntw = ntw > 0 ? ntw : 1;
    a.dy0 = (py + s.p - a.kh0) / 2;
    a.dx0 = (px + s.p - a.kw0) / 2;
    a.a_elems = s.B * s.Ho * s.Wo * s.N;
    a.b_elems = 3 * s.N * s.KH * s.KW * s.C;
    const int taps = nth * ntw;
    a.nchunks = taps > 0 ? taps * ((s.N + XBK - 1) / XBK) : 1;
    plan_x6(a, d->flags | extra_flags);
    if (taps == 0) {   // zeros: no chunks, no split
        a.nchunks = 0;
        a.chunks_per_split = 0;
        a.splits = 1;
    }
    return true;
}

bool use_x6_s2(const md2_conv_desc* d) {
    return d->stride == 2 && use_x6(d, MODE_DGRAD) && d->out_channels >= XBK;
}
// the same parity-class input gradient on bf16 operands (MD2_CONV_BF16): the flipped
// [Ci][KT][Co] plane rows run along out_channels
bool use_bf_s2(const md2_conv_desc* d) {
    return (d->flags & MD2_CONV_BF16) && d->stride == 2 && d->out_channels % 8 == 0 && d->out_channels >= XBK;
}

int run_dgrad_s2(const md2_conv_desc* d, const float* gy, const float* w, float* gx, void* ws, void* stream) {
    if (!ws) return md2_report_error(MD2_ERR_ARG, "conv_dgrad (stride 2): workspace required");
    const hipStream_t st = (hipStream_t)stream;
    const bool bf = (d->flags & MD2_CONV_BF16) != 0;   // bf16 gy / gx, `w` the one bf16 plane
    __bf16* planes = (bf || (d->flags & MD2_CONV_PRESPLIT)) ? (__bf16*)w : (__bf16*)ws;
    const size_t part_off = bf ? 0 : x6_planes_bytes(d);
    auto go = [&](const ConvArgs& a) {
        if (bf) launch_bf(a, st);
        else launch_x6(a, st);
    };
    if (!bf && !(d->flags & MD2_CONV_PRESPLIT)) {
        const int nw = d->out_channels * d->kernel_h * d->kernel_w * d->in_channels;
        hipLaunchKernelGGL(conv_wsplit_kernel, dim3((nw + 255) / 256), dim3(256), 0, st, w, planes, d->out_channels,
                           d->kernel_h * d->kernel_w, d->in_channels, 1);
    }
    // classes without taps (a 1x1 stride-2 convolution's three odd ones) are zeros:
    // one memset of grad_x instead of a GEMM launch per class that multiplies nothing
    bool tapless = false;
    for (int py = 0; py < 2; ++py)
        for (int px = 0; px < 2; ++px) {
            ConvArgs a;
            if (dgrad_s2_class(d, py, px, a) && a.nchunks == 0) tapless = true;
        }
    if (tapless) {
        const hipError_t me = hipMemsetAsync(gx, 0, (bf ? 2 : 4) * (size_t)d->batch * d->height * d->width *
                                                        d->in_channels, st);
        if (me != hipSuccess) return md2_report_error(MD2_ERR_HIP, hipGetErrorString(me));
    }
    if (d->flags & MD2_CONV_S2_ONE) {
        // one launch over the classes with taps, heaviest class first, no K split
        ConvArgs m;
        int nc = 0, blocks = 0;
        int order[4] = {0, 1, 2, 3}, taps[4] = {0, 0, 0, 0};
        ConvArgs cl[4];
        for (int c = 0; c < 4; ++c)
            if (dgrad_s2_class(d, c >> 1, c & 1, cl[c], MD2_CONV_NO_SPLIT)) taps[c] = cl[c].nchunks;
        std::sort(order, order + 4, [&](int x, int y) { return taps[x] > taps[y] || (taps[x] == taps[y] && x < y); });
        for (int k = 0; k < 4; ++k) {
            const int c = order[k];
            if (taps[c] == 0) continue;
            const ConvArgs& a = cl[c];
            if (nc == 0) m = a;
            m.cls_blk[nc] = blocks;
            m.cls_py[nc] = a.py;
            m.cls_px[nc] = a.px;
            m.cls_kh0[nc] = a.kh0;
            m.cls_kw0[nc] = a.kw0;
            m.cls_ntw[nc] = a.ntw;
            m.cls_dy0[nc] = a.dy0;
            m.cls_dx0[nc] = a.dx0;
            m.cls_Ho[nc] = a.Ho;
            m.cls_Wo[nc] = a.Wo;
            m.cls_nchunks[nc] = a.nchunks;
            blocks += a.mblocks * a.nblocks;
            ++nc;
        }
        if (nc > 0) {
            m.ncls = nc;
            m.splits = 1;
            m.mblocks = blocks / m.nblocks;   // launch_x6: grid = mblocks * nblocks * splits
            m.a = gy;
            m.b = (const float*)planes;
            m.y = gx;
            if (bf) {
                m.ybf16 = 1;
                m.b_elems /= 3;
            }
            go(m);
        }
    } else {
    for (int py = 0; py < 2; ++py)
        for (int px = 0; px < 2; ++px) {
            ConvArgs a;
            if (!dgrad_s2_class(d, py, px, a) || a.nchunks == 0) continue;
            a.a = gy;
            a.b = (const float*)planes;
            a.y = a.splits > 1 ? (float*)((char*)ws + part_off) : gx;
            if (bf) {
                a.ybf16 = 1;
                a.b_elems /= 3;
            }
            go(a);
            if (a.splits > 1) {
                const int n4 = a.M * a.N / 4;
                hipLaunchKernelGGL(bf ? conv_reduce_scatter_kernel<1> : conv_reduce_scatter_kernel<0>,
                                   dim3((n4 + kRedOut - 1) / kRedOut), dim3(256), 0, st, (const float4*)a.y,
                                   (float4*)gx, n4, a.splits, a.N / 4, a.Ho, a.Wo, a.oHf, a.oWf, py, px);
            }
        }
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

// Input gradient of a strided convolution as ONE dense GEMM plus a gather: cols
// (B, Ho, Wo, KH, KW, C) = grad_y (B, Ho, Wo, N) x W'[N][(kh, kw, c)] (a 1x1 forward
// convolution with KH·KW·C output channels, run by the caller), then
//   gx[b][y][x][c] = Σ_{kh, kw: y = s i - p + kh, x = s j - p + kw} cols[b][i][j][kh][kw][c]
// — each grad_x pixel gathers its 1, 2 or 4 (stride 2, 3x3) tap contributions in (kh, kw)
// order: deterministic, no atomics.  The GEMM's tiles are all the same K (N), where the
// parity-class form runs four GEMMs of 1, 2, 2 and 4 taps whose heaviest sets the time.
// One thread per grad_x pixel and channel quad.
__global__ __launch_bounds__(256) void conv_col2im_kernel(const float4* __restrict__ cols, float4* __restrict__ gx,
                                                          int B, int H, int W, int Q, int Ho, int Wo, int KH, int KW,
                                                          int stride, int pad) {
    const long long n = (long long)B * H * W * Q;
    for (long long t = (long long)blockIdx.x * 256 + threadIdx.x; t < n; t += (long long)gridDim.x * 256) {
        const int q = (int)(t % Q);
        long long r = t / Q;
        const int x = (int)(r % W);
        r /= W;
        const int y = (int)(r % H), b = (int)(r / H);
        float4 acc = {0.f, 0.f, 0.f, 0.f};
        for (int kh = 0; kh < KH; ++kh) {
            const int ty = y + pad - kh;
            if (ty < 0 || ty % stride) continue;
            const int i = ty / stride;
            if (i >= Ho) continue;
            for (int kw = 0; kw < KW; ++kw) {
                const int tx = x + pad - kw;
                if (tx < 0 || tx % stride) continue;
                const int j = tx / stride;
                if (j >= Wo) continue;
                const float4 v = cols[(((size_t)(b * Ho + i) * Wo + j) * (KH * KW) + kh * KW + kw) * Q + q];
                acc.x += v.x;
                acc.y += v.y;
                acc.z += v.z;
                acc.w += v.w;
            }
        }
        gx[t] = acc;
    }
}

// MD2_CONV_BF16: A / out are bf16 (the weight gradient's out fp32), B the one bf16
// weight plane (fwd / dgrad: md2_conv_bf16_weights) or grad_y (wgrad)
int run_bf(const md2_conv_desc* d, int mode, const void* A, const void* B, void* out, void* ws, void* stream,
           const char* name) {
    if (!use_bf(d, mode))
        return md2_report_error(MD2_ERR_ARG, "conv bf16: fwd in_channels % 8; dgrad stride 1, out_channels % 8; "
                                             "wgrad fewer than 2^24 output pixels");
    ConvArgs a = mode == MODE_WGRAD ? args_x6_wgrad(d) : args_of(d, mode);
    const bool pw = mode == MODE_WGRAD && use_bfpw(d);
    flat_k(a, mode);
    const bool patch = use_bfp(d, mode, a);
    if (pw) plan_x6pw(a, d->flags);
    else if (patch) plan_x6p(a, d->flags);
    else plan_x6(a, d->flags, mode == MODE_WGRAD);
    a.a = (const float*)A;
    a.b = (const float*)B;
    a.ybf16 = mode == MODE_WGRAD ? 2 : 1;
    if (mode != MODE_WGRAD) a.b_elems = d->out_channels * d->kernel_h * d->kernel_w * d->in_channels;
    if (a.splits > 1 && !ws) return md2_report_error(MD2_ERR_ARG, name);
    a.y = a.splits > 1 ? (float*)ws : (float*)out;
    const hipStream_t st = (hipStream_t)stream;
    if (pw) {
        const dim3 grid(a.mblocks * a.nblocks * a.splits);
        if (a.bm == 64) hipLaunchKernelGGL((conv_x6pw_kernel<64, true>), grid, dim3(576), 0, st, a);
        else hipLaunchKernelGGL((conv_x6pw_kernel<32, true>), grid, dim3(576), 0, st, a);
    } else if (mode == MODE_WGRAD) {
        const dim3 grid(a.mblocks * a.nblocks * a.splits);
        const bool xf = (a.Wo & 3) == 0;
        void (*k)(ConvArgs) = a.bm == 64
                                  ? (xf ? conv_x6_wgrad_kernel<64, true, true> : conv_x6_wgrad_kernel<64, false, true>)
                                  : (xf ? conv_x6_wgrad_kernel<128, true, true> : conv_x6_wgrad_kernel<128, false, true>);
        if (a.bn == 256) k = xf ? conv_x6wws256_kernel<true, true> : conv_x6wws256_kernel<false, true>;   // 256-wide
        hipLaunchKernelGGL(k, grid, dim3(512), 0, st, a);
    } else if (patch) {
        launch_x6p<true>(a, st);
    } else {
        launch_bf(a, st);
    }
    if (a.splits > 1) launch_reduce((const float4*)a.y, (float4*)out, a.M * a.N / 4, a.splits, st, a.ybf16);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int run(const md2_conv_desc* d, int mode, const float* A, const float* B, float* out, void* ws, void* stream,
        const char* name) {
    if (d->flags & MD2_CONV_BF16) return run_bf(d, mode, A, B, out, ws, stream, name);
    ConvArgs a = (mode == MODE_WGRAD && use_x6(d, mode)) ? args_x6_wgrad(d) : args_of(d, mode);
    if (use_x6(d, mode)) flat_k(a, mode);
    const bool patch = use_x6p(d, mode, a);
    const bool patch_w = mode == MODE_WGRAD && use_x6pw(d);
    if (patch) plan_x6p(a, d->flags);
    else if (patch_w) plan_x6pw(a, d->flags);
    else if (use_x6(d, mode)) plan_x6(a, d->flags, mode == MODE_WGRAD);
    else plan(a, d->flags, min_chunks_of(mode));
    const int BN = a.bn;
    a.a = A;
    a.b = B;
    if ((a.splits > 1 || (use_x6(d, mode) && mode != MODE_WGRAD)) && !ws) return md2_report_error(MD2_ERR_ARG, name);
    a.y = a.splits > 1 ? (float*)ws : out;
    const hipStream_t st = (hipStream_t)stream;
    if (patch_w) {
        const dim3 grid(a.mblocks * a.nblocks * a.splits);
        if (a.bm == 64) hipLaunchKernelGGL(conv_x6pw_kernel<64>, grid, dim3(576), 0, st, a);
        else hipLaunchKernelGGL(conv_x6pw_kernel<32>, grid, dim3(576), 0, st, a);
    } else if (use_x6(d, mode) && mode == MODE_WGRAD) {
        const dim3 grid(a.mblocks * a.nblocks * a.splits);
        const bool xf = (a.Wo & 3) == 0;   // the x-side pixel walk (conv_x6_wgrad_kernel)
        void (*k)(ConvArgs) = a.bm == 64 ? (xf ? conv_x6_wgrad_kernel<64, true> : conv_x6_wgrad_kernel<64, false>)
                                         : (xf ? conv_x6_wgrad_kernel<128, true> : conv_x6_wgrad_kernel<128, false>);
        if (a.bm == 128 && (d->flags & MD2_CONV_WS))   // warp-specialised, same results
            k = xf ? conv_x6wws_kernel<true> : conv_x6wws_kernel<false>;
        if (a.bn == 256) k = xf ? conv_x6wws256_kernel<true> : conv_x6wws256_kernel<false>;   // 256-wide tile
        hipLaunchKernelGGL(k, grid, dim3(512), 0, st, a);
    } else if (use_x6(d, mode)) {
        // B: the weights split into bf16 planes at the front of the workspace, or
        // already split by the caller (MD2_CONV_PRESPLIT: `weight` is the planes)
        __bf16* planes = (d->flags & MD2_CONV_PRESPLIT) ? (__bf16*)B : (__bf16*)ws;
        a.b = (const float*)planes;
        a.b_elems = 3 * d->out_channels * d->kernel_h * d->kernel_w * d->in_channels;
        if (a.splits > 1) a.y = (float*)((char*)ws + x6_planes_bytes(d));
        const int nw = a.b_elems / 3;
        if (!(d->flags & MD2_CONV_PRESPLIT))
            hipLaunchKernelGGL(conv_wsplit_kernel, dim3((nw + 255) / 256), dim3(256), 0, st, B, planes,
                               d->out_channels, d->kernel_h * d->kernel_w, d->in_channels, mode == MODE_DGRAD ? 1 : 0);
        if (patch) launch_x6p(a, st);
        else launch_x6(a, st, (d->flags & MD2_CONV_WS) != 0);
    } else if (mode == MODE_FWD) launch<MODE_FWD>(a, BN, st);
    else if (mode == MODE_DGRAD) launch<MODE_DGRAD>(a, BN, st);
    else launch<MODE_WGRAD>(a, BN, st);
    if (a.splits > 1) {
        const int n4 = a.M * a.N / 4;
        launch_reduce((const float4*)a.y, (float4*)out, n4, a.splits, st);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

size_t ws_bytes(const md2_conv_desc* d, int mode) {
    if (d->flags & MD2_CONV_BF16) {   // the K split's fp32 partials only (the weight plane is the caller's)
        if (mode == MODE_DGRAD && use_bf_s2(d)) {
            size_t part = 0;
            for (int py = 0; py < 2; ++py)
                for (int px = 0; px < 2; ++px) {
                    ConvArgs c;
                    if (dgrad_s2_class(d, py, px, c) && c.splits > 1)
                        part = std::max(part, sizeof(float) * (size_t)c.splits * c.M * c.N);
                }
            return part;
        }
        if (!use_bf(d, mode)) return 0;
        ConvArgs a = mode == MODE_WGRAD ? args_x6_wgrad(d) : args_of(d, mode);
        flat_k(a, mode);
        if (mode == MODE_WGRAD && use_bfpw(d)) plan_x6pw(a, d->flags);
        else if (use_bfp(d, mode, a)) plan_x6p(a, d->flags);
        else plan_x6(a, d->flags, mode == MODE_WGRAD);
        return a.splits > 1 ? sizeof(float) * (size_t)a.splits * a.M * a.N : 0;
    }
    if (mode == MODE_DGRAD && use_x6_s2(d)) {
        size_t part = 0;
        for (int py = 0; py < 2; ++py)
            for (int px = 0; px < 2; ++px) {
                ConvArgs c;
                if (dgrad_s2_class(d, py, px, c) && c.splits > 1)
                    part = std::max(part, sizeof(float) * (size_t)c.splits * c.M * c.N);
            }
        return x6_planes_bytes(d) + part;
    }
    ConvArgs a = (mode == MODE_WGRAD && use_x6(d, mode)) ? args_x6_wgrad(d) : args_of(d, mode);
    if (mode == MODE_WGRAD && use_x6pw(d)) {
        plan_x6pw(a, d->flags);
        return a.splits > 1 ? sizeof(float) * (size_t)a.splits * a.M * a.N : 0;
    }
    if (use_x6(d, mode) && mode == MODE_WGRAD) {
        plan_x6(a, d->flags, true);
        return a.splits > 1 ? sizeof(float) * (size_t)a.splits * a.M * a.N : 0;
    }
    if (use_x6(d, mode)) {
        flat_k(a, mode);
        if (use_x6p(d, mode, a)) plan_x6p(a, d->flags);
        else plan_x6(a, d->flags);
        return x6_planes_bytes(d) + (a.splits > 1 ? sizeof(float) * (size_t)a.splits * a.M * a.N : 0);
    }
    plan(a, d->flags, min_chunks_of(mode));
    return a.splits > 1 ? sizeof(float) * (size_t)a.splits * a.M * a.N : 0;
}

}  // namespace

extern "C" {

size_t md2_conv_workspace_bytes(const md2_conv_desc* d) {
    if (!valid(d)) return 0;
    size_t m = ws_bytes(d, MODE_FWD);
    if (d->stride == 1 || use_x6_s2(d) || use_bf_s2(d)) m = m > ws_bytes(d, MODE_DGRAD) ? m : ws_bytes(d, MODE_DGRAD);
    const size_t w = ws_bytes(d, MODE_WGRAD);
    return m > w ? m : w;
}

int md2_conv_split_weights(const md2_conv_desc* d, const float* weight, void* planes_fwd, void* planes_dgrad,
                           void* stream) {
    if (!valid(d) || d->in_channels % 8 || d->out_channels % 8)
        return md2_report_error(MD2_ERR_ARG, "conv_split_weights: channels % 8, pad < kernel, sizes < 2^29");
    if (!weight || !planes_fwd) return md2_report_error(MD2_ERR_ARG, "conv_split_weights: NULL operand");
    const dim3 grid((d->in_channels + 31) / 32, (d->out_channels + 31) / 32, d->kernel_h * d->kernel_w);
    hipLaunchKernelGGL(conv_wsplit_tile_kernel, grid, dim3(256), 0, (hipStream_t)stream, weight,
                       (__bf16*)planes_fwd, (__bf16*)planes_dgrad, d->out_channels, d->kernel_h * d->kernel_w,
                       d->in_channels);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_conv_bf16_weights(const md2_conv_desc* d, const float* weight, void* w_fwd, void* w_dgrad, void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "conv_bf16_weights: channels % 4, pad < kernel, sizes < 2^29");
    if (!weight || !w_fwd) return md2_report_error(MD2_ERR_ARG, "conv_bf16_weights: NULL operand");
    const dim3 grid((d->in_channels + 31) / 32, (d->out_channels + 31) / 32, d->kernel_h * d->kernel_w);
    hipLaunchKernelGGL(conv_wsplit_tile_kernel, grid, dim3(256), 0, (hipStream_t)stream, weight, (__bf16*)w_fwd,
                       (__bf16*)w_dgrad, d->out_channels, d->kernel_h * d->kernel_w, d->in_channels, 1);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_conv_bf16_weights_multi(const md2_wsplit_entry* table, int n, int total_blocks, void* stream) {
    if (!table || n <= 0 || total_blocks <= 0) return md2_report_error(MD2_ERR_ARG, "conv_bf16_weights_multi: empty");
    hipLaunchKernelGGL(conv_wsplit_multi_kernel, dim3(total_blocks), dim3(256), 0, (hipStream_t)stream, table, n, 1);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_conv_split_weights_multi(const md2_wsplit_entry* table, int n, int total_blocks, void* stream) {
    if (!table || n <= 0 || total_blocks <= 0) return md2_report_error(MD2_ERR_ARG, "conv_split_weights_multi: empty");
    hipLaunchKernelGGL(conv_wsplit_multi_kernel, dim3(total_blocks), dim3(256), 0, (hipStream_t)stream, table, n);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_conv_fwd(const md2_conv_desc* d, const float* x, const float* weight, float* y, void* workspace,
                 void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "conv_fwd: channels % 4, pad < kernel, sizes < 2^29");
    if (!x || !weight || !y) return md2_report_error(MD2_ERR_ARG, "conv_fwd: NULL operand");
    return run(d, MODE_FWD, x, weight, y, workspace, stream, "conv_fwd: workspace required (K split)");
}

int md2_conv_dgrad(const md2_conv_desc* d, const float* grad_y, const float* weight, float* grad_x,
                   void* workspace, void* stream) {
    if (!valid(d) || (d->stride != 1 && !use_x6_s2(d) && !use_bf_s2(d)))
        return md2_report_error(MD2_ERR_ARG, "conv_dgrad: stride 1 (stride 2: MD2_CONV_X6, channels % 8, >= 32 "
                                             "output channels), channels % 4, pad < kernel, sizes < 2^29");
    if (!grad_y || !weight || !grad_x) return md2_report_error(MD2_ERR_ARG, "conv_dgrad: NULL operand");
    if (d->stride == 2) return run_dgrad_s2(d, grad_y, weight, grad_x, workspace, stream);
    return run(d, MODE_DGRAD, grad_y, weight, grad_x, workspace, stream, "conv_dgrad: workspace required (K split)");
}

int md2_conv_wgrad(const md2_conv_desc* d, const float* x, const float* grad_y, float* grad_weight,
                   void* workspace, void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "conv_wgrad: channels % 4, pad < kernel, sizes < 2^29");
    if (!x || !grad_y || !grad_weight) return md2_report_error(MD2_ERR_ARG, "conv_wgrad: NULL operand");
    return run(d, MODE_WGRAD, x, grad_y, grad_weight, workspace, stream, "conv_wgrad: workspace required (K split)");
}

int md2_conv_col2im(const md2_conv_desc* d, const float* cols, float* grad_x, void* stream) {
    if (!d || !cols || !grad_x) return md2_report_error(MD2_ERR_ARG, "conv_col2im: NULL operand");
    if (d->in_channels % 4 || d->stride < 1 || d->pad < 0 || d->kernel_h < 1 || d->kernel_w < 1 || d->batch < 1 ||
        d->height < 1 || d->width < 1)
        return md2_report_error(MD2_ERR_ARG, "conv_col2im: channels % 4, stride >= 1, pad >= 0");
    const int Ho = (d->height + 2 * d->pad - d->kernel_h) / d->stride + 1;
    const int Wo = (d->width + 2 * d->pad - d->kernel_w) / d->stride + 1;
    if (Ho < 1 || Wo < 1) return md2_report_error(MD2_ERR_ARG, "conv_col2im: empty output");
    const int Q = d->in_channels / 4;
    const long long n = (long long)d->batch * d->height * d->width * Q;
    const long long blocks = (n + 255) / 256;
    hipLaunchKernelGGL(conv_col2im_kernel, dim3((unsigned)(blocks < 8192 ? blocks : 8192)), dim3(256), 0,
                       (hipStream_t)stream, (const float4*)cols, (float4*)grad_x, d->batch, d->height, d->width, Q,
                       Ho, Wo, d->kernel_h, d->kernel_w, d->stride, d->pad);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
