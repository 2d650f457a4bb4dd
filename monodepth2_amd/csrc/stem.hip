// stem.hip — weight gradient of the ResNet stem convolution (conv1: 7x7, stride 2,
// padding 3, C -> 64, no bias; networks/resnet_encoder.py -> torchvision conv1) on
// split-bf16 MFMA (f32-class: three exact bf16 planes per operand, six products,
// f32 accumulation — the scheme of conv.hip's x6 kernels).
//
// The stem's input is data (the normalised frames), so its backward is the weight
// gradient alone: dW[co][ky][kx][ci] = Σ_p dy[p][co] · x[p's 7x7 window][ky][kx][ci]
// over every output pixel p — a GEMM with M = 64 output channels, N = 49·C window taps
// and K = B·Ho·Wo output pixels (368k at B=12, 192x640).  MIOpen's backward-weights
// kernel (igemm_wrw) runs it in ~125 / ~430 us at the step's shapes (C = 3, B = 12 /
// C = 6, B = 24; 192x640); the im2col-build kernel below in ~100 / ~405 us with its split
// reduction, and the transposed-read kernel (stem_x6_wgrad_tr_kernel, the default for
// C = 3 / 6; MD2_STEM_WGRAD_BUILD=1 selects the build kernel) in ~0.082 / ~0.21 ms: the
// build, not the multiply, set the old kernel's time.
//
// Here the channels go in groups of three (one frame; the pose encoder's pair is two
// groups) padded to four, and K in chunks of one 32-pixel segment of one
// output row.  Per chunk a block stages the 7 input rows x 69 columns x 3 channels
// under the segment ONCE (fp32, coalesced row runs, one LDS buffer per chunk), and
// builds from them the seven B tiles — kernel row kh: rows (kx, ci) = 4 kx + ci, 32
// pixels, x[2 oh - 3 + kh][2 ow - 3 + kx][ci] — split into bf16 planes in LDS, beside
// the dy tile (64 co x 32 pixels, split on the way in).  Wave kh (7 waves) multiplies
// its kernel row: 64 x 32 outputs per chunk, 2 x 6 MFMAs per 16 pixels.  The next
// chunk's rows and dy are fetched into registers behind the current chunk's build /
// MFMAs; two barriers per chunk; two blocks per CU.  Blocks take contiguous chunk
// ranges (K splits) and write fp32 partials [group][split][64][147]; a second launch
// sums them in split order into dW in the weight's memory format — deterministic,
// no atomics.
// Layouts: x (B,H,W,C) and dy (B,Ho,Wo,64) channels_last fp32; dW channels_last
// [co][ky][kx][ci] (MD2_STEM_WEIGHT_CL) or contiguous [co][ci][ky][kx].

#include <hip/hip_runtime.h>

#include <type_traits>

#include <stdint.h>

#include <algorithm>
#include <stdlib.h>

#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kCo = 64;
constexpr int kWaves = 7;               // one per kernel row
constexpr int kThreads = 64 * kWaves;
constexpr int kSeg = 32;                // output pixels per chunk (one output row segment)
constexpr int kRawW = 2 * kSeg + 5;     // input columns under a segment
constexpr int kCG = 3;                  // channels per group (one frame)
// pitch of one staged (kernel row, channel, column parity) run: 35 columns used; 39
// (= 3 mod 4) spreads the build's 32-lane read groups —
// four tile rows x 8 pixel quads — over distinct banks (36: four-way on every read;
// 39: 2.6x fewer conflict cycles in an exhaustive model of the build and the store)
constexpr int kRP = 39;
constexpr int kRaw = 7 * kCG * 2 * kRP;  // floats per staged chunk ([kh][ci][parity][kRP])
constexpr int kXBK = 32;
constexpr int kPA = kCo * kXBK;         // bf16 per dy plane (64 co x 32 pixels)
constexpr int kPT = 32 * kXBK;          // bf16 per B tile plane (32 rows x 32 pixels)
constexpr int kOut = 49 * kCG;          // outputs per output channel per group
constexpr int kBlocksPerCU = 2;
constexpr int kMaxChunks = 64;          // chunks per K split at most

struct StemArgs {
    int B, C, H, W, Ho, Wo;
    int w_cl;
    int nseg, nchunks, splits, cps;     // segments per output row, chunks, K splits, chunks per split
    const float* x;
    const float* gy;
    float* part;                        // [group][split][64][147]
    float* gw;
};

// Exact three-way split by truncation (conv.hip): x == x0 + x1 + x2, each a bf16
__device__ __forceinline__ float trunc16(float x) {
    return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, x) & 0xFFFF0000u);
}
__device__ __forceinline__ uint32_t hi16x2(float lo, float hi) {
    return __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, hi), __builtin_bit_cast(uint32_t, lo), 0x07060302u);
}
// fp32 -> bf16 bits / the bf16 value as fp32, round to nearest even (torch's cast)
__device__ __forceinline__ uint16_t f2bf16(float v) {
    const uint32_t u = __builtin_bit_cast(uint32_t, v);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40u);
    return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf16_rne(float v) { return __builtin_bit_cast(float, (uint32_t)f2bf16(v) << 16); }
// [rows][32 k] bf16 planes with 16-byte quads XOR-swizzled by (row >> 2) & 3 and rows
// r, r ^ 1 swapped in odd row quads (conv.hip xidx2): conflict-free fragment reads
// and conflict-free 8-byte stores from lanes covering two adjacent rows
__device__ __forceinline__ int xidx2(int r, int k) {
    r ^= (r >> 2) & 1;
    return r * kXBK + ((((k >> 3) ^ (r >> 2)) & 3) << 3) + (k & 7);
}
__device__ __forceinline__ int xcd_contiguous_block(int bid, int n) {   // conv.hip
    const int q = n >> 3, r = n & 7;
    const int xcd = bid & 7, idx = bid >> 3;
    return xcd < r ? xcd * (q + 1) + idx : r * (q + 1) + (xcd - r) * q + idx;
}
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// two 7-wave blocks per CU put four waves on two of the SIMDs: <= 128 VGPRs
template <int C>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4))) void stem_x6_wgrad_kernel(StemArgs a) {
    __shared__ float raw[2][kRaw];   // [kh][ci][column parity][kRP]: x[2oh-3+kh][iw0 + 2m + parity][3cg+ci]
    __shared__ __bf16 At[3 * kPA];
    __shared__ __bf16 Bt[7 * 3 * kPT];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // the channel groups of one K split (same input rows, same dy) on one XCD, dispatched
    // close together, so the second group's fetches hit the first one's L2 lines: blocks
    // are dealt round-robin over the 8 XCDs (bid & 7); group cg of split ks gets
    // bid = 8 (NG (ks / 8) + cg) + ks % 8.  The grid is padded to whole octets of splits.
    const int NG = a.C / kCG;
    const int j8 = blockIdx.x >> 3;
    const int cg = j8 % NG, ks = (j8 / NG) * 8 + (blockIdx.x & 7);
    if (ks >= a.splits) return;
    const int t0 = ks * a.cps;
    const int n = min(a.cps, a.nchunks - t0);
    const int H = a.H, W = a.W;
    constexpr int runq = (kRawW * C + 3) / 4;         // float4s per staged input row run (all C channels)
    constexpr int nq = 7 * runq;                      // per chunk
    constexpr int QPT = (nq + kThreads - 1) / kThreads;   // per thread
    constexpr uint32_t cinv = (65536u + C - 1) / C;    // k / C = (k * cinv) >> 16 for k < 2^11
    const long long total = (long long)a.B * H * W * C;

    // a loader position (image, output row, segment) advanced one chunk at a time
    struct Pos {
        int seg, oh, b;
    };
    auto pos_of = [&](int t) {
        Pos p;
        const int rr = t / a.nseg;
        p.seg = t - rr * a.nseg;
        p.b = rr / a.Ho;
        p.oh = rr - p.b * a.Ho;
        return p;
    };
    auto advance = [&](Pos& p) {
        if (++p.seg == a.nseg) {
            p.seg = 0;
            if (++p.oh == a.Ho) {
                p.oh = 0;
                ++p.b;
            }
        }
    };
    Pos praw = pos_of(t0), pgy = pos_of(t0);
    // raw: float4 q = tid + kThreads j of the chunk's 7 row runs (up to 3 per thread)
    float4 RV[QPT];
    auto load_raw = [&]() {
        const int ih0 = 2 * praw.oh - 3, iw0 = 2 * praw.seg * kSeg - 3;
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            const int q = tid + kThreads * j;
            const int r = q / runq, k = 4 * (q - r * runq);
            const int ih = ih0 + r;
            RV[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (q < nq && (unsigned)ih < (unsigned)H) {
                const long long e0 = ((long long)(praw.b * H + ih) * W + iw0) * C + k;   // may start before the row
                const float* p = a.x + e0;
                if (e0 >= 0 && e0 + 4 <= total) {
                    RV[j] = *(const float4*)p;   // 4-byte aligned dwordx4
                } else {
                    float v[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) v[i] = (e0 + i >= 0 && e0 + i < total) ? p[i] : 0.f;
                    RV[j] = make_float4(v[0], v[1], v[2], v[3]);
                }
            }
        }
    };
    // store the group's channels de-interleaved by column parity; columns outside the
    // image are zeros
    auto store_raw = [&](float* dst) {
        const int iw0 = 2 * praw.seg * kSeg - 3;
#pragma unroll
        for (int j = 0; j < QPT; ++j) {
            const int q = tid + kThreads * j;
            if (q >= nq) break;
            const int r = q / runq, k0 = 4 * (q - r * runq);
            const float v[4] = {RV[j].x, RV[j].y, RV[j].z, RV[j].w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int k = k0 + i, col = (int)(((uint32_t)k * cinv) >> 16), c = k - col * C - kCG * cg;
                const int iw = iw0 + col;
                if (col < kRawW && (unsigned)c < (unsigned)kCG)
                    dst[((r * kCG + c) * 2 + (col & 1)) * kRP + (col >> 1)] = (unsigned)iw < (unsigned)W ? v[i] : 0.f;
            }
        }
    };
    // dy: threads 192 .. 319 (waves 3-4) own a 4-pixel x 4-channel micro-tile
    const int u = tid - 192, kq = u & 7, mq = u >> 3;
    const bool gyrole = u >= 0 && u < 128;
    float4 GV[4];
    auto load_gy = [&]() {
        if (!gyrole) return;
        const int ow0 = pgy.seg * kSeg + 4 * kq;
        const float* row = a.gy + (size_t)(pgy.b * a.Ho + pgy.oh) * a.Wo * kCo + 4 * mq;
#pragma unroll
        for (int i = 0; i < 4; ++i)
            GV[i] = ow0 + i < a.Wo ? *(const float4*)(row + (size_t)(ow0 + i) * kCo) : make_float4(0.f, 0.f, 0.f, 0.f);
    };
    auto store_gy = [&]() {
        if (!gyrole) return;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float c[3][4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float x = j == 0 ? GV[i].x : (j == 1 ? GV[i].y : (j == 2 ? GV[i].z : GV[i].w));
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
                *(u32x2*)(At + pl * kPA + xidx2(4 * mq + j, 4 * kq)) = v;
            }
        }
    };
    // B tiles from the staged rows: task id -> pixel quad g, tile row r (kx = r / 4,
    // ci = r % 4), kernel row kh; four pixels at stride 2 of one staged row
    // only the 21 live rows (kx < 7, ci < 3) of each tile: the dead ones are zeroed once
    constexpr int kLive = 7 * kCG;
    auto build = [&](const float* src) {
#pragma unroll 2
        for (int j = 0; j < (7 * kLive * 8 + kThreads - 1) / kThreads; ++j) {
            const int id = tid + kThreads * j;
            if (id >= 7 * kLive * 8) break;
            const int g = id & 7, rl = (id >> 3) % kLive, kh = (id >> 3) / kLive;
            const int kx = rl / kCG, ci = rl - kx * kCG, r = 4 * kx + ci;
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = src[((kh * kCG + ci) * 2 + (kx & 1)) * kRP + 4 * g + i + (kx >> 1)];
            float c[3][4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float a0 = trunc16(v[i]), r1 = v[i] - a0, a1 = trunc16(r1);
                c[0][i] = a0;
                c[1][i] = a1;
                c[2][i] = r1 - a1;
            }
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) {
                u32x2 q;
                q.x = hi16x2(c[pl][0], c[pl][1]);
                q.y = hi16x2(c[pl][2], c[pl][3]);
                *(u32x2*)(Bt + (kh * 3 + pl) * kPT + xidx2(r, 4 * g)) = q;
            }
        }
    };

    const int lr = lane & 31, h = lane >> 5;
    // one accumulator per row fragment over the split: plan() caps a split at
    // kMaxChunks chunks (2048 pixels)
    f32x16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
    auto mma = [&]() {
        const __bf16* LB = Bt + wid * 3 * kPT;
#pragma unroll
        for (int s = 0; s < kXBK / 16; ++s) {
            bf16x8 fb[3];
            const int eb = xidx2(lr, 16 * s + 8 * h);
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) fb[pl] = *(const bf16x8*)(LB + pl * kPT + eb);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                bf16x8 fa[3];
                const int e = xidx2(32 * i + lr, 16 * s + 8 * h);
#pragma unroll
                for (int pl = 0; pl < 3; ++pl) fa[pl] = *(const bf16x8*)(At + pl * kPA + e);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[2], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[2], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1], fb[0], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[1], acc[i], 0, 0, 0);
                acc[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0], fb[0], acc[i], 0, 0, 0);
            }
        }
    };

    // chunk t's rows are staged (raw[t & 1]) and its dy is in registers at the top of
    // iteration t; chunk t+1's rows are in registers
    for (int e = tid; e < 7 * 3 * 32 * 8; e += kThreads) {   // the tiles' dead rows (kx = 7 or ci = 3)
        const int g = e & 7, r = (e >> 3) & 31, khp = e >> 8;
        if ((r >> 2) == 7 || (r & 3) == kCG) *(u32x2*)(Bt + khp * kPT + xidx2(r, 4 * g)) = u32x2{0u, 0u};
    }
    if (n > 0) {
        load_raw();
        load_gy();
        store_raw(raw[0]);
        advance(praw);
        if (n > 1) load_raw();
    }
    lds_sync();
    for (int t = 0; t < n; ++t) {
        build(raw[t & 1]);
        store_gy();
        if (t + 1 < n) {
            advance(pgy);
            load_gy();
        }
        lds_sync();
        mma();
        if (t + 1 < n) {
            store_raw(raw[(t + 1) & 1]);
            advance(praw);
            if (t + 2 < n) load_raw();
        }
        lds_sync();
    }

    // tile row lr = 4 kx + ci of kernel row wid; output channel per accumulator element
    const int kx = lr >> 2, ci = lr & 3;
    if (kx < 7 && ci < kCG) {
        float* out = a.part + (((size_t)cg * a.splits + ks) * kCo) * kOut + (wid * 7 + kx) * kCG + ci;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int co = 32 * i + (e & 3) + 8 * (e >> 2) + 4 * h;
                out[(size_t)co * kOut] = acc[i][e];
            }
    }
}

// ---------------------------------------------------------------------------------
// Weight gradient without the im2col build (round 4): per kernel row kh the GEMM
// D_kh[co][n] += Σ_p dy[p][co] · X_kh[p][n], n = kw·CP + ci (CP = C padded to 4 / 8),
// K = output pixels.  Both operands need eight consecutive PIXELS of one column per lane
// — the transpose of the staged layouts — and gfx950's ds_read_b64_tr_b16 reads exactly
// that: lane 4q+p of a 16-lane group addresses pixel q's four consecutive elements, lane
// i receives element i of the four pixels.  dy is staged pixel-major ([px][64 co]) and
// the seven input rows under the chunk column-major ([kh][col][CP]); the window of
// output pixel px at tap (kh, kw) starts at column 2 px + kw, so the taps are just
// per-lane addresses into the one staged copy — the old kernel built 7 x 21 x 32 tile
// elements per 32 pixels (the build, not the MFMAs, set its time).  Wave kh (7 waves)
// multiplies its kernel row for all 64 channels x 8·CP n; a chunk is 64 pixels of one
// output row; all channel groups in one block (their dy fragments shared).  Same
// partials as the old kernel ([group][split][64][147]), same final sum.
constexpr int kTSeg = 64, kTWaves = 7, kTThreads = 64 * kTWaves;
constexpr int kTCols = 136;   // staged input columns (2·63 + 7 + 1 = 134 used)
__device__ __forceinline__ int tr_goff(int px, int co4) {   // dy: 4 pixels of one parity on distinct banks
    const int sw = ((px >> 1) & 1) | (((px >> 3) & 1) << 1);
    return px * kCo + 4 * (co4 ^ (sw << 2));
}
typedef short s16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ bf16x8 tr_pair(const __bf16* lo, const __bf16* hi) {
    const s16x4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)lo);
    const s16x4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)hi);
    return __builtin_bit_cast(bf16x8, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int C, bool BF = false, bool PF = BF>
__global__ __launch_bounds__(kTThreads, 2) void stem_x6_wgrad_tr_kernel(StemArgs a) {
    // CP: channels per staged column — 3 padded to 4 (a column pair is then 8-byte
    // aligned for the tr read); 6 unpadded (24-byte column pairs are 8-byte aligned, a
    // 4-element read may run into the next column, which is the next window tap anyway):
    // 48 instead of 64 n per kernel row for 42 real
    constexpr int CP = C == 3 ? 4 : 6, NB = (7 * CP + 15) / 16;   // n blocks of 16 per kernel row
    constexpr int XE = 7 * kTCols * CP, GE = kTSeg * kCo;
    // BF (MD2_STEM_BF16): x and dy are bf16 (config C5's autocast stem) — staged as they
    // are into one plane, one MFMA per fragment pair
    constexpr int NPL = BF ? 1 : 3;
    __shared__ __attribute__((aligned(16))) __bf16 xs[NPL][XE];
    __shared__ __attribute__((aligned(16))) __bf16 gs[NPL][GE];
    const uint16_t* xh = (const uint16_t*)a.x;
    const uint16_t* gh = (const uint16_t*)a.gy;
    const int tid = threadIdx.x, lane = tid & 63, kh = tid >> 6;
    const int ks = blockIdx.x;
    const int t0 = ks * a.cps, n = min(a.cps, a.nchunks - t0);
    const int g16 = lane >> 4, q = (lane >> 2) & 3, p4 = lane & 3;
    f32x4 acc[4][NB];
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < NB; ++ni) acc[mi][ni] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int H = a.H, W = a.W;
    auto compute = [&]() {
#pragma unroll
        for (int kk = 0; kk < kTSeg / 32; ++kk) {
            const int px = 32 * kk + 8 * g16 + q;   // this lane's pixel of the tr reads (and + 4)
            bf16x8 fb[NB][NPL];
#pragma unroll
            for (int ni = 0; ni < NB; ++ni) {
                // n0 = kw·CP + ci0: element (2 px + kw)·CP + ci0 = 2 px·CP + n0 of the row
                const int n0 = 16 * ni + 4 * p4;
                const int olo = (kh * kTCols + 2 * px) * CP + n0;
                const int ohi = (kh * kTCols + 2 * (px + 4)) * CP + n0;
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) fb[ni][pl] = tr_pair(&xs[pl][olo], &xs[pl][ohi]);
            }
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                bf16x8 fa[NPL];
                const int glo = tr_goff(px, 4 * mi + p4), ghi = tr_goff(px + 4, 4 * mi + p4);
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) fa[pl] = tr_pair(&gs[pl][glo], &gs[pl][ghi]);
#pragma unroll
                for (int ni = 0; ni < NB; ++ni) {
                    if constexpr (BF) {
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][0], acc[mi][ni], 0, 0, 0);
                        continue;
                    }
                    f32x4 c = acc[mi][ni];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][1], c, 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][0], c, 0, 0, 0);
                }
            }
        }
    };
    if constexpr (PF) {
        // PF: the next chunk's dy and input rows are loaded into registers while this
        // chunk's MFMAs run (stage -> barrier -> MFMAs -> barrier per chunk left the
        // MFMAs waiting on every chunk's loads), then stored to LDS (fp32: split into the
        // three planes) as the loop below does
        constexpr int NGT = kTSeg * 16, LG = (NGT + kTThreads - 1) / kTThreads;
        constexpr int NXT = CP == 4 ? 7 * (2 * kTSeg + 6) : 7 * ((2 * kTSeg + 6) * CP / 4);
        constexpr int LX = (NXT + kTThreads - 1) / kTThreads;
        using RT = typename std::conditional<BF, uint2, float4>::type;
        RT rg[LG], rx[LX];
        auto put3 = [&](__bf16* base, int stride, int o, float4 v) {   // three exact planes
            const float e[4] = {v.x, v.y, v.z, v.w};
            float c[3][4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a0 = trunc16(e[j]), r1 = e[j] - a0, a1 = trunc16(r1);
                c[0][j] = a0;
                c[1][j] = a1;
                c[2][j] = r1 - a1;
            }
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                *(u32x2*)(base + pl * stride + o) = u32x2{hi16x2(c[pl][0], c[pl][1]), hi16x2(c[pl][2], c[pl][3])};
        };
        auto fetch = [&](int tt) {
            const int per_img = a.nseg * a.Ho, b = tt / per_img, rem = tt - b * per_img;
            const int seg = rem / a.Ho, oh = rem - seg * a.Ho;
            const int ow0 = seg * kTSeg, iw0 = 2 * ow0 - 3;
#pragma unroll
            for (int k = 0; k < LG; ++k) {
                const int i = tid + k * kTThreads;
                const int px = i >> 4, co4 = i & 15, ow = ow0 + px;
                const size_t go = ((size_t)(b * a.Ho + oh) * a.Wo + ow) * kCo + 4 * co4;
                if constexpr (BF) rg[k] = (i < NGT && ow < a.Wo) ? *(const uint2*)(gh + go) : uint2{0u, 0u};
                else rg[k] = (i < NGT && ow < a.Wo) ? *(const float4*)(a.gy + go) : float4{0.f, 0.f, 0.f, 0.f};
            }
            if constexpr (BF) {
#pragma unroll
            for (int k = 0; k < LX; ++k) {
                const int e = tid + k * kTThreads;
                uint32_t h0 = 0u, h1 = 0u;
                if (e < NXT) {
                    if constexpr (CP == 4) {
                        const int r = e / (2 * kTSeg + 6), col = e - r * (2 * kTSeg + 6);
                        const int ih = 2 * oh - 3 + r, iw = iw0 + col;
                        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
                            const uint16_t* px = xh + ((size_t)(b * H + ih) * W + iw) * C;
                            uint32_t hh[4] = {0u, 0u, 0u, 0u};
#pragma unroll
                            for (int ci = 0; ci < C; ++ci) hh[ci] = px[ci];
                            h0 = hh[0] | (hh[1] << 16);
                            h1 = hh[2] | (hh[3] << 16);
                        }
                    } else {
                        constexpr int RQ = (2 * kTSeg + 6) * CP / 4;
                        const int r = e / RQ, kq = 4 * (e - r * RQ);
                        const int ih = 2 * oh - 3 + r;
                        if ((unsigned)ih < (unsigned)H) {
                            const long long f0 = (long long)iw0 * C + kq;
                            const uint16_t* row = xh + (size_t)(b * H + ih) * W * C;
                            if (f0 >= 0 && f0 + 4 <= (long long)W * C) {
                                h0 = *(const uint32_t*)(row + f0);
                                h1 = *(const uint32_t*)(row + f0 + 2);
                            } else {
                                uint32_t hh[2] = {0u, 0u};
#pragma unroll
                                for (int q2 = 0; q2 < 4; ++q2)
                                    if (f0 + q2 >= 0 && f0 + q2 < (long long)W * C)
                                        hh[q2 / 2] |= (uint32_t)row[f0 + q2] << (16 * (q2 & 1));
                                h0 = hh[0];
                                h1 = hh[1];
                            }
                        }
                    }
                }
                rx[k] = uint2{h0, h1};
            }
            } else {
#pragma unroll
            for (int k = 0; k < LX; ++k) {
                const int e = tid + k * kTThreads;
                float v[4] = {0.f, 0.f, 0.f, 0.f};
                if (e < NXT) {
                    if constexpr (CP == 4) {
                        const int r = e / (2 * kTSeg + 6), col = e - r * (2 * kTSeg + 6);
                        const int ih = 2 * oh - 3 + r, iw = iw0 + col;
                        if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
                            const float* px = a.x + ((size_t)(b * H + ih) * W + iw) * C;
#pragma unroll
                            for (int ci = 0; ci < C; ++ci) v[ci] = px[ci];
                        }
                    } else {
                        constexpr int RQ = (2 * kTSeg + 6) * CP / 4;
                        const int r = e / RQ, kq = 4 * (e - r * RQ);
                        const int ih = 2 * oh - 3 + r;
                        if ((unsigned)ih < (unsigned)H) {
                            const long long f0 = (long long)iw0 * C + kq;
                            const float* row = a.x + (size_t)(b * H + ih) * W * C;
                            if (f0 >= 0 && f0 + 4 <= (long long)W * C) {
                                const float4 q4 = *(const float4*)(row + f0);
                                v[0] = q4.x; v[1] = q4.y; v[2] = q4.z; v[3] = q4.w;
                            } else {
#pragma unroll
                                for (int q2 = 0; q2 < 4; ++q2)
                                    if (f0 + q2 >= 0 && f0 + q2 < (long long)W * C) v[q2] = row[f0 + q2];
                            }
                        }
                    }
                }
                rx[k] = float4{v[0], v[1], v[2], v[3]};
            }
            }
        };
        if (n > 0) fetch(t0);
        for (int t = 0; t < n; ++t) {
#pragma unroll
            for (int k = 0; k < LG; ++k) {
                const int i = tid + k * kTThreads;
                if (NGT % kTThreads && i >= NGT) break;
                if constexpr (BF) *(u32x2*)&gs[0][tr_goff(i >> 4, i & 15)] = u32x2{rg[k].x, rg[k].y};
                else put3(&gs[0][0], GE, tr_goff(i >> 4, i & 15), rg[k]);
            }
#pragma unroll
            for (int k = 0; k < LX; ++k) {
                const int e = tid + k * kTThreads;
                if (NXT % kTThreads && e >= NXT) break;
                int o;
                if constexpr (CP == 4) {
                    const int r = e / (2 * kTSeg + 6), col = e - r * (2 * kTSeg + 6);
                    o = (r * kTCols + col) * CP;
                } else {
                    constexpr int RQ = (2 * kTSeg + 6) * CP / 4;
                    const int r = e / RQ;
                    o = r * kTCols * CP + 4 * (e - r * RQ);
                }
                if constexpr (BF) *(u32x2*)&xs[0][o] = u32x2{rx[k].x, rx[k].y};
                else put3(&xs[0][0], XE, o, rx[k]);
            }
            __syncthreads();
            if (t + 1 < n) fetch(t0 + t + 1);
            compute();
            __syncthreads();
        }
    } else {
    for (int t = 0; t < n; ++t) {
        // chunks column-major within an image (oh fastest, then the 64-pixel segment): a
        // block's consecutive chunks share 5 of their 7 input rows, so its working set in
        // L2 is one column strip (row-major order streamed whole 640-wide rows through
        // every block: L2 hit 0.31, 473 MB fetched for ~260 MB of operands at C = 6)
        const int tt = t0 + t, per_img = a.nseg * a.Ho, b = tt / per_img, rem = tt - b * per_img;
        const int seg = rem / a.Ho, oh = rem - seg * a.Ho;
        const int ow0 = seg * kTSeg, iw0 = 2 * ow0 - 3;
        // dy: 64 pixels x 16 channel quads
        for (int i = tid; i < kTSeg * 16; i += kTThreads) {
            const int px = i >> 4, co4 = i & 15, ow = ow0 + px;
            if constexpr (BF) {
                uint2 v = {0u, 0u};
                if (ow < a.Wo) v = *(const uint2*)(gh + ((size_t)(b * a.Ho + oh) * a.Wo + ow) * kCo + 4 * co4);
                *(u32x2*)&gs[0][tr_goff(px, co4)] = u32x2{v.x, v.y};
                continue;
            }
            float4 v = {0.f, 0.f, 0.f, 0.f};
            if (ow < a.Wo) v = *(const float4*)(a.gy + ((size_t)(b * a.Ho + oh) * a.Wo + ow) * kCo + 4 * co4);
            const float e[4] = {v.x, v.y, v.z, v.w};
            float c[3][4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float a0 = trunc16(e[j]), r1 = e[j] - a0, a1 = trunc16(r1);
                c[0][j] = a0;
                c[1][j] = a1;
                c[2][j] = r1 - a1;
            }
            const int o = tr_goff(px, co4);
#pragma unroll
            for (int pl = 0; pl < NPL; ++pl) *(u32x2*)&gs[pl][o] = u32x2{hi16x2(c[pl][0], c[pl][1]), hi16x2(c[pl][2], c[pl][3])};
        }
        if constexpr (CP == 4) {
            // the seven input rows, one column (3 channels + a zero) per task: three
            // loads, one 8-byte store per plane
            for (int e = tid; e < 7 * (2 * kTSeg + 6); e += kTThreads) {
                const int r = e / (2 * kTSeg + 6), col = e - r * (2 * kTSeg + 6);
                const int ih = 2 * oh - 3 + r, iw = iw0 + col;
                if constexpr (BF) {
                    uint32_t h[4] = {0u, 0u, 0u, 0u};
                    if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
                        const uint16_t* px = xh + ((size_t)(b * H + ih) * W + iw) * C;
#pragma unroll
                        for (int ci = 0; ci < C; ++ci) h[ci] = px[ci];
                    }
                    *(u32x2*)&xs[0][(r * kTCols + col) * CP] = u32x2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
                    continue;
                }
                float v[4] = {0.f, 0.f, 0.f, 0.f};
                if ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) {
                    const float* px = a.x + ((size_t)(b * H + ih) * W + iw) * C;
#pragma unroll
                    for (int ci = 0; ci < C; ++ci) v[ci] = px[ci];
                }
                const int o = (r * kTCols + col) * CP;
                u32x2 pk[3];
#pragma unroll
                for (int j = 0; j < 4; j += 2) {
                    const float a0 = trunc16(v[j]), r0 = v[j] - a0, m0 = trunc16(r0);
                    const float a1 = trunc16(v[j + 1]), r1 = v[j + 1] - a1, m1 = trunc16(r1);
                    pk[0][j / 2] = hi16x2(a0, a1);
                    pk[1][j / 2] = hi16x2(m0, m1);
                    pk[2][j / 2] = hi16x2(r0 - m0, r1 - m1);
                }
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) *(u32x2*)&xs[pl][o] = pk[pl];
            }
        } else {
            // C = 6: each row's 134 columns x 6 channels are one contiguous run of the
            // NHWC input, staged as is: four floats per task, one 8-byte store per plane
            constexpr int RQ = (2 * kTSeg + 6) * CP / 4;   // float quads per row run
            for (int e = tid; e < 7 * RQ; e += kTThreads) {
                const int r = e / RQ, k = 4 * (e - r * RQ);
                const int ih = 2 * oh - 3 + r;
                if constexpr (BF) {
                    // four bf16 of the row run (element f0 is even: two 4-byte loads)
                    uint32_t h[2] = {0u, 0u};
                    if ((unsigned)ih < (unsigned)H) {
                        const long long f0 = (long long)iw0 * C + k;
                        const uint16_t* row = xh + (size_t)(b * H + ih) * W * C;
                        if (f0 >= 0 && f0 + 4 <= (long long)W * C) {
                            h[0] = *(const uint32_t*)(row + f0);
                            h[1] = *(const uint32_t*)(row + f0 + 2);
                        } else {
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                if (f0 + i >= 0 && f0 + i < (long long)W * C) h[i / 2] |= (uint32_t)row[f0 + i] << (16 * (i & 1));
                        }
                    }
                    *(u32x2*)&xs[0][r * kTCols * CP + k] = u32x2{h[0], h[1]};
                    continue;
                }
                float v[4] = {0.f, 0.f, 0.f, 0.f};
                if ((unsigned)ih < (unsigned)H) {
                    const long long f0 = (long long)iw0 * C + k;   // element of the row, may be < 0
                    const float* row = a.x + (size_t)(b * H + ih) * W * C;
                    if (f0 >= 0 && f0 + 4 <= (long long)W * C) {
                        const float4 q4 = *(const float4*)(row + f0);
                        v[0] = q4.x; v[1] = q4.y; v[2] = q4.z; v[3] = q4.w;
                    } else {
#pragma unroll
                        for (int i = 0; i < 4; ++i)
                            if (f0 + i >= 0 && f0 + i < (long long)W * C) v[i] = row[f0 + i];
                    }
                }
                const int o = r * kTCols * CP + k;
                u32x2 pk[3];
#pragma unroll
                for (int j = 0; j < 4; j += 2) {
                    const float a0 = trunc16(v[j]), r0 = v[j] - a0, m0 = trunc16(r0);
                    const float a1 = trunc16(v[j + 1]), r1 = v[j + 1] - a1, m1 = trunc16(r1);
                    pk[0][j / 2] = hi16x2(a0, a1);
                    pk[1][j / 2] = hi16x2(m0, m1);
                    pk[2][j / 2] = hi16x2(r0 - m0, r1 - m1);
                }
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) *(u32x2*)&xs[pl][o] = pk[pl];
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kTSeg / 32; ++kk) {
            const int px = 32 * kk + 8 * g16 + q;   // this lane's pixel of the tr reads (and + 4)
            bf16x8 fb[NB][NPL];
#pragma unroll
            for (int ni = 0; ni < NB; ++ni) {
                // n0 = kw·CP + ci0: element (2 px + kw)·CP + ci0 = 2 px·CP + n0 of the row
                const int n0 = 16 * ni + 4 * p4;
                const int olo = (kh * kTCols + 2 * px) * CP + n0;
                const int ohi = (kh * kTCols + 2 * (px + 4)) * CP + n0;
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) fb[ni][pl] = tr_pair(&xs[pl][olo], &xs[pl][ohi]);
            }
#pragma unroll
            for (int mi = 0; mi < 4; ++mi) {
                bf16x8 fa[NPL];
                const int glo = tr_goff(px, 4 * mi + p4), ghi = tr_goff(px + 4, 4 * mi + p4);
#pragma unroll
                for (int pl = 0; pl < NPL; ++pl) fa[pl] = tr_pair(&gs[pl][glo], &gs[pl][ghi]);
#pragma unroll
                for (int ni = 0; ni < NB; ++ni) {
                    if constexpr (BF) {
                        acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][0], acc[mi][ni], 0, 0, 0);
                        continue;
                    }
                    f32x4 c = acc[mi][ni];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[2], fb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[ni][1], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][2], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1], fb[ni][0], c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][1], c, 0, 0, 0);
                    acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0], fb[ni][0], c, 0, 0, 0);
                }
            }
        }
        __syncthreads();   // restaged next chunk
    }
    }
    // D[row = co = 16 mi + 4 g16 + e][col = n = 16 ni + lane & 15], n = kw·CP + ci
#pragma unroll
    for (int ni = 0; ni < NB; ++ni) {
        const int nn = 16 * ni + (lane & 15), kw = nn / CP, ci = nn - kw * CP;
        if (kw >= 7 || ci >= C) continue;
        const int cg = ci / kCG, cl = ci - cg * kCG;
        float* out = a.part + ((size_t)cg * a.splits + ks) * kCo * kOut + (kh * 7 + kw) * kCG + cl;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
            for (int e = 0; e < 4; ++e) out[(size_t)(16 * mi + 4 * g16 + e) * kOut] = acc[mi][ni][e];
    }
}

// dW = Σ_splits partials: sixteen lanes per output, lane l summing splits l, l + 16, ...
// in order, then the sixteen in lane order (deterministic); written in the weight's
// memory format.  (Four lanes per output ran long serial chains over the ~500 splits.)
constexpr int kFinOut = 16, kFinLanes = 256 / kFinOut;
__global__ __launch_bounds__(256) void stem_wgrad_final_kernel(StemArgs a) {
    const int NG = a.C / kCG, outs = NG * kCo * kOut;
    const int el = threadIdx.x % kFinOut, sl = threadIdx.x / kFinOut;
    const int e = blockIdx.x * kFinOut + el;
    float s = 0.f;
    if (e < outs) {
        const int cg = e / (kCo * kOut), r = e - cg * kCo * kOut;   // r = co * 147 + tap
        const float* p = a.part + (size_t)cg * a.splits * kCo * kOut + r;
#pragma unroll 4
        for (int g = sl; g < a.splits; g += kFinLanes) s += p[(size_t)g * kCo * kOut];
    }
    __shared__ float red[kFinLanes][kFinOut];
    red[sl][el] = s;
    __syncthreads();
    if (sl != 0 || e >= outs) return;
#pragma unroll
    for (int j = 1; j < kFinLanes; ++j) s += red[j][el];
    const int cg = e / (kCo * kOut), r = e - cg * kCo * kOut, co = r / kOut, tap = r - co * kOut;
    const int ky = tap / (7 * kCG), rem = tap - ky * 7 * kCG, kx = rem / kCG, ci = kCG * cg + rem - kx * kCG;
    if (a.w_cl) a.gw[((co * 7 + ky) * 7 + kx) * a.C + ci] = s;
    else a.gw[((co * a.C + ci) * 7 + ky) * 7 + kx] = s;
}

// ---------------------------------------------------------------------------------
// Forward: y[p][co] = Σ_kh Σ_k X_kh[p][k] · W[kh][k][co], a GEMM with M = output pixels,
// N = 64, K = 7 kernel rows x KP.  Within one kernel row the 7 x C window taps of an
// output pixel are C·7 CONSECUTIVE floats of the NHWC input row — x[ih][2 ow - 3 + kx][ci]
// sits at flat offset (2 ow - 3)·C + k with k = kx·C + ci — so an MFMA A fragment (eight
// consecutive k of one pixel) is two float4 loads straight from the input, no im2col:
// lanes of one pixel group read overlapping windows, the overlap served by L1.  K is
// padded to KP = 16·⌈7C/16⌉ with zero weights (C = 3: 21 -> 32, C = 6: 42 -> 48).
// The fragments are split into bf16 planes in registers (exact truncation split, six
// products: f32-class, conv.hip's x6 scheme); the weights, split once per block into
// their fragment image in LDS (84 KB at C = 3, 126 KB at C = 6), are read conflict-free
// as 1-KB runs.  A wave owns 64 pixels of one output row x all 64 channels (2 x 2
// 32x32 accumulators) and walks its tiles persistently; the next step's fragments are
// loaded behind the current step's 24 MFMAs.  MIOpen's igemm_fwd ran these at 89 /
// 334 us (B = 12, C = 3 / B = 24, C = 6; 192x640).
constexpr int kFwdWaves = 8;
constexpr int kFwdSeg = 64;   // output pixels per wave tile

struct StemFwdArgs {
    int B, C, H, W, Ho, Wo;
    int w_cl;
    int nseg, tiles;
    const float* x;
    const float* w;
    float* y;
};

// One wave tile (64 pixels of output row oh x 64 channels).  EDGE: window rows outside
// the image or fragments crossing a row end (zeros), pixels past the row (not stored).
// The (kernel row, k step) loop is unrolled with its fragment loads kPD steps ahead.
constexpr int kPD = 3;
// BF (MD2_STEM_BF16, config C5): x and y are bf16, the weight image one plane rounded to
// nearest even (autocast's cast), one MFMA per fragment pair, y rounded once (RNE).
template <int C, bool EDGE, bool BF = false>
__device__ __forceinline__ void stem_fwd_tile(const StemFwdArgs& a, const u32x4* __restrict__ wf, int b, int oh,
                                              int ow0, int lane) {
    constexpr int KP = (7 * C + 15) / 16 * 16, S = KP / 16, NQ = 7 * S;
    constexpr int NPL = BF ? 1 : 3;
    const int lr = lane & 31, h = lane >> 5;
    const int H = a.H, rowlen = a.W * C;
    const float* img = a.x + (size_t)b * H * rowlen;
    const uint16_t* imgh = (const uint16_t*)a.x + (size_t)b * H * rowlen;
    int base[2];
#pragma unroll
    for (int p = 0; p < 2; ++p) base[p] = (2 * (ow0 + 32 * p + lr) - 3) * C + 8 * h;
    // step q = (kh, s): the two pixel groups' eight k values, from input row 2 oh - 3 + kh
    auto load = [&](int q, float (&r)[2][8]) {
        const int kh = q / S, s = q - kh * S, ih = 2 * oh - 3 + kh;
        const bool rowok = !EDGE || (unsigned)ih < (unsigned)H;
        const float* rowp = img + (size_t)(rowok ? ih : 0) * rowlen;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int o = base[p] + 16 * s;
            if (!EDGE || (rowok && o >= 0 && o + 8 <= rowlen)) {
                const float4 u = *(const float4*)(rowp + o), v = *(const float4*)(rowp + o + 4);
                r[p][0] = u.x; r[p][1] = u.y; r[p][2] = u.z; r[p][3] = u.w;
                r[p][4] = v.x; r[p][5] = v.y; r[p][6] = v.z; r[p][7] = v.w;
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int f = o + i;
                    r[p][i] = (rowok && f >= 0 && f < rowlen) ? rowp[f] : 0.f;
                }
            }
        }
    };
    // BF: the eight bf16 k values of a pixel group as four packed pairs.  Their first
    // element (2 ow - 3) C + 8 h + 16 s is odd at C = 3 (two dword-aligned loads, funnel
    // shifted by 16 bits) and even at C = 6
    auto load_bf = [&](int q, uint32_t (&r)[2][4]) {
        const int kh = q / S, s = q - kh * S, ih = 2 * oh - 3 + kh;
        const bool rowok = !EDGE || (unsigned)ih < (unsigned)H;
        const uint16_t* rowp = imgh + (size_t)(rowok ? ih : 0) * rowlen;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int o = base[p] + 16 * s;
            if (!EDGE || (rowok && o >= 1 && o + 9 <= rowlen)) {
                const uint32_t* dp = (const uint32_t*)(rowp + (o & ~1));
                const u32x4 d = *(const u32x4*)dp;
                if constexpr (C % 2 == 1) {   // o odd
                    const uint32_t d4 = dp[4];
                    r[p][0] = __builtin_amdgcn_alignbyte(d[1], d[0], 2);
                    r[p][1] = __builtin_amdgcn_alignbyte(d[2], d[1], 2);
                    r[p][2] = __builtin_amdgcn_alignbyte(d[3], d[2], 2);
                    r[p][3] = __builtin_amdgcn_alignbyte(d4, d[3], 2);
                } else {
                    r[p][0] = d[0]; r[p][1] = d[1]; r[p][2] = d[2]; r[p][3] = d[3];
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; i += 2) {
                    const int f = o + i;
                    const uint32_t lo = (rowok && f >= 0 && f < rowlen) ? rowp[f] : 0u;
                    const uint32_t hi = (rowok && f + 1 >= 0 && f + 1 < rowlen) ? rowp[f + 1] : 0u;
                    r[p][i / 2] = lo | (hi << 16);
                }
            }
        }
    };
    f32x16 acc[2][2];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int e = 0; e < 16; ++e) acc[p][j][e] = 0.f;
    if constexpr (BF) {
        uint32_t rb[kPD + 1][2][4];
#pragma unroll
        for (int q = 0; q < kPD && q < NQ; ++q) load_bf(q, rb[q]);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            if (q + kPD < NQ) load_bf(q + kPD, rb[(q + kPD) % (kPD + 1)]);
            const uint32_t (&cur)[2][4] = rb[q % (kPD + 1)];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const bf16x8 fb = __builtin_bit_cast(bf16x8, wf[(q * 2 + j) * 64 + lane]);
#pragma unroll
                for (int p = 0; p < 2; ++p) {
                    const bf16x8 fa = __builtin_bit_cast(bf16x8, u32x4{cur[p][0], cur[p][1], cur[p][2], cur[p][3]});
                    acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc[p][j], 0, 0, 0);
                }
            }
        }
        uint16_t* yrow = (uint16_t*)a.y + (size_t)(b * a.Ho + oh) * a.Wo * kCo;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int e = 0; e < 16; ++e) {
                const int ow = ow0 + 32 * p + (e & 3) + 8 * (e >> 2) + 4 * h;
                if (!EDGE || ow < a.Wo) {
#pragma unroll
                    for (int j = 0; j < 2; ++j) yrow[(size_t)ow * kCo + 32 * j + lr] = f2bf16(acc[p][j][e]);
                }
            }
        return;
    }
    float raw[kPD + 1][2][8];
#pragma unroll
    for (int q = 0; q < kPD && q < NQ; ++q) load(q, raw[q]);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
        if (q + kPD < NQ) load(q + kPD, raw[(q + kPD) % (kPD + 1)]);
        const float (&cur)[2][8] = raw[q % (kPD + 1)];
        bf16x8 fa[2][3];
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            uint32_t pk[3][4];
#pragma unroll
            for (int i = 0; i < 8; i += 2) {
                const float x0 = cur[p][i], x1 = cur[p][i + 1];
                const float a0 = trunc16(x0), r0 = x0 - a0, m0 = trunc16(r0);
                const float a1 = trunc16(x1), r1 = x1 - a1, m1 = trunc16(r1);
                pk[0][i / 2] = hi16x2(a0, a1);
                pk[1][i / 2] = hi16x2(m0, m1);
                pk[2][i / 2] = hi16x2(r0 - m0, r1 - m1);
            }
#pragma unroll
            for (int pl = 0; pl < 3; ++pl)
                fa[p][pl] = __builtin_bit_cast(bf16x8, u32x4{pk[pl][0], pk[pl][1], pk[pl][2], pk[pl][3]});
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            bf16x8 fb[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) fb[pl] = __builtin_bit_cast(bf16x8, wf[((q * 2 + j) * 3 + pl) * 64 + lane]);
#pragma unroll
            for (int p = 0; p < 2; ++p) {
                acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[p][2], fb[0], acc[p][j], 0, 0, 0);
                acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[p][1], fb[1], acc[p][j], 0, 0, 0);
                acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[p][0], fb[2], acc[p][j], 0, 0, 0);
                acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[p][1], fb[0], acc[p][j], 0, 0, 0);
                acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[p][0], fb[1], acc[p][j], 0, 0, 0);
                acc[p][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[p][0], fb[0], acc[p][j], 0, 0, 0);
            }
        }
    }
    // D row (pixel) = 32 p + (e & 3) + 8 (e >> 2) + 4 h, column (channel) = 32 j + lr
    float* yrow = a.y + (size_t)(b * a.Ho + oh) * a.Wo * kCo;
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
            const int ow = ow0 + 32 * p + (e & 3) + 8 * (e >> 2) + 4 * h;
            if (!EDGE || ow < a.Wo) {
#pragma unroll
                for (int j = 0; j < 2; ++j) yrow[(size_t)ow * kCo + 32 * j + lr] = acc[p][j][e];
            }
        }
}

template <int C, bool BF = false>
__global__ __launch_bounds__(64 * kFwdWaves, 1) void stem_x6_fwd_kernel(StemFwdArgs a) {
    constexpr int KP = (7 * C + 15) / 16 * 16, S = KP / 16;
    constexpr int NQ = 7 * S;                       // (kernel row, k step) pairs
    constexpr int NPL = BF ? 1 : 3;
    __shared__ u32x4 wf[NQ * 2 * NPL * 64];         // [kh][s][co half][plane][lane] x 8 bf16
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // the weight fragment image: lane l of fragment (kh, s, j) holds W[kh][16 s + 8 h + i][32 j + l % 32]
#pragma unroll
    for (int id = tid; id < NQ * 2 * 64; id += 64 * kFwdWaves) {   // unrolled: the rounds' loads in flight together
        const int l = id & 63, j = (id >> 6) & 1, q = id >> 7;
        const int kh = q / S, s = q - kh * S;
        const int co = 32 * j + (l & 31), k0 = 16 * s + 8 * (l >> 5);
        float c[3][8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int k = k0 + i, kw = k / C, ci = k - kw * C;
            float v = 0.f;
            if (k < 7 * C)
                v = a.w_cl ? a.w[((co * 7 + kh) * 7 + kw) * C + ci] : a.w[((co * C + ci) * 7 + kh) * 7 + kw];
            if constexpr (BF) v = bf16_rne(v);   // autocast's cast of the weight: plane 0 alone
            const float a0 = trunc16(v), r1 = v - a0, a1 = trunc16(r1);
            c[0][i] = a0;
            c[1][i] = a1;
            c[2][i] = r1 - a1;
        }
#pragma unroll
        for (int pl = 0; pl < NPL; ++pl)
            wf[((q * 2 + j) * NPL + pl) * 64 + l] = u32x4{hi16x2(c[pl][0], c[pl][1]), hi16x2(c[pl][2], c[pl][3]),
                                                          hi16x2(c[pl][4], c[pl][5]), hi16x2(c[pl][6], c[pl][7])};
    }
    __syncthreads();

    // blocks are dealt round-robin over the 8 XCDs: renumber them so each XCD's blocks
    // are consecutive — its concurrent tiles are then neighbouring output rows sharing
    // input rows in its own L2 (a pose-stem pass read ~400 MB for ~260 MB of operands)
    const int bid = xcd_contiguous_block(blockIdx.x, gridDim.x);
    for (int t = bid * kFwdWaves + wid; t < a.tiles; t += gridDim.x * kFwdWaves) {
        const int rr = t / a.nseg, seg = t - rr * a.nseg, b = rr / a.Ho, oh = rr - b * a.Ho;
        const int ow0 = seg * kFwdSeg;
        // interior tile: every window row in the image and every fragment inside its row
        // (BF at odd C reads one element past a fragment: the funnel shift's extra half)
        constexpr int XTRA = (BF && (C & 1)) ? 1 : 0;
        const bool inner = 2 * oh - 3 >= 0 && 2 * oh + 3 < a.H && ow0 >= 2 &&
                           (2 * (ow0 + kFwdSeg - 1) - 3) * C + KP + XTRA <= a.W * C && ow0 + kFwdSeg <= a.Wo;
        if (inner) stem_fwd_tile<C, false, BF>(a, wf, b, oh, ow0, lane);
        else stem_fwd_tile<C, true, BF>(a, wf, b, oh, ow0, lane);
    }
}

bool valid(const md2_stem_desc* d) {
    return d && d->batch >= 1 && d->height >= 1 && d->width >= 1 &&
           (d->channels == 3 || d->channels == 6 || d->channels == 9) &&
           (long long)d->batch * d->height * d->width * d->channels < (1ll << 31);
}

// geometry and K split: about two blocks per CU over the channel groups, every split
// at least one chunk
StemArgs plan(const md2_stem_desc* d) {
    StemArgs a = {};
    a.B = d->batch;
    a.C = d->channels;
    a.H = d->height;
    a.W = d->width;
    a.Ho = (d->height - 1) / 2 + 1;   // (H + 2·3 - 7) / 2 + 1
    a.Wo = (d->width - 1) / 2 + 1;
    a.w_cl = (d->flags & MD2_STEM_WEIGHT_CL) ? 1 : 0;
    a.nseg = (a.Wo + kSeg - 1) / kSeg;
    a.nchunks = a.B * a.Ho * a.nseg;
    const int NG = a.C / kCG;
    int want = 256 * kBlocksPerCU / NG;
    want = want < 1 ? 1 : want;
    const int need = (a.nchunks + kMaxChunks - 1) / kMaxChunks;
    want = want > need ? want : need;
    a.cps = (a.nchunks + want - 1) / want;
    a.splits = (a.nchunks + a.cps - 1) / a.cps;
    return a;
}

// the transposed-read kernel (C = 3 / 6): 64-pixel chunks, all channel groups per block,
// about two blocks per CU, at most 32 chunks (2048 pixels) per K split
bool use_tr(const md2_stem_desc* d) {
    static const bool build = [] {   // A/B knob: MD2_STEM_WGRAD_BUILD=1 runs the im2col-build kernel
        const char* e = getenv("MD2_STEM_WGRAD_BUILD");
        return e && e[0] == '1';
    }();
    return !build && (d->channels == 3 || d->channels == 6);
}

StemArgs plan_tr(const md2_stem_desc* d) {
    StemArgs a = plan(d);
    a.nseg = (a.Wo + kTSeg - 1) / kTSeg;
    a.nchunks = a.B * a.Ho * a.nseg;
    int want = 256 * 2;
    const int need = (a.nchunks + 31) / 32;
    want = want > need ? want : need;
    a.cps = (a.nchunks + want - 1) / want;
    a.splits = (a.nchunks + a.cps - 1) / a.cps;
    return a;
}

}  // namespace

extern "C" {

size_t md2_stem_wgrad_workspace_bytes(const md2_stem_desc* d) {
    if (!valid(d)) return 0;
    const StemArgs a = use_tr(d) ? plan_tr(d) : plan(d);
    return sizeof(float) * (size_t)(a.C / kCG) * a.splits * kCo * kOut;
}

int md2_stem_wgrad(const md2_stem_desc* d, const float* x, const float* grad_y, float* grad_weight, void* workspace,
                   void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "stem_wgrad: channels 3/6/9, 32-bit element count");
    if (!x || !grad_y || !grad_weight || !workspace) return md2_report_error(MD2_ERR_ARG, "stem_wgrad: NULL operand");
    const bool tr = use_tr(d);
    if ((d->flags & MD2_STEM_BF16) && !tr)
        return md2_report_error(MD2_ERR_ARG, "stem_wgrad: bf16 operands (MD2_STEM_BF16) need channels 3 / 6");
    StemArgs a = tr ? plan_tr(d) : plan(d);
    a.x = x;
    a.gy = grad_y;
    a.part = (float*)workspace;
    a.gw = grad_weight;
    const int NG = a.C / kCG;
    const hipStream_t st = (hipStream_t)stream;
    if (tr) {
        const bool bf = (d->flags & MD2_STEM_BF16) != 0;
        static const bool pf32 = [] {   // A/B knob: MD2_STEM_PF32=1 prefetches in the fp32 form too
            const char* e = getenv("MD2_STEM_PF32");
            return e && e[0] == '1';
        }();
        void (*k)(StemArgs) =
            a.C == 3 ? (bf ? stem_x6_wgrad_tr_kernel<3, true>
                           : (pf32 ? stem_x6_wgrad_tr_kernel<3, false, true> : stem_x6_wgrad_tr_kernel<3>))
                     : (bf ? stem_x6_wgrad_tr_kernel<6, true>
                           : (pf32 ? stem_x6_wgrad_tr_kernel<6, false, true> : stem_x6_wgrad_tr_kernel<6>));
        hipLaunchKernelGGL(k, dim3(a.splits), dim3(kTThreads), 0, st, a);
    } else {
        void (*k)(StemArgs) =
            a.C == 3 ? stem_x6_wgrad_kernel<3> : a.C == 6 ? stem_x6_wgrad_kernel<6> : stem_x6_wgrad_kernel<9>;
        hipLaunchKernelGGL(k, dim3(NG * ((a.splits + 7) / 8) * 8), dim3(kThreads), 0, st, a);
    }
    const int outs = NG * kCo * kOut;
    hipLaunchKernelGGL(stem_wgrad_final_kernel, dim3((outs + kFinOut - 1) / kFinOut), dim3(256), 0, st, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

int md2_stem_fwd(const md2_stem_desc* d, const float* x, const float* weight, float* y, void* stream) {
    if (!valid(d) || (d->channels != 3 && d->channels != 6))
        return md2_report_error(MD2_ERR_ARG, "stem_fwd: channels 3/6, 32-bit element count");
    if (!x || !weight || !y) return md2_report_error(MD2_ERR_ARG, "stem_fwd: NULL operand");
    StemFwdArgs a = {};
    a.B = d->batch;
    a.C = d->channels;
    a.H = d->height;
    a.W = d->width;
    a.Ho = (d->height - 1) / 2 + 1;
    a.Wo = (d->width - 1) / 2 + 1;
    a.w_cl = (d->flags & MD2_STEM_WEIGHT_CL) ? 1 : 0;
    a.nseg = (a.Wo + kFwdSeg - 1) / kFwdSeg;
    a.tiles = a.B * a.Ho * a.nseg;
    a.x = x;
    a.w = weight;
    a.y = y;
    // one block per CU (the weight image fills most of the LDS), tiles walked persistently
    const int blocks = std::min(256, (a.tiles + kFwdWaves - 1) / kFwdWaves);
    const bool bf = (d->flags & MD2_STEM_BF16) != 0;   // bf16 x / y (ABI 23)
    void (*k)(StemFwdArgs) = a.C == 3 ? (bf ? stem_x6_fwd_kernel<3, true> : stem_x6_fwd_kernel<3>)
                                      : (bf ? stem_x6_fwd_kernel<6, true> : stem_x6_fwd_kernel<6>);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * kFwdWaves), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
