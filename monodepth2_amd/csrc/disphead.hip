// disphead.hip — the DepthDecoder's disparity heads for gfx950:
//   disp_s = sigmoid(Conv3x3(C -> 1)(P))                 networks/depth_decoder.py:63-64
// where P is the already reflection-padded NHWC conv input that decoder.hip builds
// (layers.py:121-136 Conv3x3 = ReflectionPad2d(1) + Conv2d(C, 1, 3)).
//
// MIOpen runs these C->1 convolutions as implicit GEMMs with N = 1 (one output
// channel): 3-30 TFLOP/s and a zeroing pass + atomics in the weight gradient — about
// 1 ms of a 16 ms training step for ~1.5 GFLOP.  They are HBM-bound streams (9·C MACs
// per output pixel against 4·C bytes of input), so here:
//   * forward: one pass over P; a pixel's C channels are spread over L lanes as
//     float4 quads (L = min(C/4, 16), QL = C/(4L) quads per lane), the lane's 9·QL
//     weight quads held in registers, 9 taps each, shuffle-reduced, bias + sigmoid
//     fused; writes disp (B,1,h,w).  32-bit index math throughout.
//   * backward: blocks walk padded rows (b, Y).  Per row, dz = dD·D·(1-D) of the three
//     output rows that read it (y = Y-2..Y) is staged in LDS once (one sigmoid-backward
//     per output pixel and tap row, instead of one per channel quad); then every
//     (padded pixel, channel quad) gives dP[Y,X,:] = Σ_taps w[tap,:]·dz (a 3x3
//     transposed conv, written once, float4) and, from the same loads,
//     dW[tap,:] += P[Y,X,:]·dz[tap] and db += dz.  Per-block partials (wave shuffles,
//     then LDS) are summed by a second launch in a fixed order (deterministic, no
//     atomics).
// Weights are read in the parameter's own memory format (channels_last: [tap][c],
// contiguous: [c][tap]) and dW is written back in that format.

#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdlib.h>

#include "md2_bf16.h"
#include "md2hot.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxC = 256;
constexpr int kBwdBlocks = 2048;
constexpr int kFwdBlocks = 4096;
constexpr int kMaxLds = 64 * 1024;

struct HeadArgs {
    int B, C, h, w;            // output (B,1,h,w); P is (B,h+2,w+2,C) NHWC
    int w_cl;                  // weight memory format: 1 = [tap][c], 0 = [c][tap]
    const float* P;
    const float* wt;
    const float* bias;         // (1,)
    float* disp;               // (B,1,h,w)
    const float* gdisp;        // (B,1,h,w)
    float* gP;                 // (B,h+2,w+2,C) NHWC
    float* part;               // [gridDim.x][9C + 1] backward partials
    float* gw;                 // (1,C,3,3) in the weight's memory format
    float* gb;                 // (1,)
};

__device__ __forceinline__ float4 wt_quad(const HeadArgs& a, int tap, int q) {
    if (a.w_cl) return reinterpret_cast<const float4*>(a.wt + tap * a.C)[q];
    const int c = q * 4;
    return make_float4(a.wt[c * 9 + tap], a.wt[(c + 1) * 9 + tap], a.wt[(c + 2) * 9 + tap], a.wt[(c + 3) * 9 + tap]);
}

__device__ __forceinline__ float dot4(float4 u, float4 v) { return u.x * v.x + u.y * v.y + u.z * v.z + u.w * v.w; }

// channel quad i of P (float4 units): fp32, or bf16 (MD2_HEAD_BF16: config C5's bf16
// decoder activations, widened exactly); gP quads stored likewise (bf16: rounded to
// nearest even, what autograd's cast of an fp32 gradient back to bf16 gives)
template <bool BF>
__device__ __forceinline__ float4 ld_quad(const float* P, unsigned i) {
    if constexpr (BF) {
        const uint2 u = reinterpret_cast<const uint2*>(P)[i];
        return make_float4(md2::bf2f(u.x & 0xffffu), md2::bf2f(u.x >> 16), md2::bf2f(u.y & 0xffffu),
                           md2::bf2f(u.y >> 16));
    } else {
        return reinterpret_cast<const float4*>(P)[i];
    }
}
template <bool BF>
__device__ __forceinline__ void st_quad(float* G, unsigned i, float4 g) {
    if constexpr (BF)
        reinterpret_cast<uint2*>(G)[i] =
            make_uint2(md2::f2bf(g.x) | (md2::f2bf(g.y) << 16), md2::f2bf(g.z) | (md2::f2bf(g.w) << 16));
    else
        reinterpret_cast<float4*>(G)[i] = g;
}

// L lanes per pixel, QL quads per lane (C = 4·L·QL)
template <int L, int QL>
__global__ __launch_bounds__(kThreads) void head_fwd_kernel(HeadArgs a) {
    constexpr int Q = L * QL;
    const unsigned Wp = a.w + 2, Hp = a.h + 2;
    const int sub = threadIdx.x % L;
    const unsigned npix = (unsigned)a.B * a.h * a.w;
    // each block walks one contiguous pixel range, and the ranges of an XCD's blocks
    // (dealt round-robin: block b runs on XCD b % 8) are contiguous too, so the three
    // padded rows an output row reads are shared in that XCD's L2 (gridDim.x % 8 == 0)
    constexpr unsigned GPB = kThreads / L;   // pixel groups per block
    const unsigned lb = (blockIdx.x % 8) * (gridDim.x / 8) + blockIdx.x / 8;
    constexpr int U = QL == 1 ? 2 : 1;
    const unsigned step = GPB * U;
    const unsigned chunk = ((npix + gridDim.x - 1) / gridDim.x + step - 1) / step * step;
    const unsigned start = lb * chunk, end = start + chunk < npix ? start + chunk : npix;
    const unsigned stride = GPB;
    unsigned pix = start + threadIdx.x / L;
    if (pix >= end) return;   // whole L-lane groups exit together (L divides 64)
    float4 wr[9][QL];          // loaded once, reused for every pixel this group walks
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int k = 0; k < QL; ++k) wr[tap][k] = wt_quad(a, tap, sub + k * L);
    const float bias = a.bias[0];
    const float4* P4 = reinterpret_cast<const float4*>(a.P) + sub;
    // U pixels per iteration: 9·QL·U independent loads in flight per lane
    for (; pix < end; pix += U * stride) {
        unsigned pp[U], base[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            pp[u] = pix + u * stride < end ? pix + u * stride : pix;   // a lone tail pixel is done twice
            const unsigned x = pp[u] % a.w, t = pp[u] / a.w;
            const unsigned y = t % a.h, b = t / a.h;
            base[u] = ((b * Hp + y) * Wp + x) * Q;
        }
        float4 v[U][9][QL];
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx)
#pragma unroll
                    for (int k = 0; k < QL; ++k) v[u][ky * 3 + kx][k] = P4[base[u] + (ky * Wp + kx) * Q + k * L];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            float acc = 0.f;
#pragma unroll
            for (int tap = 0; tap < 9; ++tap)
#pragma unroll
                for (int k = 0; k < QL; ++k) acc += dot4(v[u][tap][k], wr[tap][k]);
#pragma unroll
            for (int o = L / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, L);
            if (sub == 0) a.disp[pp[u]] = 1.f / (1.f + expf(-(acc + bias)));
        }
    }
}

// Column-walk form of the forward (the default): a block owns GPB = 256/L adjacent
// output columns x R output rows of one image; each L-lane group owns one column and
// loads the R + 2 padded rows of its 3-tap window once — (R + 2)·3 float4 loads per lane
// for R pixels instead of 9 per pixel — all of them before any arithmetic, then the
// same tap-ordered dot products, shuffle reduction, bias and sigmoid as head_fwd_kernel
// (bitwise the same outputs).  MD2_HEAD_ROWWALK=1 keeps the pixel-walk kernel above.
template <int L, int QL, bool BF = false>
__global__ __launch_bounds__(kThreads) void head_fwd_col_kernel(HeadArgs a) {
    constexpr int Q = L * QL, GPB = kThreads / L, R = QL >= 4 ? 2 : 8 / QL;
    const int Wp = a.w + 2, Hp = a.h + 2;
    const int sub = threadIdx.x % L, grp = threadIdx.x / L;
    const int ntx = (a.w + GPB - 1) / GPB, nty = (a.h + R - 1) / R;
    int t = blockIdx.x;
    const int tx = t % ntx;
    t /= ntx;
    const int ty = t % nty, b = t / nty;
    const int x = tx * GPB + grp;
    if (x >= a.w) return;   // whole L-lane groups exit together (L divides 64)
    const int y0 = ty * R;
    float4 wr[9][QL];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int k = 0; k < QL; ++k) wr[tap][k] = wt_quad(a, tap, sub + k * L);
    const float bias = a.bias[0];
    float4 v[R + 2][3][QL];
#pragma unroll
    for (int r = 0; r < R + 2; ++r) {
        const int Y = y0 + r < Hp ? y0 + r : Hp - 1;   // rows past the image: loaded, not used
        const unsigned base = ((unsigned)(b * Hp + Y) * Wp + x) * Q + sub;
#pragma unroll
        for (int kx = 0; kx < 3; ++kx)
#pragma unroll
            for (int k = 0; k < QL; ++k) v[r][kx][k] = ld_quad<BF>(a.P, base + kx * Q + k * L);
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (y0 + r >= a.h) break;   // block-uniform
        float acc = 0.f;
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx)
#pragma unroll
                for (int k = 0; k < QL; ++k) acc += dot4(v[r + ky][kx][k], wr[ky * 3 + kx][k]);
#pragma unroll
        for (int o = L / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, L);
        if (sub == 0) a.disp[((unsigned)b * a.h + y0 + r) * a.w + x] = 1.f / (1.f + expf(-(acc + bias)));
    }
}

// Blocks walk padded rows; a thread owns channel quad q = tid % Q and pixels
// X = tid / Q + k·(256/Q) of the row.  Dynamic LDS: dz[3][Wp + 2] during the walk,
// then the per-wave partials [4 waves][min(Q,64)][37].
template <int Q, bool BF = false>
__global__ __launch_bounds__(kThreads) void head_bwd_kernel(HeadArgs a) {
    extern __shared__ float lds[];
    constexpr int TP = kThreads / Q;            // pixels per pass
    const int Wp = a.w + 2, Hp = a.h + 2;
    const int Ws = Wp + 2;                      // dz row stride: x + 2 for x in [-2, Wp)
    const int q = threadIdx.x % Q, p0 = threadIdx.x / Q;
    float4 wq[9];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) wq[tap] = wt_quad(a, tap, q);
    float4 dw[9];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) dw[tap] = make_float4(0.f, 0.f, 0.f, 0.f);
    float db = 0.f;
    const int rows = a.B * Hp;
    for (int r = blockIdx.x; r < rows; r += gridDim.x) {
        const int b = r / Hp, Y = r - b * Hp;
        __syncthreads();                        // previous row's dz reads are done
        for (int e = threadIdx.x; e < 3 * Ws; e += kThreads) {
            const int ky = e / Ws, x = e - ky * Ws - 2, y = Y - ky;
            float dz = 0.f;
            if (y >= 0 && y < a.h && x >= 0 && x < a.w) {
                const int o = (b * a.h + y) * a.w + x;
                const float d = a.disp[o];
                dz = a.gdisp[o] * d * (1.f - d);   // sigmoid backward from its output
            }
            lds[e] = dz;
        }
        __syncthreads();
        const int rowbase = r * Wp;
        for (int X = p0; X < Wp; X += TP) {
            const int i = (rowbase + X) * Q + q;
            const float4 p = ld_quad<BF>(a.P, i);
            float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const float dz = lds[ky * Ws + X + 2 - kx];
                    const int tap = ky * 3 + kx;
                    g.x += wq[tap].x * dz;
                    g.y += wq[tap].y * dz;
                    g.z += wq[tap].z * dz;
                    g.w += wq[tap].w * dz;
                    dw[tap].x += p.x * dz;
                    dw[tap].y += p.y * dz;
                    dw[tap].z += p.z * dz;
                    dw[tap].w += p.w * dz;
                }
            if (q == 0) db += lds[Ws + X + 1];      // centre tap: each output pixel once
            st_quad<BF>(a.gP, i, g);
        }
    }
    // lanes with equal q inside a wave: xor-shuffle over the lane bits above Q
    float v[37];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        v[tap * 4 + 0] = dw[tap].x;
        v[tap * 4 + 1] = dw[tap].y;
        v[tap * 4 + 2] = dw[tap].z;
        v[tap * 4 + 3] = dw[tap].w;
    }
    v[36] = db;
#pragma unroll
    for (int o = Q; o < 64; o <<= 1)           // Q divides 64 (C <= 256)
#pragma unroll
        for (int j = 0; j < 37; ++j) v[j] += __shfl_xor(v[j], o, 64);
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    __syncthreads();                             // dz reads done: reuse LDS
    if (lane < Q) {
        float* dst = lds + (wave * Q + lane) * 37;
#pragma unroll
        for (int j = 0; j < 37; ++j) dst[j] = v[j];
    }
    __syncthreads();
    const int n = 9 * a.C + 1;
    float* out = a.part + (size_t)blockIdx.x * n;
    constexpr int NW = kThreads / 64;
    for (int e = threadIdx.x; e < n; e += kThreads) {
        int off;                                 // db lives on quad 0
        if (e == n - 1) {
            off = 36;
        } else {
            const int tap = e / a.C, c = e - tap * a.C;
            off = (c >> 2) * 37 + tap * 4 + (c & 3);
        }
        float s = 0.f;
#pragma unroll
        for (int wv = 0; wv < NW; ++wv) s += lds[wv * Q * 37 + off];
        out[e] = s;
    }
}

// fixed-order sum of the block partials; element e = tap*C + c (or db)
__global__ __launch_bounds__(kThreads) void head_wgrad_kernel(HeadArgs a, int G) {
    const int n = 9 * a.C + 1;
    const int e = blockIdx.x;                  // one block per element
    float s = 0.f;
    for (int g = threadIdx.x; g < G; g += kThreads) s += a.part[(size_t)g * n + e];
    __shared__ float red[kThreads];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int half = kThreads / 2; half > 0; half >>= 1) {
        if ((int)threadIdx.x < half) red[threadIdx.x] += red[threadIdx.x + half];
        __syncthreads();
    }
    if (threadIdx.x != 0) return;
    if (e == n - 1) {
        a.gb[0] = red[0];
    } else {
        const int tap = e / a.C, c = e % a.C;
        a.gw[a.w_cl ? tap * a.C + c : c * 9 + tap] = red[0];
    }
}

size_t bwd_lds(int C, int w) {
    const size_t dz = sizeof(float) * 3 * (size_t)(w + 4);
    const size_t red = sizeof(float) * (kThreads / 64) * (C / 4) * 37;
    return dz > red ? dz : red;
}

bool valid(const md2_head_desc* d) {
    return d && d->batch >= 1 && d->height >= 1 && d->width >= 1 && d->channels >= 4 && d->channels % 4 == 0 &&
           d->channels <= kMaxC && (kThreads % (d->channels / 4)) == 0 &&
           (long long)d->batch * (d->height + 2) * (d->width + 2) * (d->channels / 4) < (1ll << 31) &&
           bwd_lds(d->channels, d->width) <= (size_t)kMaxLds;
}

HeadArgs args_of(const md2_head_desc* d) {
    HeadArgs a = {};
    a.B = d->batch;
    a.C = d->channels;
    a.h = d->height;
    a.w = d->width;
    a.w_cl = (d->flags & MD2_HEAD_WEIGHT_CL) ? 1 : 0;
    return a;
}

int bwd_grid(const HeadArgs& a) {
    const int rows = a.B * (a.h + 2);           // one padded row per block pass
    return rows < kBwdBlocks ? rows : kBwdBlocks;
}

}  // namespace

extern "C" {

size_t md2_disp_head_workspace_bytes(const md2_head_desc* d) {
    if (!valid(d)) return 0;
    const HeadArgs a = args_of(d);
    return sizeof(float) * (size_t)bwd_grid(a) * (9 * a.C + 1);
}

int md2_disp_head_fwd(const md2_head_desc* d, const float* padded, const float* weight, const float* bias,
                      float* disp, void* stream) {
    if (!valid(d) || !padded || !weight || !bias || !disp) return MD2_ERR_ARG;
    HeadArgs a = args_of(d);
    a.P = padded;
    a.wt = weight;
    a.bias = bias;
    a.disp = disp;
    const int Q = a.C / 4;
    const int L = Q < 16 ? Q : 16;
    const long long threads = (long long)a.B * a.h * a.w * L;
    const long long need = (threads + kThreads - 1) / kThreads;
    long long want = (need + 3) / 4;                                // each group walks >= 4 pixels
    want = want < 8 ? 8 : (want > kFwdBlocks ? kFwdBlocks : want);
    const int grid = (int)((want + 7) / 8 * 8);                     // whole XCD rounds
    static const bool rowwalk = [] {
        const char* e = getenv("MD2_HEAD_ROWWALK");
        return e && e[0] == '1';
    }();
    const bool bf = (d->flags & MD2_HEAD_BF16) != 0;   // bf16 P (ABI 23): the column walk only
    if (!rowwalk || bf) {
        const int QL = Q > 16 ? Q / 16 : 1, R = QL >= 4 ? 2 : 8 / QL, GPB = kThreads / L;
        const long long tiles = (long long)((a.w + GPB - 1) / GPB) * ((a.h + R - 1) / R) * a.B;
        void (*kc)(HeadArgs) = Q == 1    ? (bf ? head_fwd_col_kernel<1, 1, true> : head_fwd_col_kernel<1, 1>)
                               : Q == 2  ? (bf ? head_fwd_col_kernel<2, 1, true> : head_fwd_col_kernel<2, 1>)
                               : Q == 4  ? (bf ? head_fwd_col_kernel<4, 1, true> : head_fwd_col_kernel<4, 1>)
                               : Q == 8  ? (bf ? head_fwd_col_kernel<8, 1, true> : head_fwd_col_kernel<8, 1>)
                               : Q == 16 ? (bf ? head_fwd_col_kernel<16, 1, true> : head_fwd_col_kernel<16, 1>)
                               : Q == 32 ? (bf ? head_fwd_col_kernel<16, 2, true> : head_fwd_col_kernel<16, 2>)
                                         : (bf ? head_fwd_col_kernel<16, 4, true> : head_fwd_col_kernel<16, 4>);
        if (bf && tiles >= (1ll << 31)) return MD2_ERR_ARG;
        if (tiles < (1ll << 31)) {
            hipLaunchKernelGGL(kc, dim3((unsigned)tiles), dim3(kThreads), 0, (hipStream_t)stream, a);
            return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
        }
    }
    void (*k)(HeadArgs) = Q == 1    ? head_fwd_kernel<1, 1>
                          : Q == 2  ? head_fwd_kernel<2, 1>
                          : Q == 4  ? head_fwd_kernel<4, 1>
                          : Q == 8  ? head_fwd_kernel<8, 1>
                          : Q == 16 ? head_fwd_kernel<16, 1>
                          : Q == 32 ? head_fwd_kernel<16, 2>
                                    : head_fwd_kernel<16, 4>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

int md2_disp_head_bwd(const md2_head_desc* d, const float* padded, const float* weight, const float* disp,
                      const float* grad_disp, float* grad_padded, float* grad_weight, float* grad_bias,
                      void* workspace, void* stream) {
    if (!valid(d) || !padded || !weight || !disp || !grad_disp || !grad_padded || !grad_weight || !grad_bias ||
        !workspace)
        return MD2_ERR_ARG;
    HeadArgs a = args_of(d);
    a.P = padded;
    a.wt = weight;
    a.disp = const_cast<float*>(disp);
    a.gdisp = grad_disp;
    a.gP = grad_padded;
    a.part = (float*)workspace;
    a.gw = grad_weight;
    a.gb = grad_bias;
    const int G = bwd_grid(a);
    const int Q = a.C / 4;
    const bool bf = (d->flags & MD2_HEAD_BF16) != 0;
    void (*k)(HeadArgs) = Q == 1    ? (bf ? head_bwd_kernel<1, true> : head_bwd_kernel<1>)
                          : Q == 2  ? (bf ? head_bwd_kernel<2, true> : head_bwd_kernel<2>)
                          : Q == 4  ? (bf ? head_bwd_kernel<4, true> : head_bwd_kernel<4>)
                          : Q == 8  ? (bf ? head_bwd_kernel<8, true> : head_bwd_kernel<8>)
                          : Q == 16 ? (bf ? head_bwd_kernel<16, true> : head_bwd_kernel<16>)
                          : Q == 32 ? (bf ? head_bwd_kernel<32, true> : head_bwd_kernel<32>)
                                    : (bf ? head_bwd_kernel<64, true> : head_bwd_kernel<64>);
    hipLaunchKernelGGL(k, dim3(G), dim3(kThreads), bwd_lds(a.C, a.w), (hipStream_t)stream, a);
    hipLaunchKernelGGL(head_wgrad_kernel, dim3(9 * a.C + 1), dim3(kThreads), 0, (hipStream_t)stream, a, G);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

}  // extern "C"
