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
//     float4 quads (L = min(C/4, 16)), 9 taps each, shuffle-reduced, bias + sigmoid
//     fused; writes disp (B,1,h,w).
//   * backward: one pass over the padded pixels (Y, X): dz = dD·D·(1-D) of the up to
//     9 output pixels that read (Y, X) gives dP[Y,X,:] = Σ_taps w[tap,:]·dz (a 3x3
//     transposed conv, written once, float4) and, from the same loads,
//     dW[tap,:] += P[Y,X,:]·dz[tap] and db += dz — per-block partials, summed by a
//     second launch in a fixed order (deterministic, no atomics).
// Weights are read in the parameter's own memory format (channels_last: [tap][c],
// contiguous: [c][tap]) and dW is written back in that format.

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "md2hot.h"

namespace {

constexpr int kThreads = 256;
constexpr int kMaxC = 256;
constexpr int kBwdBlocks = 1024;

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

__device__ __forceinline__ float wt_at(const HeadArgs& a, int tap, int c) {
    return a.w_cl ? a.wt[tap * a.C + c] : a.wt[c * 9 + tap];
}

// L lanes per pixel, Q = C/4 quads, QL = Q/L quads per lane
template <int L>
__global__ __launch_bounds__(kThreads) void head_fwd_kernel(HeadArgs a) {
    const int Q = a.C >> 2, QL = Q / L;
    const int Wp = a.w + 2, Hp = a.h + 2;
    const int sub = threadIdx.x % L;
    const long long npix = (long long)a.B * a.h * a.w;
    const long long pix = ((long long)blockIdx.x * kThreads + threadIdx.x) / L;
    if (pix >= npix) return;   // whole L-lane groups exit together (L divides 64)
    const int x = (int)(pix % a.w);
    const long long t = pix / a.w;
    const int y = (int)(t % a.h), b = (int)(t / a.h);
    const float4* P4 = reinterpret_cast<const float4*>(a.P);
    float acc = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
        for (int kx = 0; kx < 3; ++kx) {
            const long long base = (((long long)b * Hp + (y + ky)) * Wp + (x + kx)) * Q;
            for (int k = 0; k < QL; ++k) {
                const int q = sub + k * L;
                const float4 v = P4[base + q];
                const int tap = ky * 3 + kx, c = q * 4;
                acc += v.x * wt_at(a, tap, c) + v.y * wt_at(a, tap, c + 1) + v.z * wt_at(a, tap, c + 2) +
                       v.w * wt_at(a, tap, c + 3);
            }
        }
#pragma unroll
    for (int o = L / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o, L);
    if (sub == 0) {
        const float z = acc + a.bias[0];
        a.disp[pix] = 1.f / (1.f + expf(-z));
    }
}

// one thread per (padded pixel, channel quad); grid-stride over all of them.  Block
// partials: [9 taps x C channels] of dW, then db.
__global__ __launch_bounds__(kThreads) void head_bwd_kernel(HeadArgs a) {
    const int Q = a.C >> 2;
    const int Wp = a.w + 2, Hp = a.h + 2;
    const int q = threadIdx.x % Q;              // Q divides kThreads: a thread keeps its quad
    const long long total = (long long)a.B * Hp * Wp * Q;
    const float4* P4 = reinterpret_cast<const float4*>(a.P);
    float4* G4 = reinterpret_cast<float4*>(a.gP);
    float wq[9][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) wq[tap][j] = wt_at(a, tap, q * 4 + j);
    float dw[9][4];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) dw[tap][j] = 0.f;
    float db = 0.f;
    for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < total;
         i += (long long)gridDim.x * kThreads) {
        const long long pp = i / Q;             // padded pixel
        const int X = (int)(pp % Wp);
        const long long t = pp / Wp;
        const int Y = (int)(t % Hp), b = (int)(t / Hp);
        const float4 p = P4[i];
        float4 g = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const int y = Y - ky;
            if (y < 0 || y >= a.h) continue;
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const int x = X - kx;
                if (x < 0 || x >= a.w) continue;
                const long long o = ((long long)b * a.h + y) * a.w + x;
                const float d = a.disp[o];
                const float dz = a.gdisp[o] * d * (1.f - d);   // sigmoid backward from its output
                const int tap = ky * 3 + kx;
                g.x += wq[tap][0] * dz;
                g.y += wq[tap][1] * dz;
                g.z += wq[tap][2] * dz;
                g.w += wq[tap][3] * dz;
                dw[tap][0] += p.x * dz;
                dw[tap][1] += p.y * dz;
                dw[tap][2] += p.z * dz;
                dw[tap][3] += p.w * dz;
                if (tap == 4 && q == 0) db += dz;   // each output pixel once: its centre tap
            }
        }
        G4[i] = g;
    }
    // block reduction of the per-thread partials: threads with equal q share channels
    __shared__ float red[kThreads][37];
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[threadIdx.x][tap * 4 + j] = dw[tap][j];
    red[threadIdx.x][36] = db;
    __syncthreads();
    const int groups = kThreads / Q;            // threads per quad in this block
    const int n = 9 * a.C + 1;
    float* out = a.part + (size_t)blockIdx.x * n;
    for (int e = threadIdx.x; e < n; e += kThreads) {
        float s = 0.f;
        if (e == n - 1) {
            for (int gi = 0; gi < groups; ++gi) s += red[gi * Q][36];   // q == 0 threads
        } else {
            const int tap = e / a.C, c = e % a.C, qq = c >> 2, j = c & 3;
            for (int gi = 0; gi < groups; ++gi) s += red[gi * Q + qq][tap * 4 + j];
        }
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

bool valid(const md2_head_desc* d) {
    return d && d->batch >= 1 && d->height >= 1 && d->width >= 1 && d->channels >= 4 && d->channels % 4 == 0 &&
           d->channels <= kMaxC && (kThreads % (d->channels / 4)) == 0 &&
           (long long)d->batch * (d->height + 2) * (d->width + 2) * (d->channels / 4) < (1ll << 31);
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
    const long long total = (long long)a.B * (a.h + 2) * (a.w + 2) * (a.C / 4);
    const long long g = (total + kThreads - 1) / kThreads;
    return (int)(g < kBwdBlocks ? g : kBwdBlocks);
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
    const int grid = (int)((threads + kThreads - 1) / kThreads);
    void (*k)(HeadArgs) = L == 1    ? head_fwd_kernel<1>
                          : L == 2  ? head_fwd_kernel<2>
                          : L == 4  ? head_fwd_kernel<4>
                          : L == 8  ? head_fwd_kernel<8>
                                    : head_fwd_kernel<16>;
    if (L != 1 && L != 2 && L != 4 && L != 8 && L != 16) return MD2_ERR_ARG;
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
    hipLaunchKernelGGL(head_bwd_kernel, dim3(G), dim3(kThreads), 0, (hipStream_t)stream, a);
    hipLaunchKernelGGL(head_wgrad_kernel, dim3(9 * a.C + 1), dim3(kThreads), 0, (hipStream_t)stream, a, G);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

}  // extern "C"
