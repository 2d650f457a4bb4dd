// bias_act.hip — conv bias + ReLU epilogue for NHWC activations (the PoseDecoder's
// convolutions, networks/pose_decoder.py:43-54: relu(conv(x) + b), and the last conv's
// bare bias) on gfx950.
//
// MIOpen's convolution adds its bias in a separate pass; autograd then runs ReLU
// (clamp), its backward (threshold), a zero-fill and a reduction for the bias
// gradient — five small launches per layer on the pose stream, which is the tail of
// the training step.  Here: forward y = relu(x + b) in one pass; backward one launch
// per layer: g' = g·[y > 0] (written when the ReLU is on) streamed row-coalesced, with
// the bias gradient as per-block partial rows summed in block order by a tiny second
// launch (deterministic, no atomics).
// Layout: x, y, g, g' (pixels, C) — a channels_last tensor; C a multiple of 4.

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

constexpr int kThreads = 256;
constexpr int kBwdThreads = 1024;
constexpr unsigned kRowBlocks = 256;  // partial rows of the coalesced backward (<= kThreads)   // the pose decoder's maps are ~3k pixels: ~3 per thread

template <bool RELU>
__global__ __launch_bounds__(kThreads) void bias_act_fwd_kernel(const float4* __restrict__ x,
                                                                const float4* __restrict__ b, float4* __restrict__ y,
                                                                unsigned n4, unsigned Q) {
    for (unsigned i = blockIdx.x * kThreads + threadIdx.x; i < n4; i += gridDim.x * kThreads) {
        const float4 v = x[i], bb = b[i % Q];
        float4 o = make_float4(v.x + bb.x, v.y + bb.y, v.z + bb.z, v.w + bb.w);
        if (RELU) {
            o.x = fmaxf(o.x, 0.f); o.y = fmaxf(o.y, 0.f); o.z = fmaxf(o.z, 0.f); o.w = fmaxf(o.w, 0.f);
        }
        y[i] = o;
    }
}

// Coalesced form (C/4 dividing 256): a block iteration covers 256/Q whole pixel rows,
// thread t keeps quad t % Q; g' written as it streams, the block's per-quad sums
// folded in LDS in a fixed tree into one partial row; bias_act_final_kernel sums the
// partial rows in block order.
template <bool RELU>
__global__ __launch_bounds__(kThreads) void bias_act_bwd_rows_kernel(const float4* __restrict__ y,
                                                                     const float4* __restrict__ g,
                                                                     float4* __restrict__ gx, float4* __restrict__ part,
                                                                     unsigned P, unsigned Q) {
    const unsigned q = threadIdx.x % Q, pl = threadIdx.x / Q, ppb = kThreads / Q;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    for (unsigned p = blockIdx.x * ppb + pl; p < P; p += gridDim.x * ppb) {
        const unsigned i = p * Q + q;
        float4 gv = g[i];
        if (RELU) {
            const float4 yv = y[i];
            gv.x = yv.x > 0.f ? gv.x : 0.f; gv.y = yv.y > 0.f ? gv.y : 0.f;
            gv.z = yv.z > 0.f ? gv.z : 0.f; gv.w = yv.w > 0.f ? gv.w : 0.f;
            gx[i] = gv;
        }
        s.x += gv.x; s.y += gv.y; s.z += gv.z; s.w += gv.w;
    }
    __shared__ float4 red[kThreads];
    red[threadIdx.x] = s;
    __syncthreads();
    for (unsigned half = ppb / 2; half > 0; half >>= 1) {   // ppb a power of two
        if (pl < half) {
            const float4 o = red[threadIdx.x + half * Q];
            float4& m = red[threadIdx.x];
            m.x += o.x; m.y += o.y; m.z += o.z; m.w += o.w;
        }
        __syncthreads();
    }
    if (pl == 0) part[(size_t)blockIdx.x * Q + q] = red[threadIdx.x];
}

// one block per channel quad: thread t takes partial row t (G <= 256), fixed LDS tree
__global__ __launch_bounds__(kThreads) void bias_act_final_kernel(const float4* __restrict__ part,
                                                                  float4* __restrict__ gb, unsigned G, unsigned Q) {
    const unsigned q = blockIdx.x;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (threadIdx.x < G) s = part[(size_t)threadIdx.x * Q + q];
    __shared__ float4 red[kThreads];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int half = kThreads / 2; half > 0; half >>= 1) {
        if ((int)threadIdx.x < half) {
            const float4 o = red[threadIdx.x + half];
            float4& m = red[threadIdx.x];
            m.x += o.x; m.y += o.y; m.z += o.z; m.w += o.w;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) gb[q] = red[0];
}

// General C (C/4 not dividing 256, e.g. the 12-channel pose output): one block per
// channel quad q, threads walk pixels p = tid, tid + 1024, ...
template <bool RELU>
__global__ __launch_bounds__(kBwdThreads) void bias_act_bwd_kernel(const float4* __restrict__ y,
                                                                const float4* __restrict__ g, float4* __restrict__ gx,
                                                                float4* __restrict__ gb, unsigned P, unsigned Q) {
    const unsigned q = blockIdx.x;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll 4
    for (unsigned p = threadIdx.x; p < P; p += kBwdThreads) {
        const unsigned i = p * Q + q;
        float4 gv = g[i];
        if (RELU) {
            const float4 yv = y[i];
            gv.x = yv.x > 0.f ? gv.x : 0.f; gv.y = yv.y > 0.f ? gv.y : 0.f;
            gv.z = yv.z > 0.f ? gv.z : 0.f; gv.w = yv.w > 0.f ? gv.w : 0.f;
            gx[i] = gv;
        }
        s.x += gv.x; s.y += gv.y; s.z += gv.z; s.w += gv.w;
    }
    __shared__ float4 red[kBwdThreads];
    red[threadIdx.x] = s;
    __syncthreads();
    for (int half = kBwdThreads / 2; half > 0; half >>= 1) {
        if ((int)threadIdx.x < half) {
            const float4 o = red[threadIdx.x + half];
            float4& m = red[threadIdx.x];
            m.x += o.x; m.y += o.y; m.z += o.z; m.w += o.w;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) gb[q] = red[0];
}

bool valid(const md2_bias_act_desc* d) {
    return d && d->pixels >= 1 && d->channels >= 4 && d->channels % 4 == 0 &&
           (long long)d->pixels * (d->channels / 4) < (1ll << 31);
}

}  // namespace

extern "C" {

int md2_bias_act_fwd(const md2_bias_act_desc* d, const float* x, const float* bias, float* y, void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "bias_act_fwd: channels a multiple of 4");
    if (!x || !bias || !y) return md2_report_error(MD2_ERR_ARG, "bias_act_fwd: NULL operand");
    const unsigned Q = d->channels / 4, n4 = (unsigned)d->pixels * Q;
    const unsigned need = (n4 + kThreads - 1) / kThreads;
    const unsigned grid = need < 4096 ? need : 4096;
    auto k = (d->flags & MD2_BIAS_ACT_RELU) ? bias_act_fwd_kernel<true> : bias_act_fwd_kernel<false>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(kThreads), 0, (hipStream_t)stream, (const float4*)x, (const float4*)bias,
                       (float4*)y, n4, Q);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

size_t md2_bias_act_workspace_bytes(const md2_bias_act_desc* d) {
    if (!valid(d)) return 0;
    return sizeof(float) * 4 * (size_t)kRowBlocks * (d->channels / 4);
}

int md2_bias_act_bwd(const md2_bias_act_desc* d, const float* y, const float* grad_y, float* grad_x,
                     float* grad_bias, void* workspace, void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "bias_act_bwd: channels a multiple of 4");
    const bool relu = d->flags & MD2_BIAS_ACT_RELU;
    if (!grad_y || !grad_bias || (relu && (!y || !grad_x)))
        return md2_report_error(MD2_ERR_ARG, "bias_act_bwd: NULL operand");
    const unsigned Q = d->channels / 4, P = (unsigned)d->pixels;
    const hipStream_t st = (hipStream_t)stream;
    if (kThreads % Q == 0 && workspace) {
        const unsigned ppb = kThreads / Q;
        const unsigned rows = (P + ppb - 1) / ppb;
        const unsigned want = (rows + 3) / 4;                         // ~4 pixel rows per thread
        const unsigned G = want < 1 ? 1 : (want > kRowBlocks ? kRowBlocks : want);
        auto k = relu ? bias_act_bwd_rows_kernel<true> : bias_act_bwd_rows_kernel<false>;
        hipLaunchKernelGGL(k, dim3(G), dim3(kThreads), 0, st, (const float4*)y, (const float4*)grad_y,
                           (float4*)grad_x, (float4*)workspace, P, Q);
        hipLaunchKernelGGL(bias_act_final_kernel, dim3(Q), dim3(kThreads), 0, st, (const float4*)workspace,
                           (float4*)grad_bias, G, Q);
    } else {
        auto k = relu ? bias_act_bwd_kernel<true> : bias_act_bwd_kernel<false>;
        hipLaunchKernelGGL(k, dim3(Q), dim3(kBwdThreads), 0, st, (const float4*)y, (const float4*)grad_y,
                           (float4*)grad_x, (float4*)grad_bias, P, Q);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
