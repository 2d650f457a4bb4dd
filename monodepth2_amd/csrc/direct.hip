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

#include <stdint.h>

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
    if (ci == 16 && co == 16)
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

}  // extern "C"
