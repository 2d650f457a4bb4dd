// glue.hip — the encoders' input preparation for gfx950 in one pass.
//
// Reference: ResnetEncoder.forward normalises its input, x = (input_image - 0.45) /
// 0.225 (networks/resnet_encoder.py:93); the pose encoder's input is the channel
// concatenation of a frame pair (trainer.py:280-290); the NHWC convolutions want it
// channels_last.  Eagerly that is cat + sub + div + a layout copy — four HBM passes
// over a full-resolution batch.  Here one thread per output pixel reads the 3-channel
// NCHW planes of every frame slot and writes the normalised, interleaved pixel once
// (the fp32 operations torch performs for (x - mean) / std on the GPU: the scalar
// division is a multiplication by the fp32 reciprocal 1.f / std).

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

constexpr int kThreads = 256;
constexpr int kMaxSrc = 8;   // groups * slots

struct InputArgs {
    const float* src[kMaxSrc];   // [group * slots + slot]: (B, 3, H, W) NCHW
    float* out;                  // (groups * B, H, W, 3 * slots)
    int B, HW, slots, n;         // n = groups * B * HW
    float mean, inv_std;
};

__global__ __launch_bounds__(kThreads) void encoder_input_kernel(InputArgs a) {
    const int i = blockIdx.x * kThreads + threadIdx.x;   // (group * B + b) * HW + p
    if (i >= a.n) return;
    const int nb = i / a.HW, p = i - nb * a.HW;
    const int grp = nb / a.B, b = nb - grp * a.B;
    float* o = a.out + (size_t)i * 3 * a.slots;
    for (int k = 0; k < a.slots; ++k) {
        const float* s = a.src[grp * a.slots + k] + (size_t)b * 3 * a.HW + p;
#pragma unroll
        for (int c = 0; c < 3; ++c) o[3 * k + c] = (s[(size_t)c * a.HW] - a.mean) * a.inv_std;
    }
}

// Four pixels per thread (HW % 4 == 0): one float4 load per source channel, the
// 4 x 3·slots output floats written as 3·slots float4 stores (16-B aligned because
// the thread's first pixel is a multiple of 4).  Same arithmetic as above.
template <int SLOTS>
__global__ __launch_bounds__(kThreads) void encoder_input_v4_kernel(InputArgs a) {
    constexpr int OC = 3 * SLOTS;
    const int i4 = blockIdx.x * kThreads + threadIdx.x;   // quad of pixels
    if (i4 * 4 >= a.n) return;
    const int i = i4 * 4;
    const int nb = i / a.HW, p = i - nb * a.HW;
    const int grp = nb / a.B, b = nb - grp * a.B;
    float v[4][OC];
#pragma unroll
    for (int k = 0; k < SLOTS; ++k) {
        const float* s = a.src[grp * SLOTS + k] + (size_t)b * 3 * a.HW + p;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float4 x = *reinterpret_cast<const float4*>(s + (size_t)c * a.HW);
            v[0][3 * k + c] = (x.x - a.mean) * a.inv_std;
            v[1][3 * k + c] = (x.y - a.mean) * a.inv_std;
            v[2][3 * k + c] = (x.z - a.mean) * a.inv_std;
            v[3][3 * k + c] = (x.w - a.mean) * a.inv_std;
        }
    }
    float4* o = reinterpret_cast<float4*>(a.out + (size_t)i * OC);
#pragma unroll
    for (int q = 0; q < OC; ++q) {   // the 4·OC floats in pixel-major order, four at a time
        float4 w;
        w.x = v[(4 * q + 0) / OC][(4 * q + 0) % OC];
        w.y = v[(4 * q + 1) / OC][(4 * q + 1) % OC];
        w.z = v[(4 * q + 2) / OC][(4 * q + 2) % OC];
        w.w = v[(4 * q + 3) / OC][(4 * q + 3) % OC];
        o[q] = w;
    }
}

}  // namespace

#ifndef MD2_BUILD_ID
#define MD2_BUILD_ID "unset"
#endif

extern "C" {

// the source hash monodepth2_amd/build.py bakes in (see md2hot.h), stored behind a
// marker so that build.py can read it from the file without loading the library
static const char kBuildIdTagged[] = "md2-build-id:" MD2_BUILD_ID;
const char* md2_build_id(void) { return kBuildIdTagged + 13; }

int md2_encoder_input(int groups, int batch, int slots, int height, int width, const float* const* src, float mean,
                      float std_, float* out, void* stream) {
    if (groups < 1 || batch < 1 || slots < 1 || groups * slots > kMaxSrc || height < 1 || width < 1 || !src ||
        !out || !(std_ != 0.f))
        return md2_report_error(MD2_ERR_ARG, "encoder_input: bad shape, more than 8 sources, or NULL operand");
    const long long n = (long long)groups * batch * height * width;
    if (n * 3 * slots >= (1ll << 31)) return md2_report_error(MD2_ERR_ARG, "encoder_input: batch too large");
    InputArgs a = {};
    for (int k = 0; k < groups * slots; ++k) {
        if (!src[k]) return md2_report_error(MD2_ERR_ARG, "encoder_input: NULL source");
        a.src[k] = src[k];
    }
    a.out = out;
    a.B = batch;
    a.HW = height * width;
    a.slots = slots;
    a.n = (int)n;
    a.mean = mean;
    a.inv_std = 1.f / std_;
    bool v4 = a.HW % 4 == 0 && (slots == 1 || slots == 2) && ((uintptr_t)out & 15) == 0;
    for (int k = 0; k < groups * slots; ++k) v4 = v4 && ((uintptr_t)src[k] & 15) == 0;
    if (v4) {
        const long long n4 = n / 4;
        hipLaunchKernelGGL(slots == 1 ? encoder_input_v4_kernel<1> : encoder_input_v4_kernel<2>,
                           dim3((unsigned)((n4 + kThreads - 1) / kThreads)), dim3(kThreads), 0, (hipStream_t)stream, a);
    } else {
        hipLaunchKernelGGL(encoder_input_kernel, dim3((unsigned)((n + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                           (hipStream_t)stream, a);
    }
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
