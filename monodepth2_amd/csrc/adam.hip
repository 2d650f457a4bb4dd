// adam.hip — the training step's Adam update (torch.optim.Adam, trainer.py:102-104,
// 209) in one launch per 256 parameters (one for ResNet-18's three networks), gfx950.
//
// torch's fused Adam packs the tensor pointers into kernel arguments and splits the
// ~200 parameters of the three networks over five launches at ~2.9 TB/s.  Here a
// device table of fixed-size chunks (param, exp_avg, exp_avg_sq, length) is built
// once — those buffers never move — and the gradients, which autograd re-allocates
// every step, come as 256 base pointers in the kernel arguments; one block per
// chunk streams the four arrays with float4 loads.  Per element, in fp32 as torch's
// fused kernel:
//   m = b1*m + (1-b1)*g;  v = b2*v + (1-b2)*g*g
//   p -= (lr/bc1) * m / (sqrt(v)/sqrt(bc2) + eps)
// (no weight decay, amsgrad or maximize: the reference's optimizer.)

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "md2hot.h"

namespace {

constexpr int kThreads = 256;

// c1 = 1 - beta1, c2 = 1 - beta2, formed in double on the host as torch does
__device__ __forceinline__ void adam1(float& p, float g, float& m, float& v, float b1, float b2, float c1, float c2,
                                      float step_size, float bc2_sqrt, float eps) {
    m = b1 * m + c1 * g;
    v = b2 * v + c2 * g * g;
    p -= step_size * m / (sqrtf(v) / bc2_sqrt + eps);
}

// the gradient base pointers of up to kMaxParams parameters, as a kernel argument:
// gradients are re-allocated by autograd every step, parameters and moments are not
constexpr int kMaxParams = 256;
struct GradPtrs {
    const float* g[kMaxParams];
};

// Capturable form (hipGraph replays): the step counter and lr live on the device.  One
// thread advances the step and forms the bias corrections in double (as the host path
// does with the Python doubles), written as the two fp32 factors the update uses.
__global__ void adam_hyper_kernel(float* __restrict__ step, const double* __restrict__ lr, double b1, double b2,
                                  float* __restrict__ hyper) {
    if (threadIdx.x != 0) return;
    const float s = *step + 1.0f;
    *step = s;
    const double bc1 = 1.0 - pow(b1, (double)s);
    const double bc2 = 1.0 - pow(b2, (double)s);
    hyper[0] = (float)(*lr / bc1);
    hyper[1] = (float)sqrt(bc2);
}

template <bool DEV>
__global__ __launch_bounds__(kThreads) void adam_kernel(const md2_adam_chunk* __restrict__ table, int first_param,
                                                        GradPtrs grads, float b1, float b2, float c1, float c2,
                                                        float step_size, float bc2_sqrt, float eps,
                                                        const float* __restrict__ hyper) {
    if (DEV) {
        step_size = hyper[0];
        bc2_sqrt = hyper[1];
    }
    const md2_adam_chunk c = table[blockIdx.x];
    const long long n = c.n;
    const float* gp = grads.g[c.param - first_param] + c.off;
    const bool vec = ((((uintptr_t)c.p | (uintptr_t)gp | (uintptr_t)c.m | (uintptr_t)c.v) & 15) == 0);
    const long long n4 = vec ? n / 4 : 0;
    float4* p4 = (float4*)c.p;
    const float4* g4 = (const float4*)gp;
    float4* m4 = (float4*)c.m;
    float4* v4 = (float4*)c.v;
    for (long long i = threadIdx.x; i < n4; i += kThreads) {
        float4 p = p4[i], m = m4[i], v = v4[i];
        const float4 g = g4[i];
        adam1(p.x, g.x, m.x, v.x, b1, b2, c1, c2, step_size, bc2_sqrt, eps);
        adam1(p.y, g.y, m.y, v.y, b1, b2, c1, c2, step_size, bc2_sqrt, eps);
        adam1(p.z, g.z, m.z, v.z, b1, b2, c1, c2, step_size, bc2_sqrt, eps);
        adam1(p.w, g.w, m.w, v.w, b1, b2, c1, c2, step_size, bc2_sqrt, eps);
        p4[i] = p;
        m4[i] = m;
        v4[i] = v;
    }
    for (long long i = 4 * n4 + threadIdx.x; i < n; i += kThreads)
        adam1(c.p[i], gp[i], c.m[i], c.v[i], b1, b2, c1, c2, step_size, bc2_sqrt, eps);
}

}  // namespace

extern "C" {

int md2_adam_step(const md2_adam_chunk* table, const int* chunk_start, int nparams, const float* const* grads,
                  double lr, double beta1, double beta2, double eps, int step, void* stream) {
    if (!table || !chunk_start || !grads || nparams < 0 || step < 1 || !(lr >= 0.0) || !(eps > 0.0))
        return MD2_ERR_ARG;
    // the hyper-parameters arrive as the Python doubles torch uses: 1 - beta and the
    // bias corrections are formed in double before the fp32 kernel sees them
    const double bc1 = 1.0 - pow(beta1, (double)step);
    const double bc2 = 1.0 - pow(beta2, (double)step);
    for (int k0 = 0; k0 < nparams; k0 += kMaxParams) {   // one launch per 256 parameters
        const int k1 = k0 + kMaxParams < nparams ? k0 + kMaxParams : nparams;
        GradPtrs gp = {};
        for (int k = k0; k < k1; ++k) gp.g[k - k0] = grads[k];
        const int c0 = chunk_start[k0], c1 = chunk_start[k1];
        if (c1 <= c0) continue;
        hipLaunchKernelGGL(adam_kernel<false>, dim3(c1 - c0), dim3(kThreads), 0, (hipStream_t)stream, table + c0, k0,
                           gp, (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2),
                           (float)(lr / bc1), (float)sqrt(bc2), (float)eps, (const float*)nullptr);
    }
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

int md2_adam_hyper(const double* lr, double beta1, double beta2, float* step, float* hyper, void* stream) {
    if (!lr || !step || !hyper) return MD2_ERR_ARG;
    hipLaunchKernelGGL(adam_hyper_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, step, lr, beta1, beta2, hyper);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

int md2_adam_apply_dev(const md2_adam_chunk* table, const int* chunk_start, int k_begin, int k_end,
                       const float* const* grads, double beta1, double beta2, double eps, const float* hyper,
                       void* stream) {
    if (!table || !chunk_start || !grads || k_begin < 0 || k_end < k_begin || !hyper || !(eps > 0.0))
        return MD2_ERR_ARG;
    for (int k0 = k_begin; k0 < k_end; k0 += kMaxParams) {
        const int k1 = k0 + kMaxParams < k_end ? k0 + kMaxParams : k_end;
        GradPtrs gp = {};
        for (int k = k0; k < k1; ++k) gp.g[k - k0] = grads[k];
        const int c0 = chunk_start[k0], c1 = chunk_start[k1];
        if (c1 <= c0) continue;
        hipLaunchKernelGGL(adam_kernel<true>, dim3(c1 - c0), dim3(kThreads), 0, (hipStream_t)stream, table + c0, k0,
                           gp, (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2), 0.f, 1.f,
                           (float)eps, hyper);
    }
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

int md2_adam_step_dev(const md2_adam_chunk* table, const int* chunk_start, int nparams, const float* const* grads,
                      const double* lr, double beta1, double beta2, double eps, float* step, float* hyper,
                      void* stream) {
    if (!table || !chunk_start || !grads || nparams < 0 || !lr || !step || !hyper || !(eps > 0.0))
        return MD2_ERR_ARG;
    const int rc = md2_adam_hyper(lr, beta1, beta2, step, hyper, stream);
    if (rc != MD2_OK) return rc;
    return md2_adam_apply_dev(table, chunk_start, 0, nparams, grads, beta1, beta2, eps, hyper, stream);
}

}  // extern "C"
