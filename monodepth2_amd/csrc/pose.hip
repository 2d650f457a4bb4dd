// pose.hip — fused pose producer for gfx950.
//
// transformation_from_parameters (layers.py:28-45) with rot_from_axisangle
// (layers.py:64-103) and get_translation_matrix (layers.py:48-61) is ~55 tiny
// eager launches per source frame forward and as many backward; here all frames of
// a step are one launch each way, one thread per (frame, image).
//
// Forward, per (f, b) with v = axisangle, t = translation:
//   angle = |v|, axis = v / (angle + 1e-7), ca = cos angle, sa = sin angle, C = 1 - ca
//   R = Rodrigues(axis, ca, sa)   (the reference's exact expression order)
//   invert ? M = [R^T | -R^T t] : M = [R | t],  last row (0, 0, 0, 1)
// Backward: the adjoint of the same expressions (torch.norm's gradient is 0 at 0).

#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include "md2hot.h"

namespace {

struct Rot {
    float x, y, z, ca, sa, C;
    float R[3][3];
};

__device__ __forceinline__ void rodrigues(float x, float y, float z, float ca, float sa, float (&R)[3][3]) {
    const float C = 1.f - ca;
    const float xs = x * sa, ys = y * sa, zs = z * sa;
    const float xC = x * C, yC = y * C, zC = z * C;
    const float xyC = x * yC, yzC = y * zC, zxC = z * xC;
    R[0][0] = x * xC + ca;
    R[0][1] = xyC - zs;
    R[0][2] = zxC + ys;
    R[1][0] = xyC + zs;
    R[1][1] = y * yC + ca;
    R[1][2] = yzC - xs;
    R[2][0] = zxC - ys;
    R[2][1] = yzC + xs;
    R[2][2] = z * zC + ca;
}

__global__ void pose_fwd_kernel(int n, int B, uint32_t invert_mask, const float* __restrict__ aa,
                                const float* __restrict__ tr, float* __restrict__ T) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int f = i / B;
    const bool inv = (invert_mask >> f) & 1u;
    const float vx = aa[3 * i], vy = aa[3 * i + 1], vz = aa[3 * i + 2];
    const float angle = sqrtf(vx * vx + vy * vy + vz * vz);
    const float den = angle + 1e-7f;
    const float x = vx / den, y = vy / den, z = vz / den;
    float R[3][3];
    rodrigues(x, y, z, cosf(angle), sinf(angle), R);
    float t[3] = {tr[3 * i], tr[3 * i + 1], tr[3 * i + 2]};
    float* M = T + 16 * (size_t)i;
    if (inv) {
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) M[4 * r + c] = R[c][r];
            M[4 * r + 3] = R[0][r] * -t[0] + R[1][r] * -t[1] + R[2][r] * -t[2];
        }
    } else {
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) M[4 * r + c] = R[r][c];
            M[4 * r + 3] = t[r];
        }
    }
    M[12] = 0.f;
    M[13] = 0.f;
    M[14] = 0.f;
    M[15] = 1.f;
}

__global__ void pose_bwd_kernel(int n, int B, uint32_t invert_mask, const float* __restrict__ aa,
                                const float* __restrict__ tr, const float* __restrict__ dT,
                                float* __restrict__ daa, float* __restrict__ dtr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int f = i / B;
    const bool inv = (invert_mask >> f) & 1u;
    const float vx = aa[3 * i], vy = aa[3 * i + 1], vz = aa[3 * i + 2];
    const float angle = sqrtf(vx * vx + vy * vy + vz * vz);
    const float den = angle + 1e-7f;
    const float x = vx / den, y = vy / den, z = vz / den;
    const float ca = cosf(angle), sa = sinf(angle), C = 1.f - ca;
    float R[3][3];
    rodrigues(x, y, z, ca, sa, R);
    const float* G = dT + 16 * (size_t)i;
    const float t[3] = {tr[3 * i], tr[3 * i + 1], tr[3 * i + 2]};
    float dR[3][3], dt[3];
    if (inv) {
        // M[r][c] = R[c][r] (c<3), M[r][3] = -sum_k R[k][r] t[k]
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) dR[c][r] = G[4 * r + c] - G[4 * r + 3] * t[c];
        for (int k = 0; k < 3; ++k) dt[k] = -(R[k][0] * G[3] + R[k][1] * G[7] + R[k][2] * G[11]);
    } else {
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) dR[r][c] = G[4 * r + c];
            dt[r] = G[4 * r + 3];
        }
    }
    // adjoint of rodrigues()
    const float xC = x * C, yC = y * C, zC = z * C;
    float dx = 0.f, dy = 0.f, dz = 0.f, dca = 0.f, dsa = 0.f, dC = 0.f;
    // R00 = x*xC + ca ; R11 = y*yC + ca ; R22 = z*zC + ca
    dx += dR[0][0] * 2.f * xC;
    dC += dR[0][0] * x * x;
    dy += dR[1][1] * 2.f * yC;
    dC += dR[1][1] * y * y;
    dz += dR[2][2] * 2.f * zC;
    dC += dR[2][2] * z * z;
    dca += dR[0][0] + dR[1][1] + dR[2][2];
    // xyC = x*y*C: R01 (+), R10 (+);  zs: R01 (-), R10 (+)
    const float gxy = dR[0][1] + dR[1][0];
    dx += gxy * yC;
    dy += gxy * xC;
    dC += gxy * x * y;
    const float gzs = dR[1][0] - dR[0][1];
    dz += gzs * sa;
    dsa += gzs * z;
    // zxC = z*x*C: R02 (+), R20 (+);  ys: R02 (+), R20 (-)
    const float gzx = dR[0][2] + dR[2][0];
    dz += gzx * xC;
    dx += gzx * zC;
    dC += gzx * z * x;
    const float gys = dR[0][2] - dR[2][0];
    dy += gys * sa;
    dsa += gys * y;
    // yzC = y*z*C: R12 (+), R21 (+);  xs: R12 (-), R21 (+)
    const float gyz = dR[1][2] + dR[2][1];
    dy += gyz * zC;
    dz += gyz * yC;
    dC += gyz * y * z;
    const float gxs = dR[2][1] - dR[1][2];
    dx += gxs * sa;
    dsa += gxs * x;
    dca -= dC;  // C = 1 - ca
    float dangle = -sa * dca + ca * dsa;
    // axis = v / (angle + eps)
    const float dotv = dx * vx + dy * vy + dz * vz;
    dangle -= dotv / (den * den);
    float gvx = dx / den, gvy = dy / den, gvz = dz / den;
    if (angle > 0.f) {  // torch.norm backward: v / |v|, zero at the origin
        gvx += dangle * vx / angle;
        gvy += dangle * vy / angle;
        gvz += dangle * vz / angle;
    }
    daa[3 * i] = gvx;
    daa[3 * i + 1] = gvy;
    daa[3 * i + 2] = gvz;
    dtr[3 * i] = dt[0];
    dtr[3 * i + 1] = dt[1];
    dtr[3 * i + 2] = dt[2];
}

}  // namespace

extern "C" {

int md2_pose_fwd(int32_t frames, int32_t batch, uint32_t invert_mask, const float* axisangle,
                 const float* translation, float* T, void* stream) {
    if (frames < 1 || frames > 32 || batch < 1 || !axisangle || !translation || !T) return MD2_ERR_ARG;
    const int n = frames * batch;
    hipLaunchKernelGGL(pose_fwd_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, batch,
                       invert_mask, axisangle, translation, T);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

int md2_pose_bwd(int32_t frames, int32_t batch, uint32_t invert_mask, const float* axisangle,
                 const float* translation, const float* grad_T, float* grad_axisangle, float* grad_translation,
                 void* stream) {
    if (frames < 1 || frames > 32 || batch < 1 || !axisangle || !translation || !grad_T || !grad_axisangle ||
        !grad_translation)
        return MD2_ERR_ARG;
    const int n = frames * batch;
    hipLaunchKernelGGL(pose_bwd_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, batch,
                       invert_mask, axisangle, translation, grad_T, grad_axisangle, grad_translation);
    return hipGetLastError() == hipSuccess ? MD2_OK : MD2_ERR_HIP;
}

}  // extern "C"
