// gather_model.hip — what the texture path charges for the bilinear gathers of the
// photometric kernels: planar fp32 (the shipped layout) vs pixel-interleaved forms,
// under a smooth (near-identity) and a scattered (per-lane random, as random
// disparities give) displacement.  One wave per 64-column strip, 16 rows.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/gather_model tools/gather_model.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)
typedef float float2_a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef unsigned int uint2_a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef float float4_a4 __attribute__((ext_vector_type(4), aligned(4)));
constexpr int ROWS = 16;

struct Args { const float* planar; const float* rgba; const unsigned* rgba8; int B, H, W; float amp, jit; float* out; int passes; };

__device__ __forceinline__ unsigned hsh(unsigned x) { x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16; return x; }

template <int MODE>
__global__ __launch_bounds__(256, 2) void k(Args a) {
    const int lane = threadIdx.x & 63;
    const int strips = (a.W + 63) / 64, rbs = (a.H + ROWS - 1) / ROWS;
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wv >= a.B * strips * rbs) return;
    const int b = wv / (strips * rbs), rem = wv % (strips * rbs), rb = rem / strips, st = rem % strips;
    const int x = min(st * 64 + lane, a.W - 1), HW = a.H * a.W;
    float acc = 0.f;
    for (int p = 0; p < a.passes; ++p)
        for (int i = 0; i < ROWS; ++i) {
            const int y = min(rb * ROWS + i, a.H - 1);
            const unsigned h = hsh((unsigned)(((b * a.H + y) * a.W + x) * 8 + p));
            float ix = x + a.amp * (0.6f + 0.4f * __sinf(0.013f * x + 0.7f * p)) + a.jit * ((float)(h & 0xffff) / 65535.f - 0.5f);
            float iy = y + 0.5f * a.amp * __cosf(0.021f * y + 0.3f * p) + 0.25f * a.jit * ((float)(h >> 16) / 65535.f - 0.5f);
            ix = fminf(fmaxf(ix, 0.f), (float)(a.W - 2)); iy = fminf(fmaxf(iy, 0.f), (float)(a.H - 2));
            const int x0 = (int)ix, y0 = (int)iy;
            const float tx = ix - x0, ty = iy - y0;
            float v[3][4];
            if (MODE == 0) {          // planar fp32 pairs: 6 x dwordx2
                const float* s = a.planar + (size_t)b * 3 * HW;
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    float2_a4 t = *(const float2_a4*)(s + c * HW + y0 * a.W + x0), u = *(const float2_a4*)(s + c * HW + (y0 + 1) * a.W + x0);
                    v[c][0] = t.x; v[c][1] = t.y; v[c][2] = u.x; v[c][3] = u.y;
                }
            } else if (MODE == 1) {   // interleaved fp32 RGBA: 4 x dwordx4
                const float4_a4* s = (const float4_a4*)a.rgba + (size_t)b * HW;
                float4_a4 q[4] = {s[y0 * a.W + x0], s[y0 * a.W + x0 + 1], s[(y0 + 1) * a.W + x0], s[(y0 + 1) * a.W + x0 + 1]};
#pragma unroll
                for (int c = 0; c < 3; ++c) for (int j = 0; j < 4; ++j) v[c][j] = q[j][c];
            } else {                  // interleaved u8 RGBA: 2 x dwordx2
                const unsigned* s = a.rgba8 + (size_t)b * HW;
                uint2_a4 t = *(const uint2_a4*)(s + y0 * a.W + x0), u = *(const uint2_a4*)(s + (y0 + 1) * a.W + x0);
                unsigned q[4] = {t.x, t.y, u.x, u.y};
#pragma unroll
                for (int c = 0; c < 3; ++c) for (int j = 0; j < 4; ++j) v[c][j] = (float)((q[j] >> (8 * c)) & 255) * (1.f / 255.f);
            }
            const float e = 1.f - tx, so = 1.f - ty;
#pragma unroll
            for (int c = 0; c < 3; ++c) acc += so * (e * v[c][0] + tx * v[c][1]) + ty * (e * v[c][2] + tx * v[c][3]);
        }
    a.out[(size_t)wv * 64 + lane] = acc;
}

int main(int argc, char** argv) {
    int B = 12, H = 192, W = 640, passes = 8;
    const size_t n = (size_t)B * H * W;
    std::vector<float> hp(n * 3), hr(n * 4); std::vector<unsigned> h8(n);
    for (size_t i = 0; i < n; ++i) {
        unsigned c[3];
        for (int k = 0; k < 3; ++k) { c[k] = (unsigned)((i * 2654435761u + k * 97) % 256); }
        size_t b = i / (H * W), pix = i % (H * W);
        for (int k = 0; k < 3; ++k) { hp[(b * 3 + k) * H * W + pix] = c[k] / 255.f; hr[i * 4 + k] = c[k] / 255.f; }
        hr[i * 4 + 3] = 0.f; h8[i] = c[0] | (c[1] << 8) | (c[2] << 16);
    }
    float *dp, *dr, *out; unsigned* d8;
    CHECK(hipMalloc(&dp, n * 12)); CHECK(hipMalloc(&dr, n * 16)); CHECK(hipMalloc(&d8, n * 4));
    const int strips = (W + 63) / 64, rbs = (H + ROWS - 1) / ROWS, waves = B * strips * rbs;
    CHECK(hipMalloc(&out, (size_t)waves * 64 * 4));
    CHECK(hipMemcpy(dp, hp.data(), n * 12, hipMemcpyHostToDevice)); CHECK(hipMemcpy(dr, hr.data(), n * 16, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(d8, h8.data(), n * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    const char* names[3] = {"planar-f32 6xdwordx2", "rgba-f32 4xdwordx4", "rgba-u8 2xdwordx2"};
    float cfg[3][2] = {{2.f, 0.f}, {8.f, 6.f}, {16.f, 60.f}};
    for (int c = 0; c < 3; ++c) {
        Args a{dp, dr, d8, B, H, W, cfg[c][0], cfg[c][1], out, passes};
        for (int m = 0; m < 3; ++m) {
            float ms = 0;
            for (int rep = 0; rep < 2; ++rep) {
                CHECK(hipEventRecord(e0));
                for (int it = 0; it < 10; ++it) {
                    if (m == 0) k<0><<<(waves + 3) / 4, 256>>>(a);
                    if (m == 1) k<1><<<(waves + 3) / 4, 256>>>(a);
                    if (m == 2) k<2><<<(waves + 3) / 4, 256>>>(a);
                }
                CHECK(hipEventRecord(e1)); CHECK(hipEventSynchronize(e1)); CHECK(hipEventElapsedTime(&ms, e0, e1));
            }
            printf("amp %4.1f jitter %4.1f  %-22s %8.2f us  %6.1f Gsample/s\n", cfg[c][0], cfg[c][1], names[m], 100.f * ms,
                   (double)n * passes / (ms / 10 * 1e-3) / 1e9);
        }
    }
    return 0;
}
