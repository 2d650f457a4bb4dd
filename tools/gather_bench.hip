// gather_bench.hip — microbenchmark of the bilinear-gather forms the photometric
// kernels can use (DESIGN.md §3 "what binds the photo kernels").
//
// Workload: B x 3 x H x W fp32 source planes, one wave per 64-column strip walking
// ROWS rows; every lane samples its source at (x + dx, y + dy) with a smooth,
// near-identity displacement (|d| <= 2 px, what the bench's networks produce) or a
// large one (--far), 3 channels, and accumulates the bilinear value.
//
//   pair  : 6 global_load_dwordx2 per sample (two corners of a row per load; the
//           shipped photo kernels)
//   dword : 12 global_load_dword per sample
//   ring  : source rows staged in an LDS ring by row-coalesced dwordx4 loads, the
//           corners read back with ds_read2_b32; lanes whose footprint leaves the
//           window fall back to the pair loads
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/gather_bench tools/gather_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int kWave = 64;
constexpr int ROWS = 16;
constexpr int RING = 8;           // rows in the LDS ring
constexpr int RLO = 3;            // ring covers rows [r - RLO, r + RING - 1 - RLO]
constexpr int WC = 80;            // ring columns: strip start - 8 .. + 71
constexpr int WOFF = 8;

typedef float float2_a4 __attribute__((ext_vector_type(2), aligned(4)));

struct Args {
    const float* src;
    int B, H, W;
    float amp;   // displacement amplitude (px)
    float* out;
    int passes;
};

__device__ __forceinline__ void disp(const Args& a, int b, int y, int x, int p, float& ix, float& iy) {
    const float fx = (float)x, fy = (float)y;
    ix = fx + a.amp * (0.6f + 0.4f * __sinf(0.013f * fx + 0.7f * p + 0.1f * b)) ;
    iy = fy + a.amp * 0.5f * __cosf(0.021f * fy + 0.011f * fx + 0.3f * p);
    ix = fminf(fmaxf(ix, 0.f), (float)(a.W - 1));
    iy = fminf(fmaxf(iy, 0.f), (float)(a.H - 1));
}

template <int MODE>
__global__ __launch_bounds__(256, 2) void gather_kernel(Args a) {
    __shared__ float ring[4][3][RING][WC];
    const int lane = threadIdx.x & 63, wib = threadIdx.x >> 6;
    const int strips = (a.W + 63) / 64, rbs = (a.H + ROWS - 1) / ROWS;
    const int wv = blockIdx.x * 4 + wib;
    if (wv >= a.B * strips * rbs) return;
    const int b = wv / (strips * rbs), rem = wv % (strips * rbs);
    const int rb = rem / strips, st = rem % strips;
    const int x = min(st * 64 + lane, a.W - 1);
    const int HW = a.H * a.W;
    const float* src = a.src + (size_t)b * 3 * HW;
    const int c0 = st * 64 - WOFF;
    float acc = 0.f;
    for (int p = 0; p < a.passes; ++p) {
        int loaded_hi = -1000;  // highest source row staged in the ring so far
        for (int i = 0; i < ROWS; ++i) {
            const int y = min(rb * ROWS + i, a.H - 1);
            float ix, iy;
            disp(a, b, y, x, p, ix, iy);
            const float fx0 = floorf(ix), fy0 = floorf(iy);
            const int x0 = (int)fx0, y0 = (int)fy0;
            const float tx = ix - fx0, ty = iy - fy0;
            const bool vx1 = x0 + 1 < a.W, vy1 = y0 + 1 < a.H;
            const int y1 = vy1 ? y0 + 1 : y0;
            const int xa = vx1 ? x0 : x0 - 1;
            float v[3][4];
            if (MODE == 0) {
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const float2_a4 t = *(const float2_a4*)(src + (uint32_t)(ch * HW + y0 * a.W + xa));
                    const float2_a4 u = *(const float2_a4*)(src + (uint32_t)(ch * HW + y1 * a.W + xa));
                    v[ch][0] = t.x; v[ch][1] = t.y; v[ch][2] = u.x; v[ch][3] = u.y;
                }
            } else if (MODE == 1) {
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const float* s = src + ch * HW;
                    v[ch][0] = s[y0 * a.W + xa]; v[ch][1] = s[y0 * a.W + xa + 1];
                    v[ch][2] = s[y1 * a.W + xa]; v[ch][3] = s[y1 * a.W + xa + 1];
                }
            } else {
                // stage rows up to y + RING-1-RLO (row-coalesced: lanes = (ch, col quad))
                const int want_hi = min(y + RING - 1 - RLO, a.H - 1);
                const int want_lo = max(want_hi - RING + 1, 0);
                for (int r = max(loaded_hi + 1, want_lo); r <= want_hi; ++r) {
                    // 3 ch x 20 quads = 60 lanes
                    if (lane < 60) {
                        const int ch = lane / 20, q = lane % 20;
                        const int col = c0 + 4 * q;
                        float4 d;
                        if (col >= 0 && col + 3 < a.W) {
                            d = *(const float4*)(src + ch * HW + r * a.W + col);
                        } else {
                            d.x = (col + 0 >= 0 && col + 0 < a.W) ? src[ch * HW + r * a.W + col + 0] : 0.f;
                            d.y = (col + 1 >= 0 && col + 1 < a.W) ? src[ch * HW + r * a.W + col + 1] : 0.f;
                            d.z = (col + 2 >= 0 && col + 2 < a.W) ? src[ch * HW + r * a.W + col + 2] : 0.f;
                            d.w = (col + 3 >= 0 && col + 3 < a.W) ? src[ch * HW + r * a.W + col + 3] : 0.f;
                        }
                        *(float4*)&ring[wib][ch][r % RING][4 * q] = d;
                    }
                    loaded_hi = r;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const int lo = max(loaded_hi - RING + 1, 0);
                const bool in = xa >= c0 && xa + 1 < c0 + WC && y0 >= lo && y1 <= loaded_hi;
                if (in) {
                    const int cx = xa - c0;
#pragma unroll
                    for (int ch = 0; ch < 3; ++ch) {
                        const float* rt = &ring[wib][ch][y0 % RING][cx];
                        const float* rbm = &ring[wib][ch][y1 % RING][cx];
                        v[ch][0] = rt[0]; v[ch][1] = rt[1]; v[ch][2] = rbm[0]; v[ch][3] = rbm[1];
                    }
                } else {
#pragma unroll
                    for (int ch = 0; ch < 3; ++ch) {
                        const float2_a4 t = *(const float2_a4*)(src + (uint32_t)(ch * HW + y0 * a.W + xa));
                        const float2_a4 u = *(const float2_a4*)(src + (uint32_t)(ch * HW + y1 * a.W + xa));
                        v[ch][0] = t.x; v[ch][1] = t.y; v[ch][2] = u.x; v[ch][3] = u.y;
                    }
                }
            }
            const float e = 1.f - tx, so = 1.f - ty;
#pragma unroll
            for (int ch = 0; ch < 3; ++ch)
                acc += so * (e * v[ch][0] + tx * v[ch][1]) + ty * (e * v[ch][2] + tx * v[ch][3]);
        }
    }
    a.out[(size_t)wv * 64 + lane] = acc;
}

int main(int argc, char** argv) {
    int B = 48, H = 192, W = 640, passes = 8;
    float amp = 2.0f;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--far")) amp = 24.f;
        if (!strcmp(argv[i], "--amp")) amp = atof(argv[++i]);
    }
    const size_t n = (size_t)B * 3 * H * W;
    std::vector<float> h(n);
    for (size_t i = 0; i < n; ++i) h[i] = (float)((i * 2654435761u) % 1000) * 1e-3f;
    float *src, *out;
    const int strips = (W + 63) / 64, rbs = (H + ROWS - 1) / ROWS, waves = B * strips * rbs;
    CHECK(hipMalloc(&src, n * 4));
    CHECK(hipMalloc(&out, (size_t)waves * 64 * 4 * 3));
    CHECK(hipMemcpy(src, h.data(), n * 4, hipMemcpyHostToDevice));
    Args a{src, B, H, W, amp, out, passes};
    const int blocks = (waves + 3) / 4;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char* names[3] = {"pair(dwordx2)", "dword", "lds-ring"};
    std::vector<float> ref;
    for (int m = 0; m < 3; ++m) {
        a.out = out + (size_t)m * waves * 64;
        for (int rep = 0; rep < 2; ++rep) {
            CHECK(hipEventRecord(e0));
            const int iters = 20;
            for (int it = 0; it < iters; ++it) {
                if (m == 0) gather_kernel<0><<<blocks, 256>>>(a);
                if (m == 1) gather_kernel<1><<<blocks, 256>>>(a);
                if (m == 2) gather_kernel<2><<<blocks, 256>>>(a);
            }
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            if (rep == 1) {
                const double samples = (double)B * H * W * passes;
                printf("%-14s amp %5.1f: %8.2f us/launch  %6.2f Gsample/s\n", names[m], amp, 1e3 * ms / iters,
                       samples / (ms / iters * 1e-3) / 1e9);
            }
        }
        std::vector<float> o((size_t)waves * 64);
        CHECK(hipMemcpy(o.data(), a.out, o.size() * 4, hipMemcpyDeviceToHost));
        if (m == 0) ref = o;
        else {
            double md = 0;
            for (size_t i = 0; i < o.size(); ++i) md = fmax(md, fabs(o[i] - ref[i]));
            printf("  max |diff| vs pair: %g\n", md);
        }
    }
    return 0;
}
