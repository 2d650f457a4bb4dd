// stem.hip — weight gradient of the ResNet stem convolution (conv1: 7x7, stride 2,
// padding 3, C -> 64, no bias; networks/resnet_encoder.py -> torchvision conv1) on
// gfx950 f32 MFMA.
//
// The stem's input is data (the normalised frames), so its backward is the weight
// gradient alone: dW[co][ky][kx][ci] = Σ_p dy[p][co] · x[p's 7x7 window][ky][kx][ci]
// over every output pixel p — a GEMM with M = 64 output channels, N = 49·C window
// taps, and the reduction over B·Ho·Wo pixels (368k at B=12, 192x640).  MIOpen runs it
// at 41 TFLOP/s (C=3) / 71 TFLOP/s (C=6, the pose encoder's frame pair); here:
//   * v_mfma_f32_32x32x2_f32 (exact f32 fma chains), K = 2 pixels per instruction:
//     lane l feeds dy[pixel 2q + l/32][co tile + l%32] as A and the window tap
//     x[pixel 2q + l/32][tap tile + l%32] as B, gathered straight from the NHWC input
//     (taps of one window row are C·7 contiguous floats; zero outside the image);
//   * blocks walk 64-pixel output row segments, staging the window rows and dy in LDS
//     (double-buffered); a wave owns both 32-channel tiles × 5 tap tiles (160
//     accumulators) for its pixel pairs; the 8 waves of a block are summed in LDS in wave order,
//     blocks write partials, a second launch sums them in block order — deterministic,
//     no atomics.
// Layouts: x (B,H,W,C) and dy (B,Ho,Wo,64) channels_last fp32; dW in the weight's own
// memory format (channels_last [co][ky][kx][ci] or contiguous [co][ci][ky][kx]).

#include <hip/hip_runtime.h>

#include <stdint.h>

#include "md2hot.h"

int md2_report_error(int code, const char* msg);

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWaves = 8;       // waves per block
constexpr int kThreads = 64 * kWaves;
constexpr int kNTW = 5;         // 32-wide tap tiles per wave
constexpr int kNB = 32 * kNTW;  // taps per tap group (160)
constexpr int kCo = 64;
constexpr int kBlocks = 256;    // blocks per tap group: one per CU
constexpr int kPartStride = kCo * kNB + 64;   // floats per block partial (padded)

struct StemArgs {
    int B, C, H, W, Ho, Wo;
    int w_cl;
    const float* x;
    const float* gy;
    float* part;   // [tap group][block][64][160]
    const float* zeros;   // 64 zero floats (the workspace tail): DMA source outside the image
    float* gw;
};

// Blocks walk segments of kSeg consecutive output pixels of one output row.  Per
// segment the 7 input rows under it (2·kSeg+5 columns, zero outside the image) and
// its dy rows are staged in LDS by LDS-DMA (global_load_lds_dword: no staging
// registers), three buffers deep: segment s+2 is in flight while s is computed, so the
// MFMAs do not wait on HBM latency.  The MFMA operands come from LDS with no per-lane
// bounds checks or pixel decoding.  Wave w takes pixel pairs w, w+8, ... of the
// segment with all 2×kNTW tiles of its tap group.
constexpr int kSeg = 64;
constexpr int kSW = 2 * kSeg + 5;   // staged input columns
constexpr int kDyS = 65;            // dy row stride in LDS (pair halves on different banks)
constexpr int kBufs = 3;

template <int C>
struct StemLds {
    static constexpr int RW = kSW * C;                     // floats per staged input row
    static constexpr int RI = (RW + 63) / 64;              // DMA instructions per row
    static constexpr int XI = 7 * RI;                      // ... per segment's input rows
    static constexpr int NXI = (XI + kWaves - 1) / kWaves; // per wave (padded with dummies)
    static constexpr int K = NXI + kSeg / kWaves;          // DMA instructions per wave per segment
    static constexpr int RWP = RI * 64;                    // LDS row stride (whole DMA rows)
    static constexpr int XS = 7 * RWP;
    static constexpr int DS = kSeg * kDyS;
    static constexpr int BUF = XS + DS;
    static constexpr int TOTAL = kBufs * BUF + 64;         // + the dummies' landing row
};

// s_waitcnt vmcnt(VM) (expcnt / lgkmcnt unconstrained), gfx9 encoding
template <int VM>
__device__ __forceinline__ void wait_vm() {
    static_assert(VM >= 0 && VM < 64, "vmcnt");
    __builtin_amdgcn_s_waitcnt((VM & 0xF) | ((VM >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// Workgroup barrier that leaves the LDS-DMA prefetches in flight: __syncthreads()'s
// workgroup fence waits for every outstanding vector-memory op (vmcnt(0)), which would
// drain the pipeline each segment.  The wait_vm<> calls order the DMA explicitly; the
// "memory" clobber keeps the compiler from moving LDS accesses across the barrier.
__device__ __forceinline__ void block_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <int C>
__global__ __launch_bounds__(kThreads) void stem_wgrad_kernel(StemArgs a) {
    using L = StemLds<C>;
    constexpr int KC = 49 * C;
    static_assert(2 * L::K < 64, "in-flight DMA count exceeds vmcnt");
    __shared__ float lds[L::TOTAL > kCo * kNB ? L::TOTAL : kCo * kNB];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int col = lane & 31, half = lane >> 5;
    const int ng = blockIdx.y;
    const int H = a.H, W = a.W, Ho = a.Ho, Wo = a.Wo;
    int toff[kNTW];
    bool tv[kNTW];
#pragma unroll
    for (int t = 0; t < kNTW; ++t) {
        const int n = (ng * kNTW + t) * 32 + col;
        tv[t] = n < KC;
        const int nn = tv[t] ? n : 0;
        const int ky = nn / (7 * C), r = nn - ky * 7 * C, kx = r / C, ci = r - kx * C;
        toff[t] = ky * L::RWP + kx * C + ci;
    }
    f32x16 acc[2][kNTW];
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int t = 0; t < kNTW; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[m][t][r] = 0.f;

    const int spr = (Wo + kSeg - 1) / kSeg;   // segments per output row
    const int nseg = a.B * Ho * spr;
    float* dummy = lds + kBufs * L::BUF;
    // exactly L::K DMA instructions per wave (out-of-image lanes copy zeros)
    // Row r of the window is x[b][iy0 + r][ix0 .. ix0 + 2·kSeg + 4][0 .. C) — one
    // contiguous run of RW floats starting at element ix0·C of the image row, so a lane's
    // element e is in the image iff 0 <= ix0·C + e < W·C: no per-lane division.  The
    // address math is per wave (scalar) except for that one add and compare.
    const int WC = W * C;
    auto issue = [&](int sg, float* buf) {
        const int sx = sg % spr, t2 = sg / spr, oy = t2 % Ho, b = t2 / Ho;
        const int ox0 = sx * kSeg, iy0 = 2 * oy - 3, e0 = (2 * ox0 - 3) * C;
        const float* img = a.x + (size_t)b * H * WC;
#pragma unroll
        for (int k = 0; k < L::NXI; ++k) {
            const int ins = wave + k * kWaves;
            if (ins >= L::XI) {
                __builtin_amdgcn_global_load_lds(a.zeros + lane, (uint32_t*)dummy, 4, 0, 0);
                continue;
            }
            const int r = ins / L::RI, c0 = (ins - r * L::RI) * 64;        // wave-uniform
            const int iy = iy0 + r;
            const bool row_ok = iy >= 0 && iy < H;
            const int e = c0 + lane, eg = e0 + e;                          // element in the image row
            const bool ok = row_ok && e < L::RW && (unsigned)eg < (unsigned)WC;
            // every lane issues (the per-wave DMA count must be exactly K for the
            // vmcnt waits): outside the image / past the row, it copies a zero
            const float* src = ok ? img + (size_t)(row_ok ? iy : 0) * WC + eg : a.zeros + lane;
            __builtin_amdgcn_global_load_lds(src, (uint32_t*)(buf + r * L::RWP + c0), 4, 0, 0);
        }
        float* dy = buf + L::XS;
        const float* gyrow = a.gy + (size_t)(b * Ho + oy) * Wo * kCo;
#pragma unroll
        for (int k = 0; k < kSeg / kWaves; ++k) {
            const int j = wave + k * kWaves, ox = ox0 + j;
            const float* src = ox < Wo ? gyrow + (size_t)ox * kCo + lane : a.zeros + lane;
            __builtin_amdgcn_global_load_lds(src, (uint32_t*)(dy + j * kDyS), 4, 0, 0);
        }
    };
    int sg = blockIdx.x;
    const int G = gridDim.x;
    if (sg < nseg) issue(sg, lds);
    if (sg + G < nseg) issue(sg + G, lds + L::BUF);
    int cur = 0;
    for (; sg < nseg; sg += G) {
        const bool far = sg + 2 * G < nseg;
        if (far) {
            issue(sg + 2 * G, lds + ((cur + 2) % kBufs) * L::BUF);
            wait_vm<2 * L::K>();                 // this segment's DMA is done
        } else if (sg + G < nseg) {
            wait_vm<L::K>();
        } else {
            wait_vm<0>();
        }
        block_sync();                            // every wave's DMA for this segment landed
        const float* xb = lds + cur * L::BUF;
        const float* dyb = xb + L::XS;
#pragma unroll
        for (int i = 0; i < kSeg / 2 / kWaves; ++i) {
            const int j = 2 * (wave + i * kWaves) + half;   // pixel within the segment
            const float a0 = dyb[j * kDyS + col], a1 = dyb[j * kDyS + 32 + col];
            float bv[kNTW];
#pragma unroll
            for (int t = 0; t < kNTW; ++t) bv[t] = tv[t] ? xb[toff[t] + 2 * j * C] : 0.f;
#pragma unroll
            for (int t = 0; t < kNTW; ++t) {
                acc[0][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, bv[t], acc[0][t], 0, 0, 0);
                acc[1][t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, bv[t], acc[1][t], 0, 0, 0);
            }
        }
        block_sync();                            // buffer `cur` is refilled two segments on
        cur = (cur + 1) % kBufs;
    }
    wait_vm<0>();
    __syncthreads();

    // waves summed in wave order into LDS [co][160] (the staging buffers are free now);
    // D layout: col = lane%32 (tap), row = (r&3) + 8(r>>2) + 4(lane/32) (channel in tile)
    float* red = lds;
    for (int w = 0; w < kWaves; ++w) {
        if (wave == w) {
#pragma unroll
            for (int m = 0; m < 2; ++m)
#pragma unroll
                for (int t = 0; t < kNTW; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) {
                        const int co = m * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
                        float* d = red + co * kNB + t * 32 + col;
                        *d = w == 0 ? acc[m][t][r] : *d + acc[m][t][r];
                    }
        }
        __syncthreads();
    }
    float* out = a.part + ((size_t)ng * gridDim.x + blockIdx.x) * kPartStride;
    for (int e = threadIdx.x; e < kCo * kNB; e += kThreads) out[e] = red[e];
}

// dW[co][n] = Σ_blocks part: a block takes 64 outputs × 4 block slices (16 loads in
// flight per thread), slices combined in order through LDS — fixed order throughout.
__global__ __launch_bounds__(256) void stem_wgrad_final_kernel(StemArgs a, int G) {
    const int KC = 49 * a.C;
    const int el = threadIdx.x & 63, sl = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + el;
    float s = 0.f;
    int co = 0, n = 0;
    if (e < kCo * KC) {
        co = e / KC;
        n = e - co * KC;
        const int ng = n / kNB, nl = n - ng * kNB;
        const float* p = a.part + (size_t)ng * G * kPartStride + co * kNB + nl;
        constexpr int R = 16;
        float c[R];
#pragma unroll
        for (int r = 0; r < R; ++r) c[r] = 0.f;
        for (int g0 = sl * R; g0 < G; g0 += 4 * R)
#pragma unroll
            for (int r = 0; r < R; ++r)
                if (g0 + r < G) c[r] += p[(size_t)(g0 + r) * kPartStride];
#pragma unroll
        for (int r = 0; r < R; ++r) s += c[r];
    }
    __shared__ float red[4][64];
    red[sl][el] = s;
    __syncthreads();
    if (sl != 0 || e >= kCo * KC) return;
    s = ((red[0][el] + red[1][el]) + red[2][el]) + red[3][el];
    if (a.w_cl) {
        a.gw[e] = s;
    } else {
        const int ky = n / (7 * a.C), r = n - ky * 7 * a.C, kx = r / a.C, ci = r - kx * a.C;
        a.gw[((co * a.C + ci) * 7 + ky) * 7 + kx] = s;
    }
}

bool valid(const md2_stem_desc* d) {
    return d && d->batch >= 1 && d->height >= 1 && d->width >= 1 &&
           (d->channels == 3 || d->channels == 6 || d->channels == 9) &&
           (long long)d->batch * d->height * d->width * d->channels < (1ll << 31);
}

int groups_of(int C) { return (49 * C + kNB - 1) / kNB; }

}  // namespace

extern "C" {

size_t md2_stem_wgrad_workspace_bytes(const md2_stem_desc* d) {
    if (!valid(d)) return 0;
    return sizeof(float) * ((size_t)groups_of(d->channels) * kBlocks * kPartStride + 64);
}

int md2_stem_wgrad(const md2_stem_desc* d, const float* x, const float* grad_y, float* grad_weight, void* workspace,
                   void* stream) {
    if (!valid(d)) return md2_report_error(MD2_ERR_ARG, "stem_wgrad: channels 3/6/9, 32-bit element count");
    if (!x || !grad_y || !grad_weight || !workspace) return md2_report_error(MD2_ERR_ARG, "stem_wgrad: NULL operand");
    StemArgs a = {};
    a.B = d->batch;
    a.C = d->channels;
    a.H = d->height;
    a.W = d->width;
    a.Ho = (d->height - 1) / 2 + 1;   // (H + 2·3 - 7) / 2 + 1
    a.Wo = (d->width - 1) / 2 + 1;
    a.w_cl = (d->flags & MD2_STEM_WEIGHT_CL) ? 1 : 0;
    a.x = x;
    a.gy = grad_y;
    a.part = (float*)workspace;
    const size_t nzero = (size_t)groups_of(a.C) * kBlocks * kPartStride;
    a.zeros = a.part + nzero;
    a.gw = grad_weight;
    const int NG = groups_of(a.C);
    void (*k)(StemArgs) = a.C == 3 ? stem_wgrad_kernel<3> : a.C == 6 ? stem_wgrad_kernel<6> : stem_wgrad_kernel<9>;
    const hipStream_t st = (hipStream_t)stream;
    if (hipMemsetAsync(a.part + nzero, 0, 64 * sizeof(float), st) != hipSuccess)
        return md2_report_error(MD2_ERR_HIP, "stem_wgrad: memset");
    hipLaunchKernelGGL(k, dim3(kBlocks, NG), dim3(kThreads), 0, st, a);
    const int outs = kCo * 49 * a.C;
    hipLaunchKernelGGL(stem_wgrad_final_kernel, dim3((outs + 63) / 64), dim3(256), 0, st, a, kBlocks);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? MD2_OK : md2_report_error(MD2_ERR_HIP, hipGetErrorString(e));
}

}  // extern "C"
