// md2_bf16.h — activation storage helpers shared by the NHWC kernels (bnorm.hip,
// decoder.hip): four consecutive channels as float4, stored as fp32 or bf16
// (uint16_t bits).  Arithmetic is fp32; stores round to nearest even, as torch's
// float -> bfloat16 conversion does.  Offsets are in elements.
#pragma once

#include <hip/hip_runtime.h>

#include <stdint.h>

namespace md2 {

__device__ __forceinline__ float bf2f(uint32_t b) { return __uint_as_float(b << 16); }

__device__ __forceinline__ uint32_t f2bf(float f) {
    const uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;   // NaN stays NaN
    return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}

template <typename T>
__device__ __forceinline__ float4 ld4T(const void* p, size_t off) {
    if constexpr (sizeof(T) == 4) {
        return *(const float4*)((const float*)p + off);
    } else {
        const uint2 r = *(const uint2*)((const uint16_t*)p + off);
        return {bf2f(r.x & 0xffffu), bf2f(r.x >> 16), bf2f(r.y & 0xffffu), bf2f(r.y >> 16)};
    }
}

template <typename T>
__device__ __forceinline__ void st4T(void* p, size_t off, float4 v) {
    if constexpr (sizeof(T) == 4) {
        *(float4*)((float*)p + off) = v;
    } else {
        *(uint2*)((uint16_t*)p + off) = make_uint2(f2bf(v.x) | (f2bf(v.y) << 16), f2bf(v.z) | (f2bf(v.w) << 16));
    }
}

}  // namespace md2
