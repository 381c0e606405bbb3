// Shared helpers for SeRANN-AMD HIP kernels (gfx950 / CDNA4: 64-wide waves, MFMA, 160 KB LDS).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define SERANN_CHECK(x)                                                                       \
    do {                                                                                      \
        hipError_t e__ = (x);                                                                 \
        if (e__ != hipSuccess) throw std::runtime_error(std::string("HIP error: ") +          \
                                                        hipGetErrorString(e__) + " at " +     \
                                                        __FILE__ + ":" + std::to_string(__LINE__)); \
    } while (0)

typedef uint16_t bf16_t;   // raw bf16 storage

__device__ __forceinline__ float bf2f(bf16_t v) {
    return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even fp32 -> bf16 (NaN preserved)
__device__ __forceinline__ bf16_t f2bf(float f) {
    uint32_t u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16_t)((u >> 16) | 0x40);
    u += 0x7fffu + ((u >> 16) & 1u);
    return (bf16_t)(u >> 16);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

enum Act : int { ACT_LINEAR = 0, ACT_RELU = 1, ACT_SIGMOID = 2 };

__device__ __forceinline__ float apply_act(float x, int act) {
    if (act == ACT_RELU) return x > 0.f ? x : 0.f;
    if (act == ACT_SIGMOID) return 1.f / (1.f + __expf(-x));
    return x;
}
// derivative expressed through the activation OUTPUT y
__device__ __forceinline__ float act_grad_from_y(float y, int act) {
    if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
    if (act == ACT_SIGMOID) return y * (1.f - y);
    return 1.f;
}

static inline hipStream_t as_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename T> static inline T* as_ptr(uint64_t p) { return reinterpret_cast<T*>(p); }
