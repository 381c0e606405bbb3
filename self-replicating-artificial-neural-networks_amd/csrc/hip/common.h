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
// round-to-nearest-even fp32 -> bf16 (NaN stays NaN): one v_cvt_pk_bf16_f32 on gfx950 (the bit-manipulation
// form it replaces cost ~6 VALU ops per element in every epilogue and BatchNorm pass)
__device__ __forceinline__ bf16_t f2bf(float f) {
    return __builtin_bit_cast(bf16_t, (__bf16)f);
}
// two values -> one packed bf16 pair (lo = a, hi = b): one instruction for both
typedef __bf16 bf16x2_hw __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t f2bf2(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_hw));
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

// ---- deterministic accumulation -------------------------------------------------
// Every float reduction whose partial sums meet through atomics -- WGRAD m-splits and bias gradients
// into the gradient arena, BatchNorm statistics, the loss metrics -- accumulates in signed 64-bit fixed
// point.  Integer addition is associative and wraps modulo 2^64, so the total is independent of the
// order in which the atomics land (and of transient overflow): a replayed training step is bitwise
// reproducible, and so is the population a seeded experiment evolves.
//  * fx ("Q40", one word): the gradient arena.  40 fractional bits: resolution 2^-40 = 9.1e-13 absolute, final
//    sums within +-2^23 (8.4M; a gradient element is O(1e2) at most).  Each contribution is clamped to +-2^22
//    first (NaN -> -2^22) so the conversion is always defined.  The resolution is what Keras' eps = 1e-7 Adam
//    needs (the RiboAE trainer shares this arena): a gradient of 1e-10 carries < 1 % quantisation error, where
//    the former Q32 arena (2.3e-10) flushed it to zero or doubled it.
//  * fxm ("Q32", one word): the loss metrics (sums over up to an epoch of rows: range +-2^31).
//  * fxw ("wide", two words hi, lo): BatchNorm statistics (sums of squares over up to 588k rows).  A
//    contribution q = round(v * 2^32) is split as hi = q >> 32, lo = q & (2^32 - 1) (lo >= 0); the
//    words are summed separately, total = hi + lo * 2^-32: resolution 2^-32, range +-2^63.
typedef unsigned long long u64_t;
constexpr float FX_SCALE = 1099511627776.f;          // 2^40 (gradient arena)
constexpr float FX_INV = 9.094947017729282e-13f;     // 2^-40
constexpr float FX_CLAMP = 4194304.f;                // 2^22
constexpr float FXW_SCALE = 4294967296.f;            // 2^32 (metrics, wide statistics)

__device__ __forceinline__ long long fx_q(float v) {
    return llrintf(fminf(fmaxf(v, -FX_CLAMP), FX_CLAMP) * FX_SCALE);
}
__device__ __forceinline__ void fx_add(long long* p, float v) {
    atomicAdd(reinterpret_cast<u64_t*>(p), (u64_t)fx_q(v));
}
__device__ __forceinline__ float fx_f(long long q) { return (float)q * FX_INV; }
__device__ __forceinline__ void fxm_add(long long* p, float v) {
    atomicAdd(reinterpret_cast<u64_t*>(p), (u64_t)llrintf(fminf(fmaxf(v, -1073741824.f), 1073741824.f) * FXW_SCALE));
}

__device__ __forceinline__ void fxw_add(long long* p, float v) {
    long long hi, lo = 0;
    if (fabsf(v) < 1.0e9f) {
        const long long q = llrintf(v * FXW_SCALE);
        hi = q >> 32;
        lo = q & 0xffffffffLL;
    } else {                                          // |v| >= 1e9 > 2^24: already an integer (or NaN)
        hi = (v != v) ? 0 : (long long)fminf(fmaxf(v, -9.0e18f), 9.0e18f);
    }
    atomicAdd(reinterpret_cast<u64_t*>(p), (u64_t)hi);
    if (lo) atomicAdd(reinterpret_cast<u64_t*>(p + 1), (u64_t)lo);
}
// Sum of sum index ``idx`` over the BN_WS_STRIPES copies of a wide statistics workspace laid out as
// [stripe][2C sums][hi, lo] (serann_hip.h BN_WS_STRIPES); integer sums first, one rounding at the end.
template <int STRIPES>
__device__ __forceinline__ float fxw_sum(const long long* ws, int C, int idx) {
    long long hi = 0;
    u64_t lo = 0;
#pragma unroll
    for (int s = 0; s < STRIPES; ++s) {
        hi += ws[2 * (s * 2 * C + idx)];
        lo += (u64_t)ws[2 * (s * 2 * C + idx) + 1];
    }
    return (float)((double)hi + (double)lo * (1.0 / 4294967296.0));
}
// The same sum in double (unshifted statistics: sum x^2 - (sum x)^2 / n without fp32 cancellation)
template <int STRIPES>
__device__ __forceinline__ double fxw_sum_d(const long long* ws, int C, int idx) {
    long long hi = 0;
    u64_t lo = 0;
#pragma unroll
    for (int s = 0; s < STRIPES; ++s) {
        hi += ws[2 * (s * 2 * C + idx)];
        lo += (u64_t)ws[2 * (s * 2 * C + idx) + 1];
    }
    return (double)hi + (double)lo * (1.0 / 4294967296.0);
}

// Keras / TF ResourceApplyAdam on one element (experiment_worker.py:80): shared by the arena-wide Adam pass
// and the WGRAD epilogues that apply the step to their own tile (GF_ADAM), so both give the same bits.
// Every operation is spelled out (explicit fma, IEEE sqrt and division, no contraction) so the two call
// sites cannot be compiled into different roundings.
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float lr_t, float b1, float b2,
                                          float eps) {
#pragma clang fp contract(off)
    m = __fmaf_rn(b1, m, (1.f - b1) * g);
    v = __fmaf_rn(b2, v, ((1.f - b2) * g) * g);
    const float den = __fsqrt_rn(v) + eps;
    p = p - __fdiv_rn(lr_t * m, den);
}

static inline hipStream_t as_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename T> static inline T* as_ptr(uint64_t p) { return reinterpret_cast<T*>(p); }
