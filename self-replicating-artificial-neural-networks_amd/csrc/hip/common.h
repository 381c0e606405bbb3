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

// Divergence detection (the reference's fp16 semantics).  The Q40 arena wraps silently when a gradient sum leaves
// +-2^23; a wrapped sum lands uniformly in [-2^23, 2^23), so it still exceeds fp16's largest finite value 65504 with
// probability 0.99 per element -- and an exploding organism has many such elements.  Every Adam site (the arena pass
// and the fused WGRAD / finalize epilogues) therefore flags the organism owning a gradient element with
// |g| > FX_DIVERGE: in the reference's float16 graph that gradient is inf, the weights become NaN and so do the
// organism's metrics (experiment_worker.py:36-37); the engine reports the flagged organisms' metrics as NaN
// (fertility 0, as for an invalid organism).  org_off: int64 [norg + 1] first arena element of each organism
// (ascending; the parameter arena is laid out organism by organism); diverged: int32 [norg].
constexpr float FX_DIVERGE = 65504.f;
#ifndef SERANN_DIVERGE_CHECK
#define SERANN_DIVERGE_CHECK 1      // build-time A/B knob of the fused WGRAD epilogues' check
#endif
__device__ __forceinline__ void flag_diverged(const int64_t* __restrict__ org_off, int* __restrict__ diverged, int norg,
                                           int64_t e) {
    int lo = 0, hi = norg - 1;                       // the last organism whose first element is <= e
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (org_off[mid] <= e) lo = mid; else hi = mid - 1;
    }
    diverged[lo] = 1;
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

// Adam moment storage (AdamCtx::mode, adam_kernel<MM>).  MOM_F32: fp32 m and v.  MOM_16: both moments in 16 bits,
// as the reference keeps them (fp16 floatx: experiment_worker.py:36-37, optimizer :80), master weights fp32:
//  * m: bf16 (RNE).  b1 = 0.9 moves m by 10 % of (g - m) per step, far above bf16's half ulp (2^-9), so the EMA
//    tracks; the stored value carries 0.4 % relative error into the update.
//  * v: "log16", an unsigned 16-bit log code: q = rint(LOG16_SCALE * (log2 v + LOG16_BIAS)) in [1, 65535] covers
//    v in [2^-48, 2^32) = [3.6e-15, 4.3e9] (80 octaves, 819.2 codes per octave); q = 0 is v = 0, and v < 2^-48 flushes
//    to 0 (sqrt(v) < 6e-8, nothing next to eps = 1e-4), v >= 2^32 saturates (|g| > 65504: flag_diverged).  An EMA
//    with b2 = 0.999 moves v by 0.1 % of (g^2 - v) per step: in bf16 (half ulp 0.2 %) that increment rounds away
//    unless g^2 > 3 v, so v would freeze.  log16's neighbouring values differ by 2^(1/819.2) (half ulp 0.042 %,
//    within fp16's 0.024 .. 0.049 %), over a range fp16 lacks: fp16 flushes v below 6e-8 (|g| < 2.4e-4) and
//    overflows at 65504.  sqrt(v) is what the update reads.
// The arithmetic is adam_elem's in fp32 either way; the moments are rounded once when stored.  18 B per parameter
// and step instead of 26 in the fused WGRAD epilogues (p 4+4, m 2+2, v 2+2, bf16 shadow 2).
constexpr int MOM_F32 = 0, MOM_16 = 1;
constexpr float LOG16_SCALE = 819.2f, LOG16_BIAS = 48.f;
__device__ __forceinline__ float log16_f(uint32_t q) {          // q: the low 16 bits are the code
    q &= 0xffffu;
    return q == 0 ? 0.f : __builtin_amdgcn_exp2f((float)q * (1.f / LOG16_SCALE) - LOG16_BIAS);
}
__device__ __forceinline__ uint16_t log16_q(float v) {
    if (!(v >= 3.5527137e-15f)) return 0;                           // 0, < 2^-48 (and NaN, never produced)
    const float l = (__builtin_amdgcn_logf(v) + LOG16_BIAS) * LOG16_SCALE;
    return (uint16_t)min(max(__float2int_rn(l), 1), 65535);
}
template <int MM>
__device__ __forceinline__ float m_ld(const void* b, int64_t e) {
    if constexpr (MM == MOM_16) return bf2f(reinterpret_cast<const bf16_t*>(b)[e]);
    else return reinterpret_cast<const float*>(b)[e];
}
template <int MM>
__device__ __forceinline__ void m_st(void* b, int64_t e, float x) {
    if constexpr (MM == MOM_16) reinterpret_cast<bf16_t*>(b)[e] = f2bf(x);
    else reinterpret_cast<float*>(b)[e] = x;
}
template <int MM>
__device__ __forceinline__ float v_ld(const void* b, int64_t e) {
    if constexpr (MM == MOM_16) return log16_f(reinterpret_cast<const uint16_t*>(b)[e]);
    else return reinterpret_cast<const float*>(b)[e];
}
template <int MM>
__device__ __forceinline__ void v_st(void* b, int64_t e, float x) {
    if constexpr (MM == MOM_16) reinterpret_cast<uint16_t*>(b)[e] = log16_q(x);
    else reinterpret_cast<float*>(b)[e] = x;
}
// four consecutive moments, e % 4 == 0 (16-B fp32 / 8-B 16-bit vectors)
template <int MM>
__device__ __forceinline__ float4 m_ld4(const void* b, int64_t e) {
    if constexpr (MM == MOM_16) {
        const uint2 u = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(b) + e);
        return make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                           __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u));
    } else {
        return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(b) + e);
    }
}
template <int MM>
__device__ __forceinline__ void m_st4(void* b, int64_t e, float4 x) {
    if constexpr (MM == MOM_16)
        *reinterpret_cast<uint2*>(reinterpret_cast<bf16_t*>(b) + e) = make_uint2(f2bf2(x.x, x.y), f2bf2(x.z, x.w));
    else
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(b) + e) = x;
}
template <int MM>
__device__ __forceinline__ float4 v_ld4(const void* b, int64_t e) {
    if constexpr (MM == MOM_16) {
        const uint2 q = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(b) + e);
        return make_float4(log16_f(q.x), log16_f(q.x >> 16), log16_f(q.y), log16_f(q.y >> 16));
    } else {
        return *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(b) + e);
    }
}
template <int MM>
__device__ __forceinline__ void v_st4(void* b, int64_t e, float4 x) {
    if constexpr (MM == MOM_16)
        *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(b) + e) =
            make_uint2((uint32_t)log16_q(x.x) | ((uint32_t)log16_q(x.y) << 16),
                       (uint32_t)log16_q(x.z) | ((uint32_t)log16_q(x.w) << 16));
    else
        *reinterpret_cast<float4*>(reinterpret_cast<float*>(b) + e) = x;
}

static inline hipStream_t as_stream(uint64_t s) { return reinterpret_cast<hipStream_t>(s); }
template <typename T> static inline T* as_ptr(uint64_t p) { return reinterpret_cast<T*>(p); }
