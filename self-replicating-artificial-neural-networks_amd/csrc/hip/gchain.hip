// Fused genotype-branch chain (gfx950 / CDNA4): Conv1D on the raw genotype -> Dense (1x1) ->
// optional BatchNormalization, forward and backward, with the chain's intermediate tensors never
// written to HBM.
//
// The genome grammar opens the replication branch with g_Conv1D / g_Dense / g_BN (layer_transitions.py:
// 9-23, 61-72), and ``g_layer = Conv1D(filters=F1, kernel_size=T, strides=S)(g_layer)`` followed by
// ``g_layer = Dense(units=F2, ...)(g_layer)`` and ``g_layer = BatchNormalization()(g_layer)`` is the
// replication branch of the example.json ancestor and of most of its descendants.  Its tensors are
// large and its FLOPs tiny: for B = 750 and a 96-position conv output, Conv1D(32) -> Dense(51) -> BN is
// 72000 rows x (32 + 51 + 51) channels, ~4.4 MFLOP per row-tile, and unfused it moved ~60 MB per
// organism per training step through seven launches (conv FWD, dense FWD, BN phases 0/2/4/5, dense
// DGRAD + WGRAD, conv WGRAD): 35 % of the bench population's step.  Here the chain is *recomputed*
// from the 100-bit genotype in every pass (2 + 4 MFMAs per 16 rows) and only the chain output y and
// its gradient dy touch HBM:
//
//   mode 0 FSTAT  recompute x = act2(W2 act1(W1 * g + b1) + b2); accumulate the BatchNorm statistics
//                 (shifted sums against row 0, the BN phase-0 workspace format) -- no stores
//   mode 1 FAPPLY recompute x; y = BN(x) (batch statistics in training, moving statistics in
//                 inference, identity without BN) -> the only HBM write; the training pass updates
//                 the moving statistics and saves mean / invstd
//   mode 2 BSTAT  recompute x; read dy; accumulate sum dy and sum dy * xhat (BN phase-4 workspace)
//   mode 3 BFULL  recompute Z1 = act1(W1 * g + b1) and x; read dy; dZ2 = BN_bwd(dy) * act2'(x) in
//                 registers; dW2 += Z1^T dZ2, db2 += sum dZ2, dZ1 = dZ2 W2 * act1'(Z1), dW1 += P^T dZ1
//                 (P = genotype patches), db1 += sum dZ1; one fixed-point atomic flush per block
//
// Determinism: the 4 waves of a block combine their partial sums in LDS in wave order
// (barrier-separated phases, no LDS float atomics) and blocks meet in the fixed-point workspaces and
// gradient arena of common.h (fxw_add / fx_add), so every pass is bitwise reproducible.
//
// MFMA orientation: the chain runs transposed, D1 = W1 * P^T ([F1][rows]) and D2 = W2 * Z1^T
// ([F2][rows]), so each accumulator tile holds 4 consecutive channels of one row per lane and feeds
// the next MFMA as its B operand without any data movement (the k order inside a 32-channel step is
// permuted: element j of lane group q is channel 32 s + 16 (j >> 2) + 4 q + (j & 3); the weight
// fragments are loaded in that order).  The weight-gradient products sum over rows, so their
// operands go through per-wave LDS images [32 rows][channels] read back with ds_read_b64_tr_b16.
//
// One block = 4 waves = one problem (organism) x a chunk of rpb rows.
#include "common.h"
#include "serann_hip.h"

// dZ2 / dZ1 as bf16 hi + lo pairs in the full backward (round 5): two extra MFMAs per 16 rows for ~16 bits of dZ
// in dW1 instead of 8 (compile-time: -DGC_HILO=0 builds the single-rounding form for A/B)
#ifndef GC_HILO
#define GC_HILO 1
#endif

#ifndef GC_BWD_MINW
#define GC_BWD_MINW 2       // waves per SIMD the backward kernels are register-budgeted for
#endif
#ifndef GC_UNROLL_H
#define GC_UNROLL_H 1       // unroll of the two 16-row halves of a backward super-tile
#endif
constexpr int kGcUnrollH = GC_UNROLL_H;

typedef __attribute__((ext_vector_type(8))) __bf16 gc_bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float gc_f32x4_t;
typedef __attribute__((ext_vector_type(4))) short gc_s16x4_t;

union GcFrag {
    gc_bf16x8_t v;
    bf16_t h[8];
    uint32_t u[4];
};

__device__ __forceinline__ bf16_t gc_bf(float v) { return __builtin_bit_cast(bf16_t, (__bf16)v); }
__device__ __forceinline__ gc_f32x4_t gc_mma(const GcFrag& a, const GcFrag& b, gc_f32x4_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
// channel of element j of a lane in 16-lane group q, for an operand assembled from accumulator tiles
// 2s and 2s + 1
__device__ __forceinline__ int gc_perm(int s, int q, int j) { return 32 * s + 16 * (j >> 2) + 4 * q + (j & 3); }

typedef float gc_f2 __attribute__((ext_vector_type(2)));    // packed fp32 (v_pk_* VALU)

// Activations resolved at compile time: A = ACT_LINEAR / ACT_RELU / ACT_SIGMOID, or GC_ACT_RT (-1) for
// a runtime code (activated Conv1D layers, which the generator's template never emits).
constexpr int GC_ACT_RT = -1;
template <int A>
__device__ __forceinline__ float gc_act(float x, int rt) {
    if constexpr (A == ACT_RELU) return __builtin_amdgcn_fmed3f(x, 0.f, 3.0e38f);     // one VALU op
    else if constexpr (A == ACT_SIGMOID) return __builtin_amdgcn_rcpf(1.f + __expf(-x));
    else if constexpr (A == GC_ACT_RT) return apply_act(x, rt);
    else return x;
}
// derivative through the activation output y
template <int A>
__device__ __forceinline__ float gc_dact(float y, int rt) {
    if constexpr (A == ACT_RELU) return y > 0.f ? 1.f : 0.f;
    else if constexpr (A == ACT_SIGMOID) return y * (1.f - y);
    else if constexpr (A == GC_ACT_RT) return act_grad_from_y(y, rt);
    else return 1.f;
}

typedef __attribute__((address_space(3))) const bf16_t* gc_lds_cptr;
// explicit LDS (address space 3) types: a generic pointer into LDS compiles to flat instructions,
// which also count on vmcnt, so an LDS wait would drain the prefetched global loads
typedef __attribute__((address_space(3))) bf16_t gc_lbf16;
typedef __attribute__((address_space(3))) float gc_lf32;
typedef __attribute__((address_space(3))) uint32_t gc_lu32;
typedef unsigned int gc_u32x2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) gc_u32x2 gc_lu32x2;

__device__ __forceinline__ float gc_wsum(int64_t ws, int C, int idx) {
    return fxw_sum<BN_WS_STRIPES>(reinterpret_cast<const long long*>(ws), C, idx);
}

// Transposed LDS read of a 16x16x32 operand fragment from an image [rows][ld]: lane (q, i) receives
// column c0 + i of rows 8q .. 8q + 7 (element j = row 8q + j).  EXEC must be all ones.
__device__ __forceinline__ void gc_tr_read(GcFrag& f, const __attribute__((address_space(3))) bf16_t* img, int ld, int c0,
                                           int lane) {
    const int q = lane >> 4, i = lane & 15;
    const int row = 8 * q + (i >> 2), col = c0 + 4 * (i & 3);
    const gc_s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) gc_s16x4_t*)(img + row * ld + col));
    const gc_s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) gc_s16x4_t*)(img + (row + 4) * ld + col));
    // vector shuffle + bit cast (an element-wise copy leaves v_bfi no-ops beside the MFMAs)
    typedef __attribute__((ext_vector_type(8))) short gc_s16x8_t;
    f.v = __builtin_bit_cast(gc_bf16x8_t, (gc_s16x8_t)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Global-memory accesses through address space 1: descriptor pointers are generic, and flat
// instructions would also count on lgkmcnt, so every LDS wait would drain the prefetched loads.
typedef unsigned int gc_u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) gc_u32x4 gc_gu32x4;
typedef __attribute__((address_space(1))) bf16_t gc_gbf16;
__device__ __forceinline__ gc_u32x4 gc_gld16(const bf16_t* p) { return *(const gc_gu32x4*)p; }
__device__ __forceinline__ void gc_gst16(bf16_t* p, gc_u32x4 v) { *(gc_gu32x4*)p = v; }

// Contiguous bf16 copy from a wave's LDS slot to global memory (16-B vectors when aligned).
__device__ __forceinline__ void gc_copy_out(bf16_t* __restrict__ dst, const __attribute__((address_space(3))) bf16_t* src,
                                            int n, int lane) {
    if ((n & 7) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
        for (int e = lane * 8; e < n; e += 512)
            gc_gst16(dst + e, *(const __attribute__((address_space(3))) gc_u32x4*)(src + e));
    } else {
        for (int e = lane; e < n; e += 64) *(gc_gbf16*)(dst + e) = src[e];
    }
}

// The chain's weights held in registers (constant over the block's rows); biases in LDS.
template <int F1K, int F2K>
struct GcNet {
    static constexpr int T1 = 2 * F1K, T2 = 2 * F2K;
    GcFrag w1[T1];            // stage-1 A: W1[ch = 16 mt + i][tap = 8 q + j]
    GcFrag w2[T2][F1K];       // stage-2 A: W2[o = 16 mt + i][in = gc_perm(s, q, j)]
    const gc_lf32* sb1;       // LDS [32 F1K] / [32 F2K] biases (0 past F1 / F2)
    const gc_lf32* sb2;

    __device__ __forceinline__ void load(const GChainDesc& d, int lane) {
        const int q = lane >> 4, c = lane & 15;
        const int T = (int)d.T, F1 = (int)d.F1, F2 = (int)d.F2;
        const bf16_t* __restrict__ W1 = reinterpret_cast<const bf16_t*>(d.w1);
        const bf16_t* __restrict__ W2 = reinterpret_cast<const bf16_t*>(d.w2);
        // fragments assembled as packed 32-bit words once, so the loop never re-packs 16-bit halves
#pragma unroll
        for (int mt = 0; mt < T1; ++mt) {
            const int ch = 16 * mt + c;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int t0 = 8 * q + 2 * k;
                const uint32_t lo = (ch < F1 && t0 < T) ? W1[ch * T + t0] : 0u;
                const uint32_t hi = (ch < F1 && t0 + 1 < T) ? W1[ch * T + t0 + 1] : 0u;
                w1[mt].u[k] = lo | (hi << 16);
            }
        }
#pragma unroll
        for (int mt = 0; mt < T2; ++mt) {
            const int o = 16 * mt + c;
#pragma unroll
            for (int s = 0; s < F1K; ++s)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int i0 = gc_perm(s, q, 2 * k), i1 = gc_perm(s, q, 2 * k + 1);
                    const uint32_t lo = (o < F2 && i0 < F1) ? W2[o * F1 + i0] : 0u;
                    const uint32_t hi = (o < F2 && i1 < F1) ? W2[o * F1 + i1] : 0u;
                    w2[mt][s].u[k] = lo | (hi << 16);
                }
        }
    }

    // Recompute one 16-row tile (rows r0 .. r0 + 15; this lane's row r0 + (lane & 15), clamped to
    // rlast): z1 = act1 output (fp32, accumulator layout), zb = its bf16 B fragments, x = act2 output.
    // The genotype comes from ``src`` = the block's staged rows (LDS, first batch row b0) or global
    // memory (b0 = 0).
    template <int A1, int A2, typename GPtr>
    __device__ __forceinline__ void tile(const GChainDesc& d, GPtr src, int b0, int r0, int rlast, int lane,
                                         gc_f32x4_t (&z1)[T1], GcFrag (&zb)[F1K], gc_f32x4_t (&x)[T2]) const {
        const int q = lane >> 4;
        const int L1 = (int)d.L1, T = (int)d.T, L0 = (int)d.L0, S = (int)d.S;
        const int row = min(r0 + (lane & 15), rlast);
        const int b = (int)((__umulhi((uint32_t)row, (uint32_t)d.dvL1) + (uint32_t)row) >> (uint32_t)(d.dvL1 >> 32));
        const int p = row - b * L1;
        const GPtr g = src + ((b - b0) * L0 + p * S);
        GcFrag pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int tap = 8 * q + j;
            pb.h[j] = tap < T ? g[tap] : (bf16_t)0;
        }
        const int act1 = (int)d.act1, act2 = (int)d.act2;
        // the bias is the accumulator's initial value
#pragma unroll
        for (int mt = 0; mt < T1; ++mt) {
            gc_f32x4_t a = gc_mma(w1[mt], pb, *(const __attribute__((address_space(3))) gc_f32x4_t*)(sb1 + 16 * mt + 4 * q));
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = gc_act<A1>(a[r], act1);
            z1[mt] = a;
        }
#pragma unroll
        for (int s = 0; s < F1K; ++s)
#pragma unroll
            for (int j = 0; j < 8; ++j) zb[s].h[j] = gc_bf(z1[2 * s + (j >> 2)][j & 3]);
#pragma unroll
        for (int mt = 0; mt < T2; ++mt) {
            gc_f32x4_t a = *(const __attribute__((address_space(3))) gc_f32x4_t*)(sb2 + 16 * mt + 4 * q);
#pragma unroll
            for (int s = 0; s < F1K; ++s) a = gc_mma(w2[mt][s], zb[s], a);
#pragma unroll
            for (int r = 0; r < 4; ++r) a[r] = gc_act<A2>(a[r], act2);
            x[mt] = a;
        }
    }
};

// Block prologue shared by every mode: biases into LDS, the genotype rows of the block's batch
// elements into LDS (the host sizes rpb so they fit in GC_GMAX elements).
constexpr int GC_GMAX = 8192;

template <int F1K, int F2K>
__device__ __forceinline__ void gc_prologue(const GChainDesc& d, int R0, int R1, gc_lf32* sb1, gc_lf32* sb2, gc_lbf16* sG,
                                            int& b0) {
    const int F1 = (int)d.F1, F2 = (int)d.F2, L1 = (int)d.L1, L0 = (int)d.L0;
    const float* B1 = reinterpret_cast<const float*>(d.b1);
    const float* B2 = reinterpret_cast<const float*>(d.b2);
    for (int c = threadIdx.x; c < 32 * F1K; c += 256) sb1[c] = (B1 != nullptr && c < F1) ? B1[c] : 0.f;
    for (int c = threadIdx.x; c < 32 * F2K; c += 256) sb2[c] = (B2 != nullptr && c < F2) ? B2[c] : 0.f;
    b0 = R0 / L1;
    const int b1 = (R1 - 1) / L1;
    const int n = min((b1 - b0 + 1) * L0, GC_GMAX);   // (hip_ops.gchain_rpb keeps it in range)
    const bf16_t* g = reinterpret_cast<const bf16_t*>(d.g) + (int64_t)b0 * L0;
    // 8 loads in flight per thread before their LDS stores (a load-wait-store loop would pay the
    // global latency once per element)
    if ((L0 & 1) == 0 && (reinterpret_cast<uintptr_t>(g) & 3) == 0) {
        const __attribute__((address_space(1))) uint32_t* g32 = (const __attribute__((address_space(1))) uint32_t*)g;
        gc_lu32* s32 = (gc_lu32*)sG;
        const int n2 = n >> 1;
        for (int e0 = threadIdx.x; e0 < n2; e0 += 256 * 8) {
            uint32_t v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = e0 + 256 * k < n2 ? g32[e0 + 256 * k] : 0u;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (e0 + 256 * k < n2) s32[e0 + 256 * k] = v[k];
        }
    } else {
        const gc_gbf16* g16 = (const gc_gbf16*)g;
        for (int e0 = threadIdx.x; e0 < n; e0 += 256 * 8) {
            bf16_t v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = e0 + 256 * k < n ? g16[e0 + 256 * k] : (bf16_t)0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (e0 + 256 * k < n) sG[e0 + 256 * k] = v[k];
        }
    }
}

__device__ __forceinline__ void gc_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Sum a per-lane value over the 16 lanes of its group (the 16 rows of a tile): the group's lane 0
// ends with the total.
__device__ __forceinline__ float gc_rowsum(float v) {
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    v += __shfl_xor(v, 4, 64);
    v += __shfl_xor(v, 8, 64);
    return v;
}

// ------------------------------------------------------------------------------------------------
// forward: MODE 0 statistics, MODE 1 output
template <int F1K, int F2K, int MODE, int A1, int A2>
__global__ __launch_bounds__(256) void gchain_fwd_kernel(const GChainDesc* __restrict__ descs,
                                                         const int2* __restrict__ tiles) {
    using Net = GcNet<F1K, F2K>;
    constexpr int T1 = Net::T1, T2 = Net::T2, F2P = 32 * F2K;
    __shared__ __attribute__((aligned(16))) bf16_t sG[GC_GMAX];
    __shared__ __attribute__((aligned(16))) bf16_t sOut[MODE == 1 ? 4 * 16 * F2P : 8];
    __shared__ __attribute__((aligned(16))) float sPar[3][F2P];
    __shared__ __attribute__((aligned(16))) float sB1[32 * F1K], sB2[F2P];
    const int2 td = tiles[blockIdx.x];
    const GChainDesc& d = descs[td.x];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4;
    const int R = (int)(d.B * d.L1), F2 = (int)d.F2, C = F2;
    const int R0 = td.y * (int)d.rpb, R1 = min(R, R0 + (int)d.rpb);
    const int flags = (int)d.flags;
    const bool bn = (flags & GC_BN) != 0, train = (flags & GC_TRAIN) != 0;
    const float Rf = (float)R;
    Net net;
    net.sb1 = (const gc_lf32*)sB1;
    net.sb2 = (const gc_lf32*)sB2;
    net.load(d, lane);
    int b0;
    gc_prologue<F1K, F2K>(d, R0, R1, (gc_lf32*)sB1, (gc_lf32*)sB2, (gc_lbf16*)sG, b0);
    for (int e = threadIdx.x; e < 3 * F2P; e += 256) (&sPar[0][0])[e] = 0.f;
    __syncthreads();
    gc_f32x4_t z1[T1], x[T2];
    GcFrag zb[F1K];
    gc_f32x4_t ka[T2], kb[T2];        // MODE 0: shift K; MODE 1: scale, shift
    if (MODE == 0 || (bn && train)) {
        // row 0 of the problem (global memory): the statistics shift K_c (BN phase 0 uses x[0][c])
        net.template tile<A1, A2>(d, (const gc_gbf16*)d.g, 0, 0, R - 1, lane, z1, zb, x);
#pragma unroll
        for (int mt = 0; mt < T2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) ka[mt][r] = __shfl(x[mt][r], lane & 48, 64);
    }
    if (MODE == 1) {
        if (bn) {
            if (train && wave == 0 && (lane & 15) == 0) {
#pragma unroll
                for (int mt = 0; mt < T2; ++mt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) sPar[2][16 * mt + 4 * q + r] = ka[mt][r];
            }
            __syncthreads();
            const float eps = (float)d.eps, mom = (float)d.momentum;
            float* mm = reinterpret_cast<float*>(d.mm);
            float* mv = reinterpret_cast<float*>(d.mv);
            for (int c = threadIdx.x; c < F2; c += 256) {
                float mu, var;
                if (train) {
                    const float m1 = gc_wsum(d.ws, C, c) / Rf;
                    mu = sPar[2][c] + m1;
                    var = fmaxf(gc_wsum(d.ws, C, C + c) / Rf - m1 * m1, 0.f);
                } else {
                    mu = mm[c];
                    var = mv[c];
                }
                const float is = rsqrtf(var + eps);
                const float gsc = (flags & GC_GAMMA) ? reinterpret_cast<const float*>(d.gamma)[c] * is : is;
                const float sh = ((flags & GC_BETA) ? reinterpret_cast<const float*>(d.beta)[c] : 0.f) - mu * gsc;
                if (train && td.y == 0) {
                    // moving averages (unbiased variance factor n / (n - (1 + eps)),
                    // BatchNormalizationF16.py:134-148) and the saved statistics, once per problem
                    mm[c] = mm[c] * mom + mu * (1.f - mom);
                    mv[c] = mv[c] * mom + var * (Rf / (Rf - (1.f + eps))) * (1.f - mom);
                    reinterpret_cast<float*>(d.mean)[c] = mu;
                    reinterpret_cast<float*>(d.invstd)[c] = is;
                }
                sPar[0][c] = gsc;
                sPar[1][c] = sh;
            }
            __syncthreads();
#pragma unroll
            for (int mt = 0; mt < T2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int ch = 16 * mt + 4 * q + r;
                    ka[mt][r] = sPar[0][ch];
                    kb[mt][r] = sPar[1][ch];
                }
        } else {
#pragma unroll
            for (int mt = 0; mt < T2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) { ka[mt][r] = 1.f; kb[mt][r] = 0.f; }
        }
    }
    gc_f2 s1[T2][2], s2[T2][2];
#pragma unroll
    for (int mt = 0; mt < T2; ++mt)
#pragma unroll
        for (int h = 0; h < 2; ++h) { s1[mt][h] = gc_f2{0.f, 0.f}; s2[mt][h] = gc_f2{0.f, 0.f}; }

    // 16-row tiles, interleaved over the waves; every wave only touches its own LDS output slot
    const int ntile = (R1 - R0 + 15) >> 4;
    gc_lbf16* out = (gc_lbf16*)sOut + wave * 16 * F2P;
    bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(d.y);
    for (int ti = wave; ti < ntile; ti += 4) {
        const int r0 = R0 + 16 * ti;
        net.template tile<A1, A2>(d, (gc_lds_cptr)sG, b0, r0, R1 - 1, lane, z1, zb, x);
        const bool valid = r0 + (lane & 15) < R1;
        if (MODE == 0) {
            if (valid) {
#pragma unroll
                for (int mt = 0; mt < T2; ++mt)
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const gc_f2 v = gc_f2{x[mt][2 * h], x[mt][2 * h + 1]} - gc_f2{ka[mt][2 * h], ka[mt][2 * h + 1]};
                        s1[mt][h] += v;
                        s2[mt][h] += v * v;
                    }
            }
        } else {
            gc_wave_sync();                       // the previous copy has read the slot
            if (valid) {
#pragma unroll
                for (int mt = 0; mt < T2; ++mt) {
                    const gc_f32x4_t yv = x[mt] * ka[mt] + kb[mt];
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int ch = 16 * mt + 4 * q + r;
                        if (ch < F2) out[(lane & 15) * F2 + ch] = gc_bf(yv[r]);
                    }
                }
            }
            gc_wave_sync();
            gc_copy_out(y + (int64_t)r0 * F2, out, min(16, R1 - r0) * F2, lane);
        }
    }
    if (MODE == 0) {
        // rows of a lane group -> the group's lane 0; waves -> LDS in wave order; one fixed-point
        // atomic per channel and block
        float ra[T2][4], rb[T2][4];
#pragma unroll
        for (int mt = 0; mt < T2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                ra[mt][r] = gc_rowsum(s1[mt][r >> 1][r & 1]);
                rb[mt][r] = gc_rowsum(s2[mt][r >> 1][r & 1]);
            }
        for (int w = 0; w < 4; ++w) {
            if (wave == w && (lane & 15) == 0) {
#pragma unroll
                for (int mt = 0; mt < T2; ++mt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int ch = 16 * mt + 4 * q + r;
                        if (ch < F2) {
                            sPar[0][ch] += ra[mt][r];
                            sPar[1][ch] += rb[mt][r];
                        }
                    }
            }
            __syncthreads();
        }
        long long* wsw = reinterpret_cast<long long*>(d.ws) + (blockIdx.x % BN_WS_STRIPES) * 4 * C;
        for (int c = threadIdx.x; c < F2; c += 256) {
            fxw_add(wsw + 2 * c, sPar[0][c]);
            fxw_add(wsw + 2 * (C + c), sPar[1][c]);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// backward: MODE 2 BatchNorm gradient statistics, MODE 3 full backward.  Both walk 32-row super-tiles
// per wave with the next super-tile's dy prefetched into registers (16-B loads) while the current
// one is computed.
template <int F1K, int F2K, int MODE>
struct GcBwdLds {
    static constexpr int T1 = 2 * F1K, T2 = 2 * F2K, F1P = 32 * F1K, F2P = 32 * F2K;
    static constexpr int LD1 = F1P + 4, LD2 = F2P + 4;          // image row strides (8-B aligned rows)
    static constexpr int DY = 32 * F2P;                          // staged dy rows [32][F2]
    // MODE 2 stages dy only; MODE 3 also the Z1 / dZ1 / dZ2 images
    // (+ the dZ1 low-part image: dW1 takes dZ1 as hi + lo bf16 pairs, below)
    static constexpr int PER_WAVE = MODE == 2 ? DY : DY + (GC_HILO ? 3 : 2) * 32 * LD1 + 32 * LD2;
    // fp32 reduction slots after the loop (alias the per-wave regions)
    static constexpr int RED = MODE == 2 ? 2 * F2P : F2P * F1P + F1P * 16 + F1P + F2P;
    static constexpr int TOTAL = 4 * PER_WAVE > 2 * RED ? 4 * PER_WAVE : 2 * RED;
    static constexpr int NV = F2P / 16;                          // 16-B dy chunks per lane per super-tile
};

template <int NV>
struct GcDyPre {
    gc_u32x4 v[NV];
    // rows [base, base + nr) of dy ([R][F2] bf16, 16-B aligned at a 32-row boundary): the full 16-B
    // chunks into registers.  Unconditional loads (a chunk past the rows re-reads chunk 0; a super-tile
    // of fewer than 8 elements reads at most 7 past its end, inside the 16-element-aligned arena) keep
    // v[] in registers.
    __device__ __forceinline__ void load(const bf16_t* __restrict__ dy, int base, int nr, int F2, int lane) {
        const int n = nr * F2;
        const bf16_t* src = dy + (int64_t)base * F2;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int e = (lane + 64 * k) * 8;
            v[k] = gc_gld16(src + (e + 8 <= n ? e : 0));
        }
    }
    // ... into the wave's LDS slot, plus the tail of a partial last super-tile straight from memory
    __device__ __forceinline__ void store(gc_lbf16* dst, const bf16_t* __restrict__ dy, int base, int nr, int F2,
                                          int lane) const {
        const int n = nr * F2;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int e = (lane + 64 * k) * 8;
            if (e + 8 <= n) *(__attribute__((address_space(3))) gc_u32x4*)(dst + e) = v[k];
        }
        for (int e = (n & ~7) + lane; e < n; e += 64) dst[e] = *(const gc_gbf16*)(dy + (int64_t)base * F2 + e);
    }
};

template <int F1K, int F2K, int MODE, int A1, int A2>
__global__ __launch_bounds__(256, GC_BWD_MINW) void gchain_bwd_kernel(const GChainDesc* __restrict__ descs,
                                                         const int2* __restrict__ tiles) {
    using Net = GcNet<F1K, F2K>;
    using Lds = GcBwdLds<F1K, F2K, MODE>;
    constexpr int T1 = Net::T1, T2 = Net::T2, F1P = Lds::F1P, F2P = Lds::F2P;
    constexpr int LD1 = Lds::LD1, LD2 = Lds::LD2;
    __shared__ __attribute__((aligned(16))) bf16_t sMem[Lds::TOTAL];
    __shared__ __attribute__((aligned(16))) bf16_t sG[GC_GMAX];
    __shared__ __attribute__((aligned(16))) float sK[3][F2P];
    __shared__ __attribute__((aligned(16))) float sB1[F1P], sB2[F2P];
    const int2 td = tiles[blockIdx.x];
    const GChainDesc& d = descs[td.x];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4;
    const int R = (int)(d.B * d.L1), F1 = (int)d.F1, F2 = (int)d.F2, C = F2;
    const int T = (int)d.T, L1 = (int)d.L1, L0 = (int)d.L0, S = (int)d.S;
    const int R0 = td.y * (int)d.rpb, R1 = min(R, R0 + (int)d.rpb);
    const int flags = (int)d.flags;
    const bool bn = (flags & GC_BN) != 0;
    const float Rf = (float)R;
    const bf16_t* __restrict__ dy = reinterpret_cast<const bf16_t*>(d.dy);
    const bf16_t* __restrict__ W2 = reinterpret_cast<const bf16_t*>(d.w2);

    gc_lbf16* sDy = (gc_lbf16*)sMem + wave * Lds::PER_WAVE;
    gc_lbf16* imgZ1 = sDy + Lds::DY;               // (MODE 3 only)
    gc_lbf16* imgDZ1 = imgZ1 + 32 * LD1;
    gc_lbf16* imgDZ2 = imgDZ1 + 32 * LD1;
    gc_lbf16* imgDZ1lo = imgDZ2 + 32 * LD2;        // dZ1 - bf16(dZ1), bf16 (MODE 3)

    // super-tiles of this wave: st = wave, wave + 4, ...; the first one's dy is requested first
    const int nst = (R1 - R0 + 31) >> 5;
    GcDyPre<Lds::NV> pre;
    if (wave < nst) pre.load(dy, R0 + 32 * wave, min(32, R1 - R0 - 32 * wave), F2, lane);

    Net net;
    net.sb1 = (const gc_lf32*)sB1;
    net.sb2 = (const gc_lf32*)sB2;
    net.load(d, lane);
    int b0;
    gc_prologue<F1K, F2K>(d, R0, R1, (gc_lf32*)sB1, (gc_lf32*)sB2, (gc_lbf16*)sG, b0);

    // per-channel constants: MODE 2 (mean, invstd); MODE 3 dx = k1 dy + k2 x + k3
    for (int e = threadIdx.x; e < 3 * F2P; e += 256) (&sK[0][0])[e] = 0.f;
    __syncthreads();
    for (int c = threadIdx.x; c < F2; c += 256) {
        if (MODE == 2) {                              // xhat = x * is + (-mu * is)
            const float is = reinterpret_cast<const float*>(d.invstd)[c];
            sK[0][c] = is;
            sK[1][c] = -reinterpret_cast<const float*>(d.mean)[c] * is;
        } else if (bn) {
            const float mu = reinterpret_cast<const float*>(d.mean)[c];
            const float is = reinterpret_cast<const float*>(d.invstd)[c];
            const float gg = ((flags & GC_GAMMA) ? reinterpret_cast<const float*>(d.gamma)[c] : 1.f) * is;
            const float sdy = gc_wsum(d.wsb, C, c), sdyx = gc_wsum(d.wsb, C, C + c);
            const float ma = sdy / Rf, mb = sdyx / Rf;
            sK[0][c] = gg;
            sK[1][c] = -gg * is * mb;
            sK[2][c] = -gg * (ma - mu * is * mb);
            if (td.y == 0) {
                if (flags & GC_GAMMA) reinterpret_cast<long long*>(d.dgamma)[c] += fx_q(sdyx);
                if (flags & GC_BETA) reinterpret_cast<long long*>(d.dbeta)[c] += fx_q(sdy);
            }
        } else {
            sK[0][c] = 1.f;
        }
    }
    __syncthreads();

    gc_f32x4_t z1[T1], x[T2];
    GcFrag zb[F1K];
    const int act1 = (int)d.act1, act2 = (int)d.act2;

    gc_f32x4_t s1[T2], s2[T2];            // MODE 2 sums; MODE 3: bias-gradient partials db2 (s1)
    gc_f32x4_t db1p[T1];
#pragma unroll
    for (int mt = 0; mt < T2; ++mt) { s1[mt] = gc_f32x4_t{0.f, 0.f, 0.f, 0.f}; s2[mt] = s1[mt]; }
#pragma unroll
    for (int mt = 0; mt < T1; ++mt) db1p[mt] = gc_f32x4_t{0.f, 0.f, 0.f, 0.f};
    // MODE 3: dZ1^T = W2^T dZ2^T, A = W2[o = gc_perm(s, q, j)][i = 16 mt + (lane & 15)]
    GcFrag w2t[MODE == 3 ? T1 : 1][F2K];
    if (MODE == 3) {
#pragma unroll
        for (int mt = 0; mt < T1; ++mt) {
            const int i = 16 * mt + (lane & 15);
#pragma unroll
            for (int s = 0; s < F2K; ++s)
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int o0 = gc_perm(s, q, 2 * k), o1 = gc_perm(s, q, 2 * k + 1);
                    const uint32_t lo = (i < F1 && o0 < F2) ? W2[o0 * F1 + i] : 0u;
                    const uint32_t hi = (i < F1 && o1 < F2) ? W2[o1 * F1 + i] : 0u;
                    w2t[mt][s].u[k] = lo | (hi << 16);
                }
        }
    }
    gc_f32x4_t dw2[MODE == 3 ? T2 : 1][T1], dw1[T1];
#pragma unroll
    for (int a = 0; a < (MODE == 3 ? T2 : 1); ++a)
#pragma unroll
        for (int b = 0; b < T1; ++b) dw2[a][b] = gc_f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int b = 0; b < T1; ++b) dw1[b] = gc_f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int st = wave; st < nst; st += 4) {
        const int base = R0 + 32 * st;
        const int nr = min(32, R1 - base);
        gc_wave_sync();                           // the previous super-tile's LDS reads are done
        pre.store(sDy, dy, base, nr, F2, lane);
        if (st + 4 < nst) pre.load(dy, base + 128, min(32, R1 - base - 128), F2, lane);
        gc_wave_sync();
#pragma unroll kGcUnrollH
        for (int h = 0; h < 2; ++h) {
            const int r0 = base + 16 * h;
            net.template tile<A1, A2>(d, (gc_lds_cptr)sG, b0, r0, R1 - 1, lane, z1, zb, x);
            const int lr = 16 * h + (lane & 15);        // row inside the super-tile
            const bool valid = lr < nr;
            if (MODE == 2) {
                if (valid) {
#pragma unroll
                    for (int mt = 0; mt < T2; ++mt) {
                        const int c0 = 16 * mt + 4 * q;
                        const gc_f32x4_t is = *reinterpret_cast<const gc_f32x4_t*>(&sK[0][c0]);
                        const gc_f32x4_t nm = *reinterpret_cast<const gc_f32x4_t*>(&sK[1][c0]);
                        gc_f32x4_t gv;
#pragma unroll
                        for (int r = 0; r < 4; ++r) gv[r] = c0 + r < F2 ? bf2f(sDy[lr * F2 + c0 + r]) : 0.f;
                        s1[mt] += gv;
                        s2[mt] += gv * (x[mt] * is + nm);
                    }
                }
                continue;
            }
            gc_f32x4_t dz2[T2];
#pragma unroll
            for (int mt = 0; mt < T2; ++mt) {
                const int c0 = 16 * mt + 4 * q;
                const gc_f32x4_t k1 = *reinterpret_cast<const gc_f32x4_t*>(&sK[0][c0]);
                const gc_f32x4_t k2 = *reinterpret_cast<const gc_f32x4_t*>(&sK[1][c0]);
                const gc_f32x4_t k3 = *reinterpret_cast<const gc_f32x4_t*>(&sK[2][c0]);
                gc_f32x4_t gv;
#pragma unroll
                for (int r = 0; r < 4; ++r) gv[r] = (valid && c0 + r < F2) ? bf2f(sDy[lr * F2 + c0 + r]) : 0.f;
                gc_f32x4_t v = k1 * gv + (k2 * x[mt] + k3);   // zero past F2 (k = 0)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    float e = v[r];
                    if constexpr (A2 == ACT_RELU) e = (valid && x[mt][r] > 0.f) ? e : 0.f;
                    else e = valid ? e * gc_dact<A2>(x[mt][r], act2) : 0.f;
                    v[r] = e;
                }
                dz2[mt] = v;
                s1[mt] += v;
            }
            // dZ2 as a pair of bf16 operands, hi + lo (lo = dZ2 - hi): dZ1 = W2^T dZ2 then carries ~16 bits of
            // dZ2 instead of 8.  dW1 = sum over rows of dZ1 x genotype is a heavily cancelling sum (BN makes
            // sum_rows dZ2 = 0): with one bf16 rounding of dZ2 and one of dZ1 it was 3x torch-bf16's error on
            // the first Conv1D kernel at B = 96 (profiles/r4/diag_bf16_margin.txt).  Two extra MFMAs per 16 rows.
            GcFrag dzb[F2K], dzl[F2K];
#pragma unroll
            for (int s = 0; s < F2K; ++s)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float e = dz2[2 * s + (j >> 2)][j & 3];
                    dzb[s].h[j] = gc_bf(e);
                    if (GC_HILO) dzl[s].h[j] = gc_bf(e - bf2f(dzb[s].h[j]));
                }
            // images: rows lr, channels 16 mt + 4 q .. + 3 (8-B stores)
#pragma unroll
            for (int mt = 0; mt < T2; ++mt) {
                gc_u32x2 v;
                v.x = (uint32_t)gc_bf(dz2[mt][0]) | ((uint32_t)gc_bf(dz2[mt][1]) << 16);
                v.y = (uint32_t)gc_bf(dz2[mt][2]) | ((uint32_t)gc_bf(dz2[mt][3]) << 16);
                *(gc_lu32x2*)(&imgDZ2[lr * LD2 + 16 * mt + 4 * q]) = v;
            }
#pragma unroll
            for (int mt = 0; mt < T1; ++mt) {
                gc_u32x2 v;
                v.x = (uint32_t)gc_bf(z1[mt][0]) | ((uint32_t)gc_bf(z1[mt][1]) << 16);
                v.y = (uint32_t)gc_bf(z1[mt][2]) | ((uint32_t)gc_bf(z1[mt][3]) << 16);
                *(gc_lu32x2*)(&imgZ1[lr * LD1 + 16 * mt + 4 * q]) = v;
            }
            // dZ1^T = W2^T dZ2^T, times act1'(Z1)
#pragma unroll
            for (int mt = 0; mt < T1; ++mt) {
                gc_f32x4_t v = gc_f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < F2K; ++s) if (GC_HILO) v = gc_mma(w2t[mt][s], dzl[s], v);
#pragma unroll
                for (int s = 0; s < F2K; ++s) v = gc_mma(w2t[mt][s], dzb[s], v);
                if constexpr (A1 != ACT_LINEAR) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[r] *= gc_dact<A1>(z1[mt][r], act1);
                }
                db1p[mt] += v;
                bf16_t hb[4], lb[4];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    hb[r] = gc_bf(v[r]);
                    lb[r] = gc_bf(v[r] - bf2f(hb[r]));
                }
                gc_u32x2 u;
                u.x = (uint32_t)hb[0] | ((uint32_t)hb[1] << 16);
                u.y = (uint32_t)hb[2] | ((uint32_t)hb[3] << 16);
                *(gc_lu32x2*)(&imgDZ1[lr * LD1 + 16 * mt + 4 * q]) = u;
                u.x = (uint32_t)lb[0] | ((uint32_t)lb[1] << 16);
                u.y = (uint32_t)lb[2] | ((uint32_t)lb[3] << 16);
                if (GC_HILO) *(gc_lu32x2*)(&imgDZ1lo[lr * LD1 + 16 * mt + 4 * q]) = u;
            }
        }
        if (MODE == 2) continue;
        gc_wave_sync();
        // weight gradients over the super-tile's 32 rows
        GcFrag bz[T1];
#pragma unroll
        for (int mt = 0; mt < T1; ++mt) gc_tr_read(bz[mt], imgZ1, LD1, 16 * mt, lane);
#pragma unroll
        for (int m2 = 0; m2 < T2; ++m2) {
            GcFrag a2;
            gc_tr_read(a2, imgDZ2, LD2, 16 * m2, lane);
#pragma unroll
            for (int m1 = 0; m1 < T1; ++m1) dw2[m2][m1] = gc_mma(a2, bz[m1], dw2[m2][m1]);
        }
        // dW1: B = genotype patches P[row = 8 q + j][tap = lane & 15] from the staged rows
        GcFrag pp;
        {
            const int tap = lane & 15;
            int row = min(base + 8 * q, R1 - 1);
            int b = row / L1, p = row - b * L1;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const bool ok = base + 8 * q + j < R1 && tap < T;
                pp.h[j] = ok ? ((gc_lds_cptr)sG)[(b - b0) * L0 + p * S + tap] : (bf16_t)0;
                if (++p == L1) { p = 0; ++b; }
            }
        }
#pragma unroll
        for (int m1 = 0; m1 < T1; ++m1) {
            GcFrag a1, a1l;
            gc_tr_read(a1, imgDZ1, LD1, 16 * m1, lane);
            if (GC_HILO) {
                gc_tr_read(a1l, imgDZ1lo, LD1, 16 * m1, lane);
                dw1[m1] = gc_mma(a1l, pp, dw1[m1]);
            }
            dw1[m1] = gc_mma(a1, pp, dw1[m1]);
        }
    }
    // ---- flush: waves -> LDS in wave order (the images are dead), one fixed-point atomic per element
    // and block ----
    __syncthreads();
    gc_lf32* red = (gc_lf32*)sMem;
    if (MODE == 2) {
        for (int e = threadIdx.x; e < 2 * F2P; e += 256) red[e] = 0.f;
        float ra[T2][4], rb[T2][4];
#pragma unroll
        for (int mt = 0; mt < T2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                ra[mt][r] = gc_rowsum(s1[mt][r]);
                rb[mt][r] = gc_rowsum(s2[mt][r]);
            }
        __syncthreads();
        for (int w = 0; w < 4; ++w) {
            if (wave == w && (lane & 15) == 0) {
#pragma unroll
                for (int mt = 0; mt < T2; ++mt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int ch = 16 * mt + 4 * q + r;
                        if (ch < F2) {
                            red[ch] += ra[mt][r];
                            red[F2P + ch] += rb[mt][r];
                        }
                    }
            }
            __syncthreads();
        }
        long long* wsw = reinterpret_cast<long long*>(d.wsb) + (blockIdx.x % BN_WS_STRIPES) * 4 * C;
        for (int c = threadIdx.x; c < F2; c += 256) {
            fxw_add(wsw + 2 * c, red[c]);
            fxw_add(wsw + 2 * (C + c), red[F2P + c]);
        }
        return;
    }
    gc_lf32* red1 = red + F2P * F1P;
    gc_lf32* redb1 = red1 + F1P * 16;
    gc_lf32* redb2 = redb1 + F1P;
    for (int e = threadIdx.x; e < Lds::RED; e += 256) red[e] = 0.f;
    __syncthreads();
    // every lane of a wave owns distinct LDS elements; the waves add in order 0..3 (the branch is
    // wave-uniform, so the row-sum shuffles inside it are well defined)
    for (int w = 0; w < 4; ++w) {
        if (wave == w) {
#pragma unroll
            for (int m2 = 0; m2 < (MODE == 3 ? T2 : 1); ++m2)
#pragma unroll
                for (int m1 = 0; m1 < T1; ++m1)
#pragma unroll
                    for (int r = 0; r < 4; ++r) red[(16 * m2 + 4 * q + r) * F1P + 16 * m1 + (lane & 15)] += dw2[m2][m1][r];
#pragma unroll
            for (int m1 = 0; m1 < T1; ++m1)
#pragma unroll
                for (int r = 0; r < 4; ++r) red1[(16 * m1 + 4 * q + r) * 16 + (lane & 15)] += dw1[m1][r];
#pragma unroll
            for (int mt = 0; mt < T1; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = gc_rowsum(db1p[mt][r]);
                    if ((lane & 15) == 0) redb1[16 * mt + 4 * q + r] += v;
                }
#pragma unroll
            for (int mt = 0; mt < T2; ++mt)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const float v = gc_rowsum(s1[mt][r]);
                    if ((lane & 15) == 0) redb2[16 * mt + 4 * q + r] += v;
                }
        }
        __syncthreads();
    }
    long long* gw2 = reinterpret_cast<long long*>(d.dw2);     // Q40 gradient arena (common.h)
    long long* gw1 = reinterpret_cast<long long*>(d.dw1);
    long long* gb1 = reinterpret_cast<long long*>(d.db1);
    long long* gb2 = reinterpret_cast<long long*>(d.db2);
    for (int e = threadIdx.x; e < F2 * F1; e += 256) {
        const int o = e / F1, i = e - o * F1;
        fx_add(&gw2[e], red[o * F1P + i]);
    }
    for (int e = threadIdx.x; e < F1 * T; e += 256) {
        const int i = e / T, t = e - i * T;
        fx_add(&gw1[e], red1[i * 16 + t]);
    }
    if (gb1 != nullptr)
        for (int c = threadIdx.x; c < F1; c += 256) fx_add(&gb1[c], redb1[c]);
    if (gb2 != nullptr)
        for (int c = threadIdx.x; c < F2; c += 256) fx_add(&gb2[c], redb2[c]);
}

// ------------------------------------------------------------------------------------------------
// Host-side limits mirrored in hip_ops.gchain_variant: T <= 16 taps, (F1K, F2K) in {1} x {1..4} or
// {2} x {1, 2} (F1 <= 32 with F2 <= 128, or F1 <= 64 with F2 <= 64).  variant = F1K * 8 + F2K.
template <int F1K, int F2K, int A1, int A2>
static void launch_gchain_a(int mode, dim3 grid, hipStream_t s, const GChainDesc* dp, const int2* tp) {
    const dim3 block(256);
    switch (mode) {
        case 0: hipLaunchKernelGGL((gchain_fwd_kernel<F1K, F2K, 0, A1, A2>), grid, block, 0, s, dp, tp); break;
        case 1: hipLaunchKernelGGL((gchain_fwd_kernel<F1K, F2K, 1, A1, A2>), grid, block, 0, s, dp, tp); break;
        case 2: hipLaunchKernelGGL((gchain_bwd_kernel<F1K, F2K, 2, A1, A2>), grid, block, 0, s, dp, tp); break;
        case 3: hipLaunchKernelGGL((gchain_bwd_kernel<F1K, F2K, 3, A1, A2>), grid, block, 0, s, dp, tp); break;
        default: throw std::runtime_error("gchain: bad mode");
    }
}

// acts = 3 * (Conv1D activated) + Dense activation code
template <int F1K, int F2K>
static void launch_gchain_v(int mode, int acts, dim3 grid, hipStream_t s, const GChainDesc* dp, const int2* tp) {
    switch (acts) {
        case 0: launch_gchain_a<F1K, F2K, ACT_LINEAR, ACT_LINEAR>(mode, grid, s, dp, tp); break;
        case 1: launch_gchain_a<F1K, F2K, ACT_LINEAR, ACT_RELU>(mode, grid, s, dp, tp); break;
        case 2: launch_gchain_a<F1K, F2K, ACT_LINEAR, ACT_SIGMOID>(mode, grid, s, dp, tp); break;
        case 3: launch_gchain_a<F1K, F2K, GC_ACT_RT, ACT_LINEAR>(mode, grid, s, dp, tp); break;
        case 4: launch_gchain_a<F1K, F2K, GC_ACT_RT, ACT_RELU>(mode, grid, s, dp, tp); break;
        case 5: launch_gchain_a<F1K, F2K, GC_ACT_RT, ACT_SIGMOID>(mode, grid, s, dp, tp); break;
        default: throw std::runtime_error("gchain: bad activation code");
    }
}

// variant = acts * 64 + F1K * 8 + F2K (hip_ops.gchain_variant + the activation code of the descriptors)
void launch_gchain(int mode, int variant, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    const dim3 grid((unsigned)ntiles);
    const GChainDesc* dp = as_ptr<const GChainDesc>(descs);
    const int2* tp = as_ptr<const int2>(tiles);
    hipStream_t s = as_stream(stream);
    const int acts = variant >> 6;
    switch (variant & 63) {
        case 9: launch_gchain_v<1, 1>(mode, acts, grid, s, dp, tp); break;
        case 10: launch_gchain_v<1, 2>(mode, acts, grid, s, dp, tp); break;
        case 11: launch_gchain_v<1, 3>(mode, acts, grid, s, dp, tp); break;
        case 12: launch_gchain_v<1, 4>(mode, acts, grid, s, dp, tp); break;
        case 17: launch_gchain_v<2, 1>(mode, acts, grid, s, dp, tp); break;
        case 18: launch_gchain_v<2, 2>(mode, acts, grid, s, dp, tp); break;
        default: throw std::runtime_error("gchain: bad variant");
    }
    SERANN_CHECK(hipGetLastError());
}
