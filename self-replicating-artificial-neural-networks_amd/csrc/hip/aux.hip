// Auxiliary grouped kernels for the SeRANN population engine:
//   gather_batch (K14), DGRAD weight transposes, fused BatchNormalizationF16
//   train/infer/backward (K05/K06), maxpool fwd/bwd (K03), concat copies (K08), fused heads loss
//   (softmax-CE + sigmoid-MSE + accuracy + dlogits, K10/K11/K12/K17).
// Grouped kernels take a descriptor array and an int2 tile table (problem, chunk).
#include <hip/hip_fp16.h>
#include "common.h"
#include "serann_hip.h"

// ------------------------------------------------------------------------------------------------
__global__ void gather_batch_kernel(const bf16_t* __restrict__ x_all, const bf16_t* __restrict__ g_all,
                                    const int* __restrict__ y_all, const int* __restrict__ perm,
                                    const int* __restrict__ counter, int base, int B, int n_perm, int x_cols,
                                    int g_cols, bf16_t* __restrict__ x_out, bf16_t* __restrict__ g_out,
                                    int* __restrict__ y_out) {
    const int row = blockIdx.x;
    if (row >= B) return;
    int p = base + (counter ? *counter : 0) * B + row;
    if (p >= n_perm) p = n_perm - 1;
    const int src = perm[p];
    if ((x_cols & 1) == 0) {
        const uint32_t* xs = reinterpret_cast<const uint32_t*>(x_all + (int64_t)src * x_cols);
        uint32_t* xd = reinterpret_cast<uint32_t*>(x_out + (int64_t)row * x_cols);
        for (int i = threadIdx.x; i < x_cols / 2; i += blockDim.x) xd[i] = xs[i];
    } else {
        for (int i = threadIdx.x; i < x_cols; i += blockDim.x)
            x_out[(int64_t)row * x_cols + i] = x_all[(int64_t)src * x_cols + i];
    }
    for (int i = threadIdx.x; i < g_cols; i += blockDim.x) g_out[(int64_t)row * g_cols + i] = g_all[(int64_t)src * g_cols + i];
    if (threadIdx.x == 0) y_out[row] = y_all[src];
}

__global__ void counter_add_kernel(int* c, int v) { *c += v; }

__global__ void memset32_kernel(uint32_t* p, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) p[i] = 0u;
}

// ------------------------------------------------------------------------------------------------
// Channel-strided reduction layout of the wide-channel (C > 256) BatchNormalization (data [R][C] row-major):
// a block owns a chunk of rows; for C <= 256 its 256 threads are arranged as (256/C) row lanes x C
// channel lanes, so every thread keeps ONE channel for the whole chunk (parameters in registers, no
// per-element division, no atomics in the loop); per-channel partials are combined through LDS and
// leave the block as one fixed-point atomic per channel.  For C > 256 threads stride over channels.
constexpr int RED_ELEMS = 16384;   // elements per block (chunk rows = max(1, RED_ELEMS / C))

struct ChanMap {
    int c0, cstride, rlane, rstride;   // first channel, channel step, first row offset, row step
    bool active;
};

__device__ __forceinline__ ChanMap chan_map(int C) {
    ChanMap m;
    const int t = threadIdx.x;
    if (C <= 256) {
        const int rp = 256 / C;
        m.c0 = t % C;
        m.cstride = 1 << 30;          // one channel per thread
        m.rlane = t / C;
        m.rstride = rp;
        m.active = t < rp * C;
    } else {
        m.c0 = t;
        m.cstride = 256;
        m.rlane = 0;
        m.rstride = 1;
        m.active = true;
    }
    return m;
}

__device__ __forceinline__ int chunk_rows(int C) { return max(1, RED_ELEMS / max(C, 1)); }

// ------------------------------------------------------------------------------------------------
// BatchNormalizationF16 (channel-last, rows x C).  Phases:
//   0: ws[c] += sum (x - K_c), ws[C+c] += sum (x - K_c)^2 with the shift K_c = x[0][c]
//      (one pass, shifted sums keep the variance accurate when |mean| >> std)
//   2: train apply (+ moving statistics, saved mean / invstd)      3: inference apply
//   4: ws2[c] += sum dy, ws2[C+c] += sum dy*xhat                      5: backward apply (+ dgamma, dbeta)
__device__ __forceinline__ void bn_stats(const BnDesc& d, int C, float R, const long long* ws, int c, float& mu,
                                         float& var) {
    const float K = bf2f(reinterpret_cast<const bf16_t*>(d.x)[c]);
    const float m1 = fxw_sum<1>(ws, C, c) / R;
    mu = K + m1;
    var = fmaxf(fxw_sum<1>(ws, C, C + c) / R - m1 * m1, 0.f);
}

// ------------------------------------------------------------------------------------------------
// Vectorised BatchNormalizationF16 for C <= 256 (every BN of a SeRANN: X/g channels <= 128, merged
// units <= 256).  The [R][C] tensor is walked in "super-rows" of 8 rows = C chunks of 8 elements, so
// a thread that always takes chunk i of a super-row always sees the same 8 channels
// ((8i + j) mod C): 16-B loads/stores, per-thread registers for the 8 channels' parameters and
// partial sums, per-channel combination through LDS float atomics, one global atomic per channel
// and block.  Works for any C (odd channel counts included).
constexpr int BN_VEC_ELEMS = 16384;     // elements per block (super-rows per block = 2048 / C)
constexpr int BN_RED_MULT = 4;          // statistics phases: BN_RED_MULT x BN_VEC_ELEMS per block ...
constexpr int BN_STAT_SMALL = 2048;     // ... unless the problem spans fewer blocks than this at 1x

// rows-per-block multiplier of the statistics phases.  Large problems take BN_RED_MULT (1x: more
// device-scope atomics per channel, measured slower; 8x: too few blocks, also slower).  Small ones
// (< 2048 blocks at 1x, e.g. the merged-branch BN on [B][D]) are bound by the serial chain of loads in each
// block / too few CUs and keep 1x: [750][128] phase 4 16 -> 7 us, [96000][128] phase 0 21 -> 9 us (with the
// striped workspace below; before striping, 1x lost on mid-size problems).
__host__ __device__ __forceinline__ int bn_stat_mult(int nsr, int srb1) {
    return (nsr + srb1 - 1) / srb1 < BN_STAT_SMALL ? 1 : BN_RED_MULT;
}

// Statistics workspace of the vectorised path: BN_WS_STRIPES copies of the 2C wide fixed-point sums
// (common.h fxw_*); block `tile` adds into copy tile % BN_WS_STRIPES (an eighth of the same-address
// atomics: they serialise in L2 and bounded the statistics phases), readers sum the copies in integer
// arithmetic -- the result does not depend on the order of the atomics (deterministic training).
// Producers fused into other kernels (GF_BNSTAT, gemm3.hip; gchain.hip) stripe the same way, by their own
// blockIdx.x % BN_WS_STRIPES.
__device__ __forceinline__ float wsum(const long long* ws, int C, int idx) {
    return fxw_sum<BN_WS_STRIPES>(ws, C, idx);
}

// BnDesc::pdb targets (serann_hip.h): the producing GEMM's per-channel bias gradient (channel c -> pdb[c]), or
// with flags 128 / 256 ONE bias element that receives -/+ the sum over every channel: the Dense(units=1)
// subtracted from / added to the BN input (x = a - Dense(..)): its bias gradient is -sum(dx), taken here in fp32
// (the bf16 dx the sub's reduction sees left noise ~1000x torch-bf16's on that mathematically-zero sum).
// Batch mean and biased variance of channel c from the phase-0 workspace: shifted sums against K = x[0][c] (bn phase 0,
// the narrow FWD kernel), or with flag 512 unshifted sums accumulated by the producing GEMM's epilogue (GF_BNUSTAT),
// finished in double
__device__ __forceinline__ void bn_mu_var(const BnDesc& d, const long long* ws, int C, float Rf, int c, float& mu,
                                          float& var) {
    if (d.flags & 512) {
        const double m = fxw_sum_d<BN_WS_STRIPES>(ws, C, c) / (double)Rf;
        mu = (float)m;
        var = (float)fmax(fxw_sum_d<BN_WS_STRIPES>(ws, C, C + c) / (double)Rf - m * m, 0.0);
    } else {
        const float K = bf2f(reinterpret_cast<const bf16_t*>(d.x)[c]);
        const float m1 = wsum(ws, C, c) / Rf;
        mu = K + m1;
        var = fmaxf(wsum(ws, C, C + c) / Rf - m1 * m1, 0.f);
    }
}

__device__ __forceinline__ int pdb_index(const BnDesc& d, int c) { return (d.flags & (128 | 256)) ? 0 : c; }
__device__ __forceinline__ float pdb_sign(const BnDesc& d) { return (d.flags & 128) ? -1.f : 1.f; }

template <int phase>
__device__ __forceinline__ void bn_vec(const BnDesc& d, int tile, float* sA, float* sB) {
    const int R = (int)d.R, C = (int)d.C;
    const int flags = (int)d.flags;
    const float eps = (float)d.eps;
    const float Rf = (float)R;
    const int t = threadIdx.x;
    const int G = 256 / C;                       // super-rows processed together
    const bool active = t < G * C;
    const int q = t / C, i = t - q * C;
    // the statistics phases (0, 4) walk BN_RED_MULT times more rows per block: every block ends with
    // 2C device-scope float atomics, which dominated those phases at 16K elements per block
    const int nsr = (R + 7) / 8;
    const int srb1 = max(1, (BN_VEC_ELEMS / 8) / C);
    const int srb = srb1 * ((phase == 0 || phase == 4) ? bn_stat_mult(nsr, srb1) : 1);
    const int sr0 = tile * srb, sr1 = min(nsr, sr0 + srb);
    const int64_t total = (int64_t)R * C;
    const bf16_t* __restrict__ x = reinterpret_cast<const bf16_t*>(d.x);
    const long long* ws = reinterpret_cast<const long long*>(d.ws);
    long long* wsw = reinterpret_cast<long long*>(d.ws) + (tile % BN_WS_STRIPES) * 4 * C;   // this block's copy
    int ch[8];
    {
        int c = (8 * i) % C;
#pragma unroll
        for (int j = 0; j < 8; ++j) { ch[j] = c; c = (c + 1 == C) ? 0 : c + 1; }
    }
    const bf16_t* __restrict__ dy = reinterpret_cast<const bf16_t*>(d.dy);
    bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(d.y);
    bf16_t* __restrict__ dx = reinterpret_cast<bf16_t*>(d.dx);
    const bool skip_dx = phase == 5 && (flags & 8);
    const bool acc_dx = phase == 5 && (flags & 4);
    const int pact = (flags >> 4) & 3;           // phase 5: fold the producer's act' into dx

    // Data loads are software-pipelined one batch of U super-rows ahead, and the first batch is issued
    // BEFORE the per-channel parameter setup (whose workspace reads are a dependent chain of global
    // loads): the block pays the parameter latency and the data latency once, overlapped.
    constexpr int U = 4;
    union V8 { uint4 u; bf16_t h[8]; };
    struct Batch { V8 xv[U], gv[U], old[U]; int64_t e[U]; int nv[U]; };
    auto issue = [&](Batch& bt, int sr) {
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const int s_ = sr + k * G;
            bt.e[k] = (int64_t)s_ * 8 * C + 8 * i;
            bt.nv[k] = (active && s_ < sr1) ? (int)max((int64_t)0, min((int64_t)8, total - bt.e[k])) : 0;
            bt.xv[k].u = make_uint4(0, 0, 0, 0);
            bt.gv[k].u = make_uint4(0, 0, 0, 0);
            bt.old[k].u = make_uint4(0, 0, 0, 0);
            if (bt.nv[k] == 8) {
                bt.xv[k].u = *reinterpret_cast<const uint4*>(x + bt.e[k]);
                if (phase >= 4) bt.gv[k].u = *reinterpret_cast<const uint4*>(dy + bt.e[k]);
                if (acc_dx) bt.old[k].u = *reinterpret_cast<const uint4*>(dx + bt.e[k]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {           // static indices: stays in registers
                    if (j < bt.nv[k]) {
                        bt.xv[k].h[j] = x[bt.e[k] + j];
                        if (phase >= 4) bt.gv[k].h[j] = dy[bt.e[k] + j];
                        if (acc_dx) bt.old[k].h[j] = dx[bt.e[k] + j];
                    }
                }
            }
        }
    };
    // phase 5 streams three tensors: a second batch in registers costs it occupancy (measured slower),
    // so it only issues its first batch early and loads later batches in the loop
    constexpr bool kAhead = phase != 5;
    Batch cur, nxt;
    if (!skip_dx) issue(cur, sr0 + q);

    // per-channel parameters into LDS (sA: scale-like, sB: shift-like)
    for (int c = t; c < C; c += 256) {
        float a = 0.f, b = 0.f;
        if (phase == 0) {
            a = bf2f(x[c]);                                    // shift K_c = x[0][c]
        } else if (phase == 2 || phase == 3) {
            float mu, var;
            if (phase == 2) {
                bn_mu_var(d, ws, C, Rf, c, mu, var);
            } else {
                mu = reinterpret_cast<const float*>(d.mm)[c];
                var = reinterpret_cast<const float*>(d.mv)[c];
            }
            const float is = rsqrtf(var + eps);
            const float gsc = (flags & 1) ? reinterpret_cast<const float*>(d.gamma)[c] * is : is;
            a = gsc;
            b = ((flags & 2) ? reinterpret_cast<const float*>(d.beta)[c] : 0.f) - mu * gsc;
        } else if (phase == 4) {
            a = reinterpret_cast<const float*>(d.mean)[c];
            b = reinterpret_cast<const float*>(d.invstd)[c];
        } else {   // phase 5: dx = gg * (dy - ma - (x - mu) * is * mb) = k1 * dy + k2 * x + k3
            const float mu = reinterpret_cast<const float*>(d.mean)[c];
            const float is = reinterpret_cast<const float*>(d.invstd)[c];
            const float gg = ((flags & 1) ? reinterpret_cast<const float*>(d.gamma)[c] : 1.f) * is;
            const float ma = wsum(ws, C, c) / Rf, mb = wsum(ws, C, C + c) / Rf;
            a = gg;                                            // k1
            b = -gg * is * mb;                                 // k2
            sA[256 + c] = -gg * (ma - mu * is * mb);           // k3
        }
        sA[c] = a;
        sB[c] = b;
    }
    if (phase == 2 && tile == 0) {
        const float mom = (float)d.momentum;
        float* mm = reinterpret_cast<float*>(d.mm);
        float* mv = reinterpret_cast<float*>(d.mv);
        float* mean = reinterpret_cast<float*>(d.mean);
        float* invstd = reinterpret_cast<float*>(d.invstd);
        for (int c = t; c < C; c += 256) {
            float mu, var;
            bn_mu_var(d, ws, C, Rf, c, mu, var);
            mm[c] = mm[c] * mom + mu * (1.f - mom);
            // BatchNormalizationF16's n / (n - (1 + eps)) (BatchNormalizationF16.py:134-140); flag 64: the
            // plain Bessel factor n / (n - 1) of a standard BatchNormalization (the RiboAE's)
            const float ub = (flags & 64) ? Rf / (Rf - 1.f) : Rf / (Rf - (1.f + eps));
            mv[c] = mv[c] * mom + var * ub * (1.f - mom);
            mean[c] = mu;
            invstd[c] = rsqrtf(var + eps);
        }
    }
    if (phase == 5 && tile == 0) {
        for (int c = t; c < C; c += 256) {
            if (flags & 1) reinterpret_cast<long long*>(d.dgamma)[c] += fx_q(wsum(ws, C, C + c));   // Q40 arena
            if (flags & 2) reinterpret_cast<long long*>(d.dbeta)[c] += fx_q(wsum(ws, C, c));
        }
    }
    __syncthreads();
    float pa[8], pb[8], p3[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        pa[j] = sA[ch[j]];
        pb[j] = sB[ch[j]];
        p3[j] = (phase == 5) ? sA[256 + ch[j]] : 0.f;
    }
    __syncthreads();
    long long* pdb = reinterpret_cast<long long*>(d.pdb);
    const bool reduce = phase == 0 || phase == 4 || (phase == 5 && pdb != nullptr);
    if (skip_dx) return;
    float acc0[8], acc1[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { acc0[j] = 0.f; acc1[j] = 0.f; }
    if (active) {
        for (int sr = sr0 + q; sr < sr1; sr += U * G) {
            const bool more = sr + U * G < sr1;
            if (!kAhead && sr != sr0 + q) issue(cur, sr);
            if (kAhead && more) issue(nxt, sr + U * G);
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const int nvk = cur.nv[k];
                if (nvk <= 0) continue;
                V8 ov;
                if (phase == 0) {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < nvk) { const float v = bf2f(cur.xv[k].h[j]) - pa[j]; acc0[j] += v; acc1[j] += v * v; }
                    continue;
                }
                if (phase == 4) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float g = bf2f(cur.gv[k].h[j]);
                        acc0[j] += g;
                        acc1[j] += g * (bf2f(cur.xv[k].h[j]) - pa[j]) * pb[j];
                    }
                    continue;
                }
                bf16_t* dst = (phase == 5) ? dx : y;
                if (phase == 5) {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const float xj = bf2f(cur.xv[k].h[j]);
                        float v = pa[j] * bf2f(cur.gv[k].h[j]) + pb[j] * xj + p3[j] + bf2f(cur.old[k].h[j]);
                        if (pact != ACT_LINEAR) v *= act_grad_from_y(xj, pact);
                        if (j < nvk) acc0[j] += v;
                        ov.h[j] = f2bf(v);
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) ov.h[j] = f2bf(bf2f(cur.xv[k].h[j]) * pa[j] + pb[j]);
                }
                if (nvk == 8) {
                    *reinterpret_cast<uint4*>(dst + cur.e[k]) = ov.u;
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < nvk) dst[cur.e[k] + j] = ov.h[j];
                }
            }
            if (kAhead && more) cur = nxt;
        }
    }
    if (reduce) {
        // slot (q, 8i + j) holds channel (8i + j) mod C of super-row group q; channel c owns the
        // slots c, c + C, ..., c + 7C of every group -- a gather instead of LDS atomics
        float* r0 = sA;
        float* r1 = sA + 2048;
        __syncthreads();
        if (active) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                r0[q * 8 * C + 8 * i + j] = acc0[j];
                r1[q * 8 * C + 8 * i + j] = acc1[j];
            }
        }
        __syncthreads();
        if ((C & (C - 1)) == 0 && C < 64) {
            // power-of-two C < 64: slot s holds channel s mod C and 256 % C == 0, so every slot thread t
            // sums (t, t + 256, ...; 8 of them) is channel t mod C; lanes of equal t mod C then combine by
            // xor shuffles.  All 256 threads share the 2048-slot gather (the per-channel loop below leaves
            // C threads walking 2048 / C slots each: 256 serial LDS reads at C = 8).
            const int lane = t & 63;
            float a = 0.f, b = 0.f;
#pragma unroll
            for (int s = t; s < 2048; s += 256) { a += r0[s]; b += r1[s]; }
            for (int o = C; o < 64; o <<= 1) { a += __shfl_xor(a, o, 64); b += __shfl_xor(b, o, 64); }
            if (lane < C) {
                if (phase == 5) {
                    fx_add(pdb + pdb_index(d, lane), pdb_sign(d) * a);
                } else {
                    fxw_add(wsw + 2 * lane, a);
                    fxw_add(wsw + 2 * (C + lane), b);
                }
            }
            return;
        }
        for (int c = t; c < C; c += 256) {
            float a = 0.f, b = 0.f;
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    a += r0[g * 8 * C + c + k * C];
                    b += r1[g * 8 * C + c + k * C];
                }
            if (phase == 5) {
                fx_add(pdb + pdb_index(d, c), pdb_sign(d) * a);
            } else {
                fxw_add(wsw + 2 * c, a);
                fxw_add(wsw + 2 * (C + c), b);
            }
        }
    }
}

// One instantiation per phase: each keeps only the registers its phase uses (the software-pipelined
// load batches of phase 5 hold x, dy and the accumulated dx; phases 0 / 2 / 3 only x).
template <int phase>
__global__ __launch_bounds__(256) void bn_kernel(const BnDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    __shared__ float s0[4096];           // vectorised path: 2 x (G * 8 * C <= 2048) reduction slots
    __shared__ float s1[256];
    const int2 td = tiles[blockIdx.x];
    const BnDesc& d = descs[td.x];
    if (d.C <= 256) {
        bn_vec<phase>(d, td.y, s0, s1);
        return;
    }
    const int R = (int)d.R, C = (int)d.C;
    const int flags = (int)d.flags;
    const float eps = (float)d.eps;
    const bf16_t* __restrict__ x = reinterpret_cast<const bf16_t*>(d.x);
    long long* ws = reinterpret_cast<long long*>(d.ws);     // one wide copy (C > 256: no stripes)
    const float* gamma = reinterpret_cast<const float*>(d.gamma);
    const float* beta = reinterpret_cast<const float*>(d.beta);
    float* mean = reinterpret_cast<float*>(d.mean);
    float* invstd = reinterpret_cast<float*>(d.invstd);
    const int rows = chunk_rows(C);
    const int r0 = td.y * rows, r1 = min(R, r0 + rows);
    const float Rf = (float)R;
    const ChanMap m = chan_map(C);

    if (phase == 2 && td.y == 0) {
        // moving averages (K.moving_average_update) and saved statistics, once per problem
        const float mom = (float)d.momentum;
        float* mm = reinterpret_cast<float*>(d.mm);
        float* mv = reinterpret_cast<float*>(d.mv);
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            float mu, var;
            bn_stats(d, C, Rf, ws, c, mu, var);
            const float unbiased = var * ((flags & 64) ? Rf / (Rf - 1.f) : Rf / (Rf - (1.f + eps)));
            mm[c] = mm[c] * mom + mu * (1.f - mom);
            mv[c] = mv[c] * mom + unbiased * (1.f - mom);
            mean[c] = mu;
            invstd[c] = rsqrtf(var + eps);
        }
    }

    for (int c = m.c0; c < C && m.active; c += m.cstride) {
        const int rl = (C <= 256) ? m.rlane : 0, rs = (C <= 256) ? m.rstride : 1;
        if (phase == 0) {
            const float K = bf2f(x[c]);
            float a = 0.f, b = 0.f;
            for (int r = r0 + rl; r < r1; r += rs) {
                const float v = bf2f(x[(int64_t)r * C + c]) - K;
                a += v;
                b += v * v;
            }
            if (C <= 256) { s0[threadIdx.x] = a; s1[threadIdx.x] = b; }
            else { fxw_add(ws + 2 * c, a); fxw_add(ws + 2 * (C + c), b); }
        } else if (phase == 4) {
            const float mu = mean[c], is = invstd[c];
            const bf16_t* __restrict__ dy = reinterpret_cast<const bf16_t*>(d.dy);
            float a = 0.f, b = 0.f;
            for (int r = r0 + rl; r < r1; r += rs) {
                const int64_t off = (int64_t)r * C + c;
                const float g = bf2f(dy[off]);
                a += g;
                b += g * (bf2f(x[off]) - mu) * is;
            }
            if (C <= 256) { s0[threadIdx.x] = a; s1[threadIdx.x] = b; }
            else { fxw_add(ws + 2 * c, a); fxw_add(ws + 2 * (C + c), b); }
        } else if (phase == 2 || phase == 3) {
            float mu, is;
            if (phase == 2) {
                float var;
                bn_stats(d, C, Rf, ws, c, mu, var);
                is = rsqrtf(var + eps);
            } else {
                mu = reinterpret_cast<const float*>(d.mm)[c];
                is = rsqrtf(reinterpret_cast<const float*>(d.mv)[c] + eps);
            }
            const float gsc = (flags & 1) ? gamma[c] * is : is;
            const float sh = ((flags & 2) ? beta[c] : 0.f) - mu * gsc;
            bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(d.y);
            for (int r = r0 + rl; r < r1; r += rs) {
                const int64_t off = (int64_t)r * C + c;
                y[off] = f2bf(bf2f(x[off]) * gsc + sh);
            }
        } else {   // phase 5
            if (td.y == 0 && rl == 0) {
                long long* dg = reinterpret_cast<long long*>(d.dgamma);
                long long* db = reinterpret_cast<long long*>(d.dbeta);
                if (flags & 1) dg[c] += fx_q(fxw_sum<1>(ws, C, C + c));
                if (flags & 2) db[c] += fx_q(fxw_sum<1>(ws, C, c));
            }
            if (flags & 8) continue;
            const float mu = mean[c], is = invstd[c];
            const float gg = ((flags & 1) ? gamma[c] : 1.f) * is;
            const float a = fxw_sum<1>(ws, C, c) / Rf, b = fxw_sum<1>(ws, C, C + c) / Rf;
            const bf16_t* __restrict__ dy = reinterpret_cast<const bf16_t*>(d.dy);
            bf16_t* __restrict__ dx = reinterpret_cast<bf16_t*>(d.dx);
            float sdz = 0.f;
            for (int r = r0 + rl; r < r1; r += rs) {
                const int64_t off = (int64_t)r * C + c;
                const float xh = (bf2f(x[off]) - mu) * is;
                float v = gg * (bf2f(dy[off]) - a - xh * b);
                if (flags & 4) v += bf2f(dx[off]);
                if ((flags >> 4) & 3) v *= act_grad_from_y(bf2f(x[off]), (int)((flags >> 4) & 3));
                sdz += v;
                dx[off] = f2bf(v);
            }
            if (d.pdb) fx_add(reinterpret_cast<long long*>(d.pdb) + pdb_index(d, c), pdb_sign(d) * sdz);   // C > 256
        }
    }
    if ((phase == 0 || phase == 4) && C <= 256) {
        __syncthreads();
        if (threadIdx.x < C) {
            float a = 0.f, b = 0.f;
            for (int k = threadIdx.x; k < m.rstride * C; k += C) { a += s0[k]; b += s1[k]; }
            fxw_add(ws + 2 * threadIdx.x, a);
            fxw_add(ws + 2 * (C + threadIdx.x), b);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// MaxPool2D valid.  Forward stores the argmax window offset (uint8); backward is a gather over the
// windows covering each input element (handles overlapping windows from explicit strides).
constexpr int POOL_ELEMS = 1024;

// A work unit is V consecutive channels of one pixel: V = 8 (16-B vectors, 8-B argmax bytes) when
// C % 8 == 0 -- every pooled conv output, whose filter counts are powers of two -- else V = 1.  Index
// math is 32-bit (the tensors of one organism stay far below 2^31 elements).
__device__ __forceinline__ int pool_vec(int C) { return (C & 7) == 0 ? 8 : 1; }

// Unit -> (pixel, channel) -> (image, row, column) index math by fp64 reciprocals: n * (1 / d) rounded down is
// n / d exactly for 0 <= n < 2^31 and 1 <= d < 2^19 (the product's error is below 2^-21, the offset 2^-20 lifts
// exact quotients over it, and a true fractional part is at most 1 - 2^-19).  The integer divisions they replace
// (~30 instructions each, five to seven per unit) made the element-unit (C % 8 != 0) passes issue-bound.
__device__ __forceinline__ double pinv(int d) { return 1.0 / (double)d; }
__device__ __forceinline__ int pdiv(int n, double inv) { return (int)fma((double)n, inv, 0x1p-20); }

template <int V>
__device__ __forceinline__ void pool_fwd_units(const PoolDesc& d, int u0, int u1) {
    const int C = (int)d.C, OW = (int)d.OW, OH = (int)d.OH, W = (int)d.W, H = (int)d.H;
    const int PH = (int)d.PH, PW = (int)d.PW, SH = (int)d.SH, SW = (int)d.SW;
    const int CV = C / V;
    const double iCV = pinv(CV), iOHW = pinv(OH * OW), iOW = pinv(OW);
    const bf16_t* __restrict__ x = reinterpret_cast<const bf16_t*>(d.x);
    bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(d.y);
    uint8_t* __restrict__ idx = reinterpret_cast<uint8_t*>(d.idx);
    for (int u = u0 + (int)threadIdx.x; u < u1; u += blockDim.x) {
        const int pix = pdiv(u, iCV);
        const int c = (u - pix * CV) * V;
        const int b = pdiv(pix, iOHW);
        const int r = pix - b * (OH * OW);
        const int oh = pdiv(r, iOW), ow = r - oh * OW;
        float best[V];
        uint8_t bi[V];
#pragma unroll
        for (int j = 0; j < V; ++j) { best[j] = -INFINITY; bi[j] = 0; }
        for (int i = 0; i < PH; ++i)
            for (int jj = 0; jj < PW; ++jj) {
                const int off = ((b * H + oh * SH + i) * W + ow * SW + jj) * C + c;
                union { uint4 u; bf16_t h[8]; } xv;
                if (V == 8) xv.u = *reinterpret_cast<const uint4*>(x + off);
                else xv.h[0] = x[off];
#pragma unroll
                for (int j = 0; j < V; ++j) {
                    const float v = bf2f(xv.h[j]);
                    if (v > best[j] || (v != v && best[j] == best[j])) { best[j] = v; bi[j] = (uint8_t)(i * PW + jj); }
                }
            }
        const int o = pix * C + c;
        if (V == 8) {
            union { uint4 u; bf16_t h[8]; } ov;
            union { uint2 u; uint8_t b[8]; } iv;
#pragma unroll
            for (int j = 0; j < 8; ++j) { ov.h[j] = f2bf(best[j]); iv.b[j] = bi[j]; }
            *reinterpret_cast<uint4*>(y + o) = ov.u;
            *reinterpret_cast<uint2*>(idx + o) = iv.u;
        } else {
            y[o] = f2bf(best[0]);
            idx[o] = bi[0];
        }
    }
}

template <int V>
__device__ __forceinline__ void pool_bwd_units(const PoolDesc& d, int u0, int u1) {
    const int C = (int)d.C, OW = (int)d.OW, OH = (int)d.OH, W = (int)d.W, H = (int)d.H;
    const int PH = (int)d.PH, PW = (int)d.PW, SH = (int)d.SH, SW = (int)d.SW;
    const int CV = C / V;
    const double iCV = pinv(CV), iHW = pinv(H * W), iW = pinv(W), iSH = pinv(SH), iSW = pinv(SW);
    // non-overlapping windows (strides = pool size, Keras' default): an input element lies in at most one window
    const bool tiled = SH == PH && SW == PW;
    const bf16_t* __restrict__ dy = reinterpret_cast<const bf16_t*>(d.dy);
    bf16_t* __restrict__ dx = reinterpret_cast<bf16_t*>(d.dx);
    const uint8_t* __restrict__ idx = reinterpret_cast<const uint8_t*>(d.idx);
    for (int u = u0 + (int)threadIdx.x; u < u1; u += blockDim.x) {
        const int pix = pdiv(u, iCV);
        const int c = (u - pix * CV) * V;
        const int b = pdiv(pix, iHW);
        const int r = pix - b * (H * W);
        const int ih = pdiv(r, iW), iw = r - ih * W;
        float acc[V];
#pragma unroll
        for (int j = 0; j < V; ++j) acc[j] = 0.f;
        int oh_lo, oh_hi, ow_lo, ow_hi;
        if (tiled) {
            oh_lo = oh_hi = pdiv(ih, iSH);
            ow_lo = ow_hi = pdiv(iw, iSW);
            if (oh_lo >= OH) oh_hi = -1;                  // past the last window: no window, zero gradient
            if (ow_lo >= OW) ow_hi = -1;
        } else {
            oh_lo = max(0, pdiv(max(ih - PH + SH, 0), iSH)); oh_hi = min(OH - 1, pdiv(ih, iSH));
            ow_lo = max(0, pdiv(max(iw - PW + SW, 0), iSW)); ow_hi = min(OW - 1, pdiv(iw, iSW));
        }
        for (int oh = oh_lo; oh <= oh_hi; ++oh) {
            const int i = ih - oh * SH;
            if (i < 0 || i >= PH) continue;
            for (int ow = ow_lo; ow <= ow_hi; ++ow) {
                const int jj = iw - ow * SW;
                if (jj < 0 || jj >= PW) continue;
                const uint8_t want = (uint8_t)(i * PW + jj);
                const int o = ((b * OH + oh) * OW + ow) * C + c;
                union { uint4 u; bf16_t h[8]; } gv;
                union { uint2 u; uint8_t b[8]; } iv;
                if (V == 8) { gv.u = *reinterpret_cast<const uint4*>(dy + o); iv.u = *reinterpret_cast<const uint2*>(idx + o); }
                else { gv.h[0] = dy[o]; iv.b[0] = idx[o]; }
#pragma unroll
                for (int j = 0; j < V; ++j)
                    if (iv.b[j] == want) acc[j] += bf2f(gv.h[j]);
            }
        }
        const int e = pix * C + c;
        if (V == 8) {
            union { uint4 u; bf16_t h[8]; } ov, old;
            if (d.flags & 1) old.u = *reinterpret_cast<const uint4*>(dx + e);
#pragma unroll
            for (int j = 0; j < 8; ++j) ov.h[j] = f2bf(acc[j] + ((d.flags & 1) ? bf2f(old.h[j]) : 0.f));
            *reinterpret_cast<uint4*>(dx + e) = ov.u;
        } else {
            float v = acc[0];
            if (d.flags & 1) v += bf2f(dx[e]);
            dx[e] = f2bf(v);
        }
    }
}

// one block = POOL_ELEMS work units (units of V channels; tiles from hip_ops.pool_units)
__global__ __launch_bounds__(256) void pool_fwd_kernel(const PoolDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const PoolDesc& d = descs[td.x];
    const int V = pool_vec((int)d.C);
    const int total = (int)(d.B * d.OH * d.OW * d.C / V);
    const int u0 = td.y * POOL_ELEMS, u1 = min(total, u0 + POOL_ELEMS);
    if (V == 8) pool_fwd_units<8>(d, u0, u1);
    else pool_fwd_units<1>(d, u0, u1);
}

__global__ __launch_bounds__(256) void pool_bwd_kernel(const PoolDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const PoolDesc& d = descs[td.x];
    const int V = pool_vec((int)d.C);
    const int total = (int)(d.B * d.H * d.W * d.C / V);
    const int u0 = td.y * POOL_ELEMS, u1 = min(total, u0 + POOL_ELEMS);
    if (V == 8) pool_bwd_units<8>(d, u0, u1);
    else pool_bwd_units<1>(d, u0, u1);
}

// ------------------------------------------------------------------------------------------------
constexpr int COPY_ROWS = 16;   // rows per block

__global__ __launch_bounds__(256) void copy2d_kernel(const CopyDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const CopyDesc& d = descs[td.x];
    const bf16_t* __restrict__ src = reinterpret_cast<const bf16_t*>(d.src);
    bf16_t* __restrict__ dst = reinterpret_cast<bf16_t*>(d.dst);
    const int64_t cols = d.cols;
    const bool acc = d.flags & 1;
    const int64_t r0 = (int64_t)td.y * COPY_ROWS, r1 = min(d.rows, r0 + COPY_ROWS);
    for (int64_t r = r0; r < r1; ++r) {
        const bf16_t* s = src + r * d.src_stride;
        bf16_t* o = dst + r * d.dst_stride;
        // 16-B vectors (gfx950 serves them at any 2-B alignment), scalar tail
        const int64_t nv = cols / 8;
        for (int64_t v = threadIdx.x; v < nv; v += blockDim.x) {
            uint4 val = *reinterpret_cast<const uint4*>(s + v * 8);
            if (acc) {
                uint4 old = *reinterpret_cast<const uint4*>(o + v * 8);
                const bf16_t* a = reinterpret_cast<const bf16_t*>(&val);
                const bf16_t* b = reinterpret_cast<const bf16_t*>(&old);
                uint4 res;
                bf16_t* c = reinterpret_cast<bf16_t*>(&res);
#pragma unroll
                for (int j = 0; j < 8; ++j) c[j] = f2bf(bf2f(a[j]) + bf2f(b[j]));
                val = res;
            }
            *reinterpret_cast<uint4*>(o + v * 8) = val;
        }
        for (int64_t c = nv * 8 + threadIdx.x; c < cols; c += blockDim.x) {
            float v = bf2f(s[c]);
            if (acc) v += bf2f(o[c]);
            o[c] = f2bf(v);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Fused heads loss: one wave per sample row.  logits fp32 [B][NC+L] (classification logits then
// replication logits), labels int [B], target bf16 [B][L].  Train: writes dlogits bf16 (d(lb*CE +
// (1-lb)*MSE)/dz, Keras mean reduction over the batch) and accumulates metrics[0]+=loss,
// metrics[1]+=correct, metrics[2]+=sum_row mean_j (sigmoid-g)^2, metrics[3]+=rows (int64 Q32 fixed point,
// common.h: the sums do not depend on the order of the blocks' atomics).
constexpr int LOSS_ROWS = 64;   // rows per block (16 per wave); metrics reduced per block

__global__ __launch_bounds__(256) void loss_kernel(const LossDesc* __restrict__ descs, int train, int nvalid) {
    __shared__ float red[4][4];
    const LossDesc& d = descs[blockIdx.y];
    const int B = (int)d.B, NC = (int)d.NC, L = (int)d.L;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const float lb = (float)d.lb;
    const float invB = 1.f / (float)B;
    float m_loss = 0.f, m_corr = 0.f, m_sq = 0.f, m_n = 0.f;
    const int r0 = blockIdx.x * LOSS_ROWS + wave * (LOSS_ROWS / 4);
    for (int row = r0; row < min(B, r0 + LOSS_ROWS / 4); ++row) {
        const bool valid = train ? true : (row < nvalid);
        const float* z = reinterpret_cast<const float*>(d.logits) + (int64_t)row * (NC + L);
        const int label = reinterpret_cast<const int*>(d.labels)[row];
        const bf16_t* tg = reinterpret_cast<const bf16_t*>(d.target) + (int64_t)row * L;
        // --- softmax cross-entropy over NC <= 64 classes
        const float zc = lane < NC ? z[lane] : -INFINITY;
        float mx = zc;
        int amax = lane < NC ? lane : 1 << 30;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float om = __shfl_xor(mx, o, 64);
            const int oi = __shfl_xor(amax, o, 64);
            if (om > mx || (om == mx && oi < amax)) { mx = om; amax = oi; }
        }
        const float ex = lane < NC ? __expf(zc - mx) : 0.f;
        const float se = warp_sum(ex);
        const float zl = __shfl(zc, label < 64 ? label : 0, 64);
        const float ce = (__logf(se) + mx) - zl;
        // --- sigmoid MSE over L replication outputs
        float sq = 0.f;
        for (int j = lane; j < L; j += 64) {
            const float sg = 1.f / (1.f + __expf(-z[NC + j]));
            const float err = sg - bf2f(tg[j]);
            sq += err * err;
            if (train) {
                const float gr = (1.f - lb) * invB * 2.f * err / (float)L * sg * (1.f - sg);
                reinterpret_cast<bf16_t*>(d.dlogits)[(int64_t)row * (NC + L) + NC + j] = f2bf(gr);
            }
        }
        sq = warp_sum(sq);
        if (train && lane < NC) {
            const float p = ex / se;
            const float gc = lb * invB * (p - (lane == label ? 1.f : 0.f));
            reinterpret_cast<bf16_t*>(d.dlogits)[(int64_t)row * (NC + L) + lane] = f2bf(gc);
        }
        if (valid) {
            m_loss += lb * ce + (1.f - lb) * sq / (float)L;
            m_corr += amax == label ? 1.f : 0.f;
            m_sq += sq / (float)L;
            m_n += 1.f;
        }
    }
    if (lane == 0) { red[wave][0] = m_loss; red[wave][1] = m_corr; red[wave][2] = m_sq; red[wave][3] = m_n; }
    __syncthreads();
    if (threadIdx.x < 4) {
        const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
        if (v != 0.f) fxm_add(reinterpret_cast<long long*>(d.metrics) + threadIdx.x, v);   // Q32 (deterministic)
    }
}

// ================================================================================================
void launch_gather_batch(uint64_t x_all, uint64_t g_all, uint64_t y_all, uint64_t perm, uint64_t counter,
                         int64_t base, int64_t B, int64_t n_perm, int64_t x_cols, int64_t g_cols,
                         uint64_t x_out, uint64_t g_out, uint64_t y_out, uint64_t stream) {
    if (B <= 0) return;
    hipLaunchKernelGGL(gather_batch_kernel, dim3((unsigned)B), dim3(128), 0, as_stream(stream),
                       as_ptr<const bf16_t>(x_all), as_ptr<const bf16_t>(g_all), as_ptr<const int>(y_all),
                       as_ptr<const int>(perm), as_ptr<const int>(counter), (int)base, (int)B, (int)n_perm,
                       (int)x_cols, (int)g_cols, as_ptr<bf16_t>(x_out), as_ptr<bf16_t>(g_out), as_ptr<int>(y_out));
    SERANN_CHECK(hipGetLastError());
}

void launch_counter_add(uint64_t counter, int64_t value, uint64_t stream) {
    hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(1), 0, as_stream(stream), as_ptr<int>(counter), (int)value);
    SERANN_CHECK(hipGetLastError());
}

void launch_memset32(uint64_t ptr, int64_t n, uint64_t stream) {
    if (n <= 0) return;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(memset32_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), as_ptr<uint32_t>(ptr), n);
    SERANN_CHECK(hipGetLastError());
}

void launch_bn(int phase, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    const dim3 grid((unsigned)ntiles), block(256);
    const BnDesc* dp = as_ptr<const BnDesc>(descs);
    const int2* tp = as_ptr<const int2>(tiles);
    hipStream_t s = as_stream(stream);
    switch (phase) {
        case 0: hipLaunchKernelGGL(bn_kernel<0>, grid, block, 0, s, dp, tp); break;
        case 2: hipLaunchKernelGGL(bn_kernel<2>, grid, block, 0, s, dp, tp); break;
        case 3: hipLaunchKernelGGL(bn_kernel<3>, grid, block, 0, s, dp, tp); break;
        case 4: hipLaunchKernelGGL(bn_kernel<4>, grid, block, 0, s, dp, tp); break;
        case 5: hipLaunchKernelGGL(bn_kernel<5>, grid, block, 0, s, dp, tp); break;
        default: throw std::runtime_error("bn: bad phase");
    }
    SERANN_CHECK(hipGetLastError());
}

void launch_pool(int backward, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    if (backward)
        hipLaunchKernelGGL(pool_bwd_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                           as_ptr<const PoolDesc>(descs), as_ptr<const int2>(tiles));
    else
        hipLaunchKernelGGL(pool_fwd_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                           as_ptr<const PoolDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}

void launch_copy2d(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(copy2d_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const CopyDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}

void launch_loss(int train, uint64_t descs, int64_t nprob, int64_t B, uint64_t stream, int64_t nvalid) {
    if (nprob <= 0 || B <= 0) return;
    dim3 grid((unsigned)((B + LOSS_ROWS - 1) / LOSS_ROWS), (unsigned)nprob);
    hipLaunchKernelGGL(loss_kernel, grid, dim3(256), 0, as_stream(stream), as_ptr<const LossDesc>(descs), train,
                       (int)nvalid);
    SERANN_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// RiboAE decode epilogue: argmax over each group of V logits (K35).  One wave per group.
__global__ __launch_bounds__(256) void group_argmax_kernel(const float* __restrict__ logits, int* __restrict__ out,
                                                           int64_t ngroups, int V) {
    const int64_t grp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (grp >= ngroups) return;
    const int lane = threadIdx.x & 63;
    const float* z = logits + grp * V;
    float best = -INFINITY;
    int bi = 1 << 30;
    for (int v = lane; v < V; v += 64) {
        const float x = z[v];
        if (x > best) { best = x; bi = v; }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float ob = __shfl_xor(best, o, 64);
        const int oi = __shfl_xor(bi, o, 64);
        if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) out[grp] = bi;
}

void launch_group_argmax(uint64_t logits, uint64_t out, int64_t ngroups, int64_t V, uint64_t stream) {
    if (ngroups <= 0) return;
    hipLaunchKernelGGL(group_argmax_kernel, dim3((unsigned)((ngroups + 3) / 4)), dim3(256), 0, as_stream(stream),
                       as_ptr<const float>(logits), as_ptr<int>(out), ngroups, (int)V);
    SERANN_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Split-K finalize of the LDS-tiled FWD GEMM (GF_SPLITWS): out[m][n] = act(sum_s ws[s][m][n] + bias[n]),
// bf16 (or fp32 with flags & 1: the heads).  Grouped: tiles (problem, chunk of SPLITFIN_ELEMS outputs).
constexpr int SPLITFIN_ELEMS = 2048;

__global__ __launch_bounds__(256) void splitk_finalize_kernel(const SplitFinDesc* __restrict__ descs,
                                                              const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const SplitFinDesc& d = descs[td.x];
    const int64_t MN = d.M * d.N;
    const int N = (int)d.N, S = (int)d.S, act = (int)d.act;
    const float* __restrict__ ws = reinterpret_cast<const float*>(d.ws);
    const float* __restrict__ bias = reinterpret_cast<const float*>(d.bias);
    bf16_t* __restrict__ out = reinterpret_cast<bf16_t*>(d.out);
    float* __restrict__ out32 = reinterpret_cast<float*>(d.out);
    const bool f32 = d.flags & 1;
    const int64_t e0 = (int64_t)td.y * SPLITFIN_ELEMS;
    const int64_t e1 = min(MN, e0 + SPLITFIN_ELEMS);
    // 4 consecutive elements per thread (16-B partial loads, 8- / 16-B stores) when the slabs allow it; the
    // column index advances incrementally (no 64-bit modulo per element).  Splits are added in order.
    if ((MN & 3) == 0 && ((d.ws | d.out) & 15) == 0) {
        int64_t e = e0 + 4 * threadIdx.x;
        int col = (int)(e % N);
        const int step = (int)(1024 % N);
        for (; e < e1; e += 1024) {
            float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
            for (int s_ = 0; s_ < S; ++s_) {
                const float4 w = *reinterpret_cast<const float4*>(ws + s_ * MN + e);
                v.x += w.x; v.y += w.y; v.z += w.z; v.w += w.w;
            }
            float r[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                int c = col + j;
                if (c >= N) c -= N;
                if (c >= N) c %= N;                   // N < 4
                if (bias) r[j] += bias[c];
                r[j] = apply_act(r[j], act);
            }
            if (f32) *reinterpret_cast<float4*>(out32 + e) = make_float4(r[0], r[1], r[2], r[3]);
            else *reinterpret_cast<uint2*>(out + e) = make_uint2(f2bf2(r[0], r[1]), f2bf2(r[2], r[3]));
            col += step;
            if (col >= N) col -= N;
        }
        return;
    }
    for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
        float v = 0.f;
        for (int s_ = 0; s_ < S; ++s_) v += ws[s_ * MN + e];
        if (bias) v += bias[(int)(e % N)];
        v = apply_act(v, act);
        if (f32) out32[e] = v;
        else out[e] = f2bf(v);
    }
}

// Split WGRAD finalize (serann_hip.h WgFinDesc).  Grouped: tiles (problem, chunk of WGFIN_ELEMS outputs).
// A block sums 64 outputs over all S splits: the 4 waves take splits w, w + 4, ... (a wave's 64 lanes read 64
// consecutive slab floats per split, 4 splits in flight), then wave 0 adds the 4 partial sums in wave order --
// a fixed association, so the result is bitwise reproducible.  (One thread per output walking all S splits
// left a 15-block launch latency-bound: 100-240 us for a 15 MB slab set.)
__global__ __launch_bounds__(256) void wgrad_finalize_kernel(const WgFinDesc* __restrict__ descs,
                                                             const int2* __restrict__ tiles) {
    __shared__ float part[4][64];
    const int2 td = tiles[blockIdx.x];
    const WgFinDesc& d = descs[td.x];
    const int N = (int)d.N, C = (int)d.C, Cp = (int)d.Cp, S = (int)d.S;
    const int64_t ldp = (int64_t)(N / C) * Cp;
    const int64_t slab = d.M * ldp;
    const int64_t MN = d.M * (int64_t)N;
    const float* __restrict__ ws = reinterpret_cast<const float*>(d.ws);
    long long* __restrict__ out = reinterpret_cast<long long*>(d.out);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e = (int64_t)td.y * WGFIN_ELEMS + lane;
    const bool ok = e < MN;
    int64_t src = 0;
    if (ok) {
        const int64_t f = e / N;
        const int col = (int)(e - f * N);
        const int tap = col / C;
        src = f * ldp + (int64_t)tap * Cp + (col - tap * C);
    }
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;     // splits w + 16 i + {0, 4, 8, 12}: 4 loads in flight
    int s_ = w;
    if (ok) {
        for (; s_ + 12 < S; s_ += 16) {
            const float a = ws[s_ * slab + src], b = ws[(s_ + 4) * slab + src];
            const float c = ws[(s_ + 8) * slab + src], g = ws[(s_ + 12) * slab + src];
            v0 += a; v1 += b; v2 += c; v3 += g;
        }
        for (; s_ < S; s_ += 4) v0 += ws[s_ * slab + src];
    }
    part[w][lane] = (v0 + v1) + (v2 + v3);
    __syncthreads();
    if (w != 0 || !ok) return;
    const float v = ((part[0][lane] + part[1][lane]) + part[2][lane]) + part[3][lane];
    const long long q = fx_q(v);
    if (d.ldo) {                                      // a column slice of a wider dW (fused-concat K slice)
        const int64_t f = e / N;
        out += f * (d.ldo - N);                       // (element e of the slice -> f * ldo + col)
    }
    const AdamCtx* ac = reinterpret_cast<const AdamCtx*>(d.adam);
    if (ac == nullptr) {
        out[e] = q;
    } else {
        // sole writer of this parameter: the optimizer step here (as the GF_ADAM WGRAD epilogue)
        const int64_t pe = (out - reinterpret_cast<const long long*>(ac->g)) + e;
        float* P = reinterpret_cast<float*>(ac->p);
        void* Mo = reinterpret_cast<void*>(ac->m);
        void* Vo = reinterpret_cast<void*>(ac->v);
        bf16_t* Pb = reinterpret_cast<bf16_t*>(ac->pbf);    // (read before the stores below)
        const bool m16 = ac->mode == MOM_16;
        if (ac->org_off && fabsf(fx_f(q)) > FX_DIVERGE)
            flag_diverged(reinterpret_cast<const int64_t*>(ac->org_off), reinterpret_cast<int*>(ac->diverged),
                          (int)ac->norg, pe);
        float p_ = P[pe];
        float m_ = m16 ? m_ld<MOM_16>(Mo, pe) : m_ld<MOM_F32>(Mo, pe);
        float v_ = m16 ? v_ld<MOM_16>(Vo, pe) : v_ld<MOM_F32>(Vo, pe);
        adam_elem(p_, m_, v_, fx_f(q), *reinterpret_cast<const float*>(ac->lr_t), ac->b1, ac->b2, ac->eps);
        P[pe] = p_;
        if (m16) { m_st<MOM_16>(Mo, pe, m_); v_st<MOM_16>(Vo, pe, v_); }
        else { m_st<MOM_F32>(Mo, pe, m_); v_st<MOM_F32>(Vo, pe, v_); }
        Pb[pe] = f2bf(p_);
    }
}

void launch_wgrad_finalize(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(wgrad_finalize_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const WgFinDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}

void launch_splitk_finalize(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(splitk_finalize_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const SplitFinDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// RiboAE encoder input: out[r][e] = table[tokens[r]][e] for r < rows, e < E, where the
// table already holds the eval-mode BatchNormalization (one channel) folded into the embedding.
// Token ids are clamped into [0, V) so a corrupt id never reads outside the table.
__global__ __launch_bounds__(256) void embed_gather_kernel(const int* __restrict__ tokens,
                                                           const bf16_t* __restrict__ table,
                                                           bf16_t* __restrict__ out, int64_t rows, int E, int V) {
    const int64_t total = rows * E;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / E;
        const int e = (int)(i - r * E);
        const int tk = min(max(tokens[r], 0), V - 1);
        out[i] = table[(int64_t)tk * E + e];
    }
}

void launch_embed_gather(uint64_t tokens, uint64_t table, uint64_t out, int64_t rows, int64_t E, int64_t V,
                         uint64_t stream) {
    if (rows <= 0) return;
    const int64_t total = rows * E;
    const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 65536);
    hipLaunchKernelGGL(embed_gather_kernel, dim3(blocks), dim3(256), 0, as_stream(stream),
                       as_ptr<const int>(tokens), as_ptr<const bf16_t>(table), as_ptr<bf16_t>(out), rows,
                       (int)E, (int)V);
    SERANN_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Shared im2col of a single-channel network input (MNIST image X or genotype g) for one
// (KH, KW, SH, SW) configuration: out[m][k] (row stride K8 = roundup(KH*KW, 8), zero padded).
// Every organism of the population reads the SAME input batch, so the first-layer convolutions of
// all organisms with this configuration share one materialised im2col matrix, which turns their
// forward and weight-gradient GEMMs into aligned 16-B-vector 1x1 problems.
constexpr int IMCOL_ROWS = 64;

__global__ __launch_bounds__(256) void imcol_kernel(const ImcolDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const ImcolDesc& d = descs[td.x];
    const int H = (int)d.H, W = (int)d.W, OH = (int)d.OH, OW = (int)d.OW, KW = (int)d.KW, KH = (int)d.KH;
    const int SH = (int)d.SH, SW = (int)d.SW, K8 = (int)d.K8, K = KH * KW;
    const int64_t M = d.B * OH * OW;
    const bf16_t* __restrict__ x = reinterpret_cast<const bf16_t*>(d.x);
    bf16_t* __restrict__ out = reinterpret_cast<bf16_t*>(d.out);
    const int chunks = K8 / 8;
    const int64_t m0 = (int64_t)td.y * IMCOL_ROWS;
    for (int e = threadIdx.x; e < IMCOL_ROWS * chunks; e += blockDim.x) {
        const int64_t m = m0 + e / chunks;
        if (m >= M) break;
        const int c8 = (e % chunks) * 8;
        const int64_t b = m / (OH * OW);
        const int r = (int)(m - b * OH * OW);
        const int oh = r / OW, ow = r - (r / OW) * OW;
        const bf16_t* src = x + (b * H + oh * SH) * W + ow * SW;
        union { uint4 u; bf16_t h[8]; } v;
        v.u = make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = c8 + j;
            if (k < K) {
                const int kh = k / KW, kw = k - (k / KW) * KW;
                v.h[j] = src[kh * W + kw];
            }
        }
        *reinterpret_cast<uint4*>(out + m * K8 + c8) = v.u;
    }
}

void launch_imcol(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(imcol_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const ImcolDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Transposed bf16 weights for DGRAD kernels that cannot read the natural layout:
// Wt[c][kh][kw][f] = Wm[f][kh][kw][c], grouped over problems (4096 destination elements per block).
__global__ __launch_bounds__(256) void transpose_weights_kernel(const TransDesc* __restrict__ descs,
                                                                const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const TransDesc& d = descs[td.x];
    const int64_t total = d.F * d.P * d.C;
    const bf16_t* src = reinterpret_cast<const bf16_t*>(d.src);
    bf16_t* dst = reinterpret_cast<bf16_t*>(d.dst);
    const int64_t e0 = (int64_t)td.y * 4096;
    for (int64_t e = e0 + threadIdx.x; e < min(total, e0 + 4096); e += blockDim.x) {
        const int64_t f = e % d.F;                   // e indexes the destination [c][p][f]
        const int64_t rest = e / d.F;
        const int64_t pp = rest % d.P;
        const int64_t c = rest / d.P;
        dst[e] = src[(f * d.P + pp) * d.C + c];
    }
}

void launch_transpose_weights(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(transpose_weights_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const TransDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------------------------------------
// Replication epilogue (reference experiment_worker.py:151-160, experiment.py:206-209):
// offspring locus j of a row = round(clip(fp16(sigmoid(z_j)), 0, 1)) -- Keras predicts in fp16, and
// numpy rounds half to even, so the bit is fp16(sigmoid(z)) > 0.5 (NaN -> 0) -- packed 8 loci per byte,
// MSB first.  One thread per output byte; grid (row blocks, organisms).
__global__ __launch_bounds__(256) void rep_bits_kernel(const RepBitsDesc* __restrict__ descs) {
    const RepBitsDesc& d = descs[blockIdx.y];
    const int L = (int)d.L, NC = (int)d.NC, nb = (L + 7) >> 3;
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;       // byte index
    if (e >= d.rows * nb) return;
    const int64_t r = e / nb;
    const int j0 = (int)(e - r * nb) * 8;
    const float* z = reinterpret_cast<const float*>(d.logits) + r * (NC + L) + NC;
    uint32_t byte = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const int j = j0 + k;
        uint32_t bit = 0;
        if (j < L) {
            const float s = 1.f / (1.f + expf(-z[j]));
            bit = __half2float(__float2half_rn(s)) > 0.5f ? 1u : 0u;
        }
        byte |= bit << (7 - k);
    }
    reinterpret_cast<uint8_t*>(d.out)[e] = (uint8_t)byte;
}

void launch_rep_bits(uint64_t descs, int64_t ndesc, int64_t max_rows, int64_t row_bytes, uint64_t stream) {
    if (ndesc <= 0 || max_rows <= 0 || row_bytes <= 0) return;
    const int64_t bytes = max_rows * row_bytes;          // row_bytes = max over problems of ceil(L / 8)
    hipLaunchKernelGGL(rep_bits_kernel, dim3((unsigned)((bytes + 255) / 256), (unsigned)ndesc), dim3(256), 0,
                       as_stream(stream), as_ptr<const RepBitsDesc>(descs));
    SERANN_CHECK(hipGetLastError());
}
