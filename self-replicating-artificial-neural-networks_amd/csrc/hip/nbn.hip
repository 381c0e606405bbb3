// Fused raw-input Dense -> BatchNormalization for training plans ("nbn").
//
// The genome's most common replication branch (the example.json ancestor: g_layer = Dense(75)(g_layer);
// BatchNormalization) and many image branches apply a Dense with K <= 4 input channels to a raw input
// (genotype [B][100][1], image [B][28][28][1]) and feed it only to a BatchNormalization.  The Dense output
// y = act(x . w + b) then costs K + 1 flops per element to recompute from the raw input, against
// 2 B of HBM per element to store and re-read -- so it is never stored:
//   FWD  narrow Dense kernel with GF_BNSTAT | GF_NOSTORE: phase-0 statistics only (gemm3.hip)
//        nbn phase 2: recompute y, write the BN output, moving statistics     (reads x, writes out)
//   BWD  nbn phase 4: recompute y, sum dy and dy * xhat                        (reads x, dy)
//        nbn phase 5: recompute y, dz = (k1 dy + k2 y + k3) * act'(y) in fp32, the Dense's dW and db,
//                     BN dgamma / dbeta                                         (reads x, dy)
// Unfused, the same layer moves 9 tensors of [R][F] bf16 per step (Dense Y write; BN phase 2 read Y +
// write; phase 4 read Y, dY; phase 5 read Y, dY + write dZ; WGRAD read dZ); fused, 3.  The Dense's input
// is a raw input (no DGRAD).  dz never rounds to bf16, so the weight and bias gradients are also closer
// to fp32 than the unfused path's.
//
// Layout (the narrow "super-row" form, gemm3.hip g3_narrow_fwd_sr_kernel, and bn_vec): the [R][F] tensor
// is walked in super-rows of 8 rows = F chunks of 8 elements; thread i of a super-row group always takes
// chunk i, so its 8 elements keep their channels (8i + j) mod F and lie in rows ro[j] = (8i + j) / F
// (at most two distinct rows: 8 <= F <= 256).  All [R][F] accesses are aligned 16-B vectors.  Block
// partial sums meet in fixed point (common.h fx / fxw): bitwise reproducible in any grouping.
// Semantics: reference common/BatchNormalizationF16.py:81-153 (unbiased moving variance n / (n - 1 - eps)),
// Keras Dense (experiment_worker.py:66-128 trains the organism).
#include <type_traits>

#include "common.h"
#include "serann_hip.h"

namespace {

struct NbnCtx {
    int F, t, G, q, i;
    bool active;
    int ch[8], ro[8];
};

__device__ __forceinline__ NbnCtx nbn_ctx(int F) {
    NbnCtx c;
    c.F = F;
    c.t = threadIdx.x;
    c.G = 256 / F;
    c.q = c.t / F;
    c.i = c.t - c.q * F;
    c.active = c.q < c.G;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int e = 8 * c.i + j;
        c.ch[j] = e % F;
        c.ro[j] = e / F;
    }
    return c;
}

// y of channel f for one raw-input row: exactly the narrow FWD kernel's arithmetic (bias first, then the
// K products in order, activation), so the recomputed value is the one the statistics saw.  The Dense output
// is never stored, so it is never rounded to bf16 either (the statistics-only FWD pass keeps it fp32 too).
template <int K>
__device__ __forceinline__ float nbn_y(const float* xr, const float* w, float b, int act) {
    float v = b;
#pragma unroll
    for (int k = 0; k < K; ++k) v += xr[k] * w[k];
    return apply_act(v, act);
}

}  // namespace

template <int PHASE, int K>
__global__ __launch_bounds__(256) void nbn_kernel(const NbnDesc* __restrict__ descs, const int4* __restrict__ tiles) {
    constexpr int NQ = PHASE == 5 ? K + 1 : (PHASE == 4 ? 2 : 1);   // reduced quantities per element slot
    __shared__ float red[NQ * 2048];
    __shared__ float pa[256], pb[256], pc[256];
    const int4 td = tiles[blockIdx.x];       // (problem, first super-row, end super-row, first-block flag)
    const NbnDesc& d = descs[td.x];
    const int R = (int)d.R, F = (int)d.F, act = (int)d.act, ldx = (int)d.ldx;
    const int flags = (int)d.flags;
    const float Rf = (float)R, eps = (float)d.eps;
    const NbnCtx c = nbn_ctx(F);
    const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(d.x);
    const bf16_t* __restrict__ Wm = reinterpret_cast<const bf16_t*>(d.w);
    const float* bias = reinterpret_cast<const float*>(d.bias);
    const float* gamma = reinterpret_cast<const float*>(d.gamma);
    const float* beta = reinterpret_cast<const float*>(d.beta);
    float* mean = reinterpret_cast<float*>(d.mean);
    float* invstd = reinterpret_cast<float*>(d.invstd);

    // per-channel parameters into LDS: phase 2 scale / shift; phase 4 mean / invstd; phase 5 k1, k2, k3
    for (int f = c.t; f < F; f += 256) {
        float a, b, e = 0.f;
        if (PHASE == 2) {
            const long long* ws = reinterpret_cast<const long long*>(d.ws);
            float x0[K], w[K];
#pragma unroll
            for (int k = 0; k < K; ++k) { x0[k] = bf2f(X[k]); w[k] = bf2f(Wm[f * K + k]); }
            const float K0 = nbn_y<K>(x0, w, bias ? bias[f] : 0.f, act);     // the phase-0 shift (row 0)
            const float m1 = fxw_sum<BN_WS_STRIPES>(ws, F, f) / Rf;
            const float mu = K0 + m1;
            const float var = fmaxf(fxw_sum<BN_WS_STRIPES>(ws, F, F + f) / Rf - m1 * m1, 0.f);
            const float is = rsqrtf(var + eps);
            const float gsc = (flags & 1) ? gamma[f] * is : is;
            a = gsc;
            b = ((flags & 2) ? beta[f] : 0.f) - mu * gsc;
            if (td.w) {
                const float mom = (float)d.momentum;
                float* mm = reinterpret_cast<float*>(d.mm);
                float* mv = reinterpret_cast<float*>(d.mv);
                const float ub = (flags & 64) ? Rf / (Rf - 1.f) : Rf / (Rf - (1.f + eps));
                mm[f] = mm[f] * mom + mu * (1.f - mom);
                mv[f] = mv[f] * mom + var * ub * (1.f - mom);
                mean[f] = mu;
                invstd[f] = is;
            }
        } else if (PHASE == 4) {
            a = mean[f];
            b = invstd[f];
        } else {
            const long long* wsb = reinterpret_cast<const long long*>(d.wsb);
            const float mu = mean[f], is = invstd[f];
            const float gg = ((flags & 1) ? gamma[f] : 1.f) * is;
            const float sdy = fxw_sum<BN_WS_STRIPES>(wsb, F, f), sdyx = fxw_sum<BN_WS_STRIPES>(wsb, F, F + f);
            const float ma = sdy / Rf, mb = sdyx / Rf;
            a = gg;                                   // k1
            b = -gg * is * mb;                        // k2
            e = -gg * (ma - mu * is * mb);            // k3
            if (td.w) {                               // BN parameter gradients, once per problem
                if (flags & 1) reinterpret_cast<long long*>(d.dgamma)[f] += fx_q(sdyx);
                if (flags & 2) reinterpret_cast<long long*>(d.dbeta)[f] += fx_q(sdy);
            }
        }
        pa[f] = a;
        pb[f] = b;
        pc[f] = e;
    }
    __syncthreads();
    float w[8][K], bv[8], ka[8], kb[8], kc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int f = c.ch[j];
        bv[j] = bias ? bias[f] : 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) w[j][k] = bf2f(Wm[f * K + k]);
        ka[j] = pa[f];
        kb[j] = pb[f];
        kc[j] = pc[f];
    }
    float acc[8 * NQ];
#pragma unroll
    for (int j = 0; j < 8 * NQ; ++j) acc[j] = 0.f;

    // super-row range of this block: chosen by the planner (hip_ops.nbn_tiles), a function of the problem
    const int nsr = (R + 7) / 8;
    const int sr0 = td.y, sr1 = min(nsr, td.z);
    const int64_t total = (int64_t)R * F;
    const bf16_t* __restrict__ dY = reinterpret_cast<const bf16_t*>(d.dy);
    bf16_t* __restrict__ Yo = reinterpret_cast<bf16_t*>(d.y);
    union V8 { uint4 u; bf16_t h[8]; };
    if (c.active) {
        constexpr int U = 4;                          // super-rows in flight per thread
        for (int sb = sr0 + c.q; sb < sr1; sb += U * c.G) {
            float xa[U][K], xb[U][K];
            V8 g[U];
            int nv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int sr = sb + u * c.G;
                const int64_t e = (int64_t)sr * 8 * F + 8 * c.i;
                nv[u] = sr < sr1 ? (int)max((int64_t)0, min((int64_t)8, total - e)) : 0;
                const int ra = min(R - 1, min(sr, sr1 - 1) * 8 + c.ro[0]), rb = min(R - 1, ra + 1);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    xa[u][k] = bf2f(X[(int64_t)ra * ldx + k]);
                    xb[u][k] = bf2f(X[(int64_t)rb * ldx + k]);
                }
                if (PHASE != 2) {
                    g[u].u = make_uint4(0, 0, 0, 0);
                    if (nv[u] == 8) {
                        g[u].u = *reinterpret_cast<const uint4*>(dY + e);
                    } else {
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            if (j < nv[u]) g[u].h[j] = dY[e + j];
                    }
                }
            }
            // full super-rows take the unguarded path; only the problem's last super-row can be partial
            auto body = [&](int u, auto full_tag) {
                constexpr bool FULL = decltype(full_tag)::value;
                const int64_t e = (int64_t)(sb + u * c.G) * 8 * F + 8 * c.i;
                float yv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool hi = c.ro[j] != c.ro[0];
                    float xr[K];
#pragma unroll
                    for (int k = 0; k < K; ++k) xr[k] = hi ? xb[u][k] : xa[u][k];
                    const float y = nbn_y<K>(xr, w[j], bv[j], act);
                    yv[j] = y;
                    if (PHASE == 4) {
                        const float gy = bf2f(g[u].h[j]);              // 0 past the end
                        acc[j] += gy;
                        acc[8 + j] += gy * (y - ka[j]) * kb[j];
                    } else if (PHASE == 5 && (FULL || j < nv[u])) {
                        const float gy = bf2f(g[u].h[j]);
                        float dz = ka[j] * gy + kb[j] * y + kc[j];
                        if (act == ACT_RELU) dz = y > 0.f ? dz : 0.f;
                        else if (act == ACT_SIGMOID) dz *= y * (1.f - y);
#pragma unroll
                        for (int k = 0; k < K; ++k) acc[j * K + k] += dz * xr[k];
                        acc[8 * K + j] += dz;
                    }
                }
                if (PHASE == 2) {
                    uint4 o;
                    o.x = f2bf2(yv[0] * ka[0] + kb[0], yv[1] * ka[1] + kb[1]);
                    o.y = f2bf2(yv[2] * ka[2] + kb[2], yv[3] * ka[3] + kb[3]);
                    o.z = f2bf2(yv[4] * ka[4] + kb[4], yv[5] * ka[5] + kb[5]);
                    o.w = f2bf2(yv[6] * ka[6] + kb[6], yv[7] * ka[7] + kb[7]);
                    if (FULL) {
                        *reinterpret_cast<uint4*>(Yo + e) = o;
                    } else {
                        V8 ov;
                        ov.u = o;
#pragma unroll
                        for (int j = 0; j < 8; ++j)
                            if (j < nv[u]) Yo[e + j] = ov.h[j];
                    }
                }
            };
#pragma unroll
            for (int u = 0; u < U; ++u) {
                if (nv[u] == 8) body(u, std::true_type{});
                else if (nv[u] > 0) body(u, std::false_type{});
            }
        }
    }
    if (PHASE == 2) return;
    // slot q * 8F + 8i + j holds channel (8i + j) mod F of super-row group q (bn_vec layout); quantity p of
    // a slot lives at red[p * 2048 + slot]
    if (c.active) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int slot = c.q * 8 * F + 8 * c.i + j;
            if (PHASE == 4) {
                red[slot] = acc[j];
                red[2048 + slot] = acc[8 + j];
            } else {
#pragma unroll
                for (int k = 0; k < K; ++k) red[k * 2048 + slot] = acc[j * K + k];
                red[K * 2048 + slot] = acc[8 * K + j];
            }
        }
    }
    __syncthreads();
    for (int o = c.t; o < F * NQ; o += 256) {
        const int f = o / NQ, p = o - f * NQ;
        float v = 0.f;
        for (int g = 0; g < c.G; ++g)
#pragma unroll
            for (int m = 0; m < 8; ++m) v += red[p * 2048 + g * 8 * F + f + m * F];
        if (PHASE == 4) {
            long long* ws = reinterpret_cast<long long*>(d.wsb) + (blockIdx.x % BN_WS_STRIPES) * 4 * F;
            fxw_add(ws + 2 * (p * F + f), v);
        } else if (p < K) {
            fx_add(reinterpret_cast<long long*>(d.dw) + (int64_t)f * K + p, v);
        } else if (d.db) {
            fx_add(reinterpret_cast<long long*>(d.db) + f, v);
        }
    }
}

// Phase 6: the BN backward + Dense WGRAD of a K = 1 pair whose consumer DGRAD reduced the per-column sums into
// NbnDesc::part (gemm3.hip g3_tiled_kernel, GF_NBNSUM) -- the replacement of phases 4 and 5, which re-read the
// stored dY twice.  With gg = gamma * invstd, ma = sum(dy) / R, mb = sum(dy xhat) / R, the BN backward is
//   dz = a * gg * (dy - mb xhat - ma)          (a = act'(y); nbn.hip phase 5 forms the same dz per element)
// so dW = gg (S[a x dy] - mb S[a x xhat] - ma S[a x]), db = gg (S[a dy] - mb S[a xhat] - ma S[a]),
// dgamma = S[dy xhat], dbeta = S[dy].  A block owns NBN_FIN_CH channels of one problem; thread (channel, sum,
// part) adds a fixed share of the (m tile, position) slots in a fixed order (fp64), the parts are then added in
// order: bitwise reproducible.
constexpr int NBN_FIN_CH = 8, NBN_FIN_PARTS = 16;
__global__ __launch_bounds__(1024) void nbn_fin_kernel(const NbnDesc* __restrict__ descs, const int4* __restrict__ tiles) {
    __shared__ double tot[NBN_FIN_PARTS][NBN_FIN_CH * NBN_NSUM];
    const int4 td = tiles[blockIdx.x];                 // (problem, first channel, 0, 0)
    const NbnDesc& d = descs[td.x];
    const int F = (int)d.F, np = (int)d.np, mt = (int)d.mtiles;
    const int64_t N = (int64_t)np * F;
    const int f0 = td.y, nch = min(NBN_FIN_CH, F - f0);
    const float* __restrict__ part = reinterpret_cast<const float*>(d.part);
    const int t = threadIdx.x, slot = t & (NBN_FIN_CH * NBN_NSUM - 1), q = t / (NBN_FIN_CH * NBN_NSUM);
    static_assert(NBN_FIN_CH * NBN_NSUM * NBN_FIN_PARTS == 1024, "one thread per (channel, sum, part)");
    double v = 0.0;
    if (slot < nch * NBN_NSUM) {
        // the (m tile, position) slots of this (channel, sum), flattened and dealt round-robin to the parts:
        // each thread adds its share in a fixed order (a direct consumer has np = 1 and hundreds of m tiles,
        // the fused-concat one np = 100 and a few)
        const int u = f0 * NBN_NSUM + slot;            // (channel f0 + slot / 8, sum slot % 8): contiguous
        const int total = mt * np;
#pragma unroll 4
        for (int i = q; i < total; i += NBN_FIN_PARTS) {
            const int m = i / np, p = i - m * np;
            v += (double)part[((int64_t)m * N + (int64_t)p * F) * NBN_NSUM + u];
        }
    }
    tot[q][slot] = v;
    __syncthreads();
    if (t < nch) {
        const int f = f0 + t;
        double S[NBN_NSUM];
        // (pq outermost and not unrolled: the fully unrolled 16 x 8 double loads were hoisted into registers and
        // spilled 548 B of scratch per thread for the whole 1024-thread block)
#pragma unroll
        for (int k = 0; k < NBN_NSUM; ++k) S[k] = 0.0;
#pragma unroll 1
        for (int pq = 0; pq < NBN_FIN_PARTS; ++pq)
#pragma unroll
            for (int k = 0; k < NBN_NSUM; ++k) S[k] += tot[pq][t * NBN_NSUM + k];   // fixed order per sum
        const double Rf = (double)d.R;
        const double is = reinterpret_cast<const float*>(d.invstd)[f];
        const double gg = ((d.flags & 1) ? (double)reinterpret_cast<const float*>(d.gamma)[f] : 1.0) * is;
        const double ma = S[0] / Rf, mb = S[1] / Rf;
        if (d.flags & 1) fx_add(reinterpret_cast<long long*>(d.dgamma) + f, (float)S[1]);
        if (d.flags & 2) fx_add(reinterpret_cast<long long*>(d.dbeta) + f, (float)S[0]);
        fx_add(reinterpret_cast<long long*>(d.dw) + f, (float)(gg * (S[5] - mb * S[6] - ma * S[7])));
        if (d.db) fx_add(reinterpret_cast<long long*>(d.db) + f, (float)(gg * (S[2] - mb * S[3] - ma * S[4])));
    }
}

// Phase 7: the statistics of a K = 1 pair whose input is binary (a genotype batch of 0 / 1; the bnbn.hip
// factorisation's training plans).  y takes v0 = act(b) where x = 0 and v1 = act(b + w) where x = 1, so with C1
// ones among the R inputs the batch mean is (C0 v0 + C1 v1) / R and the biased variance (C0 (v0 - mu)^2 +
// C1 (v1 - mu)^2) / R (two-pass form, fp64): one pass over the R inputs instead of the statistics-only narrow FWD
// over the R x F outputs.  Moving statistics and mean / invstd as phase 2's first block.  tiles: (problem, ...).
__global__ __launch_bounds__(256) void nbn_binstat_kernel(const NbnDesc* __restrict__ descs, const int4* __restrict__ tiles) {
    __shared__ int red[4];
    const NbnDesc& d = descs[tiles[blockIdx.x].x];
    const int R = (int)d.R, F = (int)d.F, act = (int)d.act, flags = (int)d.flags, t = threadIdx.x;
    const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(d.x);
    // ones among the R inputs (K = 1: x is [R] contiguous; 16-B loads, four in flight)
    int c = 0;
    const int nv = (d.ldx == 1 && (d.x & 15) == 0) ? R / 8 : 0;
    const uint4* __restrict__ Xv = reinterpret_cast<const uint4*>(X);
    for (int i0 = t; i0 < nv; i0 += 4 * 256) {
        uint4 u[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = i0 + k * 256 < nv ? Xv[i0 + k * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t w4[4] = {u[k].x, u[k].y, u[k].z, u[k].w};
#pragma unroll
            for (int h = 0; h < 4; ++h)
                c += (__uint_as_float(w4[h] << 16) > 0.5f) + (__uint_as_float(w4[h] & 0xffff0000u) > 0.5f);
        }
    }
    for (int r = 8 * nv + t; r < R; r += 256) c += bf2f(X[(int64_t)r * d.ldx]) > 0.5f;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
    if ((t & 63) == 0) red[t >> 6] = c;
    __syncthreads();
    const double C1 = (double)(red[0] + red[1] + red[2] + red[3]), C0 = (double)R - C1, Rd = (double)R;
    const bf16_t* __restrict__ Wm = reinterpret_cast<const bf16_t*>(d.w);
    const float* bias = reinterpret_cast<const float*>(d.bias);
    const float eps = (float)d.eps, Rf = (float)R;
    for (int f = t; f < F; f += 256) {
        const float w = bf2f(Wm[f]), b = bias ? bias[f] : 0.f, zero = 0.f, one = 1.f;
        const double v0 = nbn_y<1>(&zero, &w, b, act), v1 = nbn_y<1>(&one, &w, b, act);
        const double mu = (C0 * v0 + C1 * v1) / Rd;
        const float var = (float)((C0 * (v0 - mu) * (v0 - mu) + C1 * (v1 - mu) * (v1 - mu)) / Rd);
        const float is = rsqrtf(var + eps);
        const float mom = (float)d.momentum;
        float* mm = reinterpret_cast<float*>(d.mm);
        float* mv = reinterpret_cast<float*>(d.mv);
        const float ub = (flags & 64) ? Rf / (Rf - 1.f) : Rf / (Rf - (1.f + eps));
        mm[f] = mm[f] * mom + (float)mu * (1.f - mom);
        mv[f] = mv[f] * mom + var * ub * (1.f - mom);
        reinterpret_cast<float*>(d.mean)[f] = (float)mu;
        reinterpret_cast<float*>(d.invstd)[f] = is;
    }
}

void launch_nbn(int phase, int k, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    const dim3 grid((unsigned)ntiles), block(256);
    hipStream_t s = as_stream(stream);
    const NbnDesc* dp = as_ptr<const NbnDesc>(descs);
    const int4* tp = as_ptr<const int4>(tiles);
    if (phase == 6) {
        hipLaunchKernelGGL(nbn_fin_kernel, grid, dim3(1024), 0, s, dp, tp);
        return;
    }
    if (phase == 7) {
        hipLaunchKernelGGL(nbn_binstat_kernel, grid, block, 0, s, dp, tp);
        return;
    }
#define NBN_CASE(P_, K_) \
    if (phase == P_ && k == K_) { hipLaunchKernelGGL((nbn_kernel<P_, K_>), grid, block, 0, s, dp, tp); return; }
#define NBN_K(K_) NBN_CASE(2, K_) NBN_CASE(4, K_) NBN_CASE(5, K_)
    NBN_K(1) NBN_K(2) NBN_K(3) NBN_K(4)
#undef NBN_K
#undef NBN_CASE
    throw std::runtime_error("nbn: unsupported phase " + std::to_string(phase) + " / K " + std::to_string(k));
}
