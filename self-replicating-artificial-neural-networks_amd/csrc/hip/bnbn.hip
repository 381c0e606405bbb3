// Binary-genotype factorisation of the replication branch's raw-input Dense -> BatchNormalization pair and the
// merged-Dense K slice that reads it ("bnbn"; training plans).
//
// The example.json ancestor and most of its descendants open the replication branch with
//   g_layer = Dense(units=F)(g_layer); g_layer = BatchNormalization()(g_layer)
// on the raw genotype g [B][L][1] (the organism's 100-bit genotype: every element is 0 or 1, experiment_worker.py
// 226-227, common/logic.py:38-55), flatten it and concatenate it into the merged Dense (layer_transitions.py:61-72).
// With one binary input channel the BN output y[m][p][f] = BN(act(g[m][p] w[f] + b[f])) takes exactly two values
// per unit f, Y0[f] (g = 0) and Y1[f] (g = 1), so with D = Y1 - Y0 the merged Dense's K slice of width L * F
//   out[m][n]  = sum_{p,f} y[m][p][f] W[n][pF + f] = C0[n] + sum_p g[m][p] E[p][n]
//                C0[n] = sum_{p,f} Y0[f] W[n][pF + f],   E[p][n] = sum_f D[f] W[n][pF + f]
//   dW[n][pF + f] = sum_m dZ[m][n] y[m][pF + f] = Y0[f] cs[n] + D[f] H[p][n]
//                cs[n] = sum_m dZ[m][n],                 H[p][n] = sum_m g[m][p] dZ[m][n]
// and the eight per-column backward sums the BN / Dense backward needs (gemm3.hip GF_NBNSUM, nbn.hip phase 6)
// follow from S1[p][f] = sum_n H[p][n] W[n][pF + f], St[p][f] = sum_n cs[n] W[n][pF + f] and the count N1[p] of
// ones at position p.  The slice's GEMMs (FWD over K = L F = 7500, DGRAD to [B][7500], WGRAD over B rows) become
// K = L GEMMs and elementwise passes, and y is never written: the same function of the weights and the genotype
// batch (Y0 / Y1 are the bf16 values the unfactorised GEMMs read), summed in another order.
//   bin_prep  per (problem, n): Y0, D (LDS), E[.][n], C0[n]               (reads W once)
//   bin_fwd   per (problem, 32 rows): the slice's fp32 partial of out into its split-K workspace slot
//   (H and cs: one Dense WGRAD launch of the existing gemm3 kernel, dW = dZ^T g with dZ's column sums as the "bias
//    gradient", in Q40 fixed point into the step's zeroed workspace -- the planner adds it, K = B rows)
//   bin_s     per (problem, position): N1, the 8 sums into NbnDesc::part slot 0 (nbn phase 6 finishes them)
//   bin_wg    per (problem, n): dW of the slice -> Q40 store, or Keras-Adam applied in place (sole writer)
// Every sum runs in a fixed order (no atomics besides the consumer-bias fx_add): bitwise reproducible.
#include "common.h"
#include "serann_hip.h"

namespace {

// per-unit constants of the pair: the pre-BN values v0 / v1 (fp32, as nbn.hip recomputes them), their activation
// derivatives, the normalised values and the bf16 BN outputs the consumer GEMM reads
struct BinUnit {
    float v0, v1, a0, a1, xh0, xh1, Y0, D;
};

__device__ __forceinline__ float act_d(float y, int act) {
    if (act == ACT_RELU) return y > 0.f ? 1.f : 0.f;
    if (act == ACT_SIGMOID) return y * (1.f - y);
    return 1.f;
}

__device__ __forceinline__ BinUnit bin_unit(const BinDesc& d, int f) {
    BinUnit u;
    const float w = bf2f(reinterpret_cast<const bf16_t*>(d.w)[f]);
    const float b = d.bias ? reinterpret_cast<const float*>(d.bias)[f] : 0.f;
    const int act = (int)d.act;
    // nbn.hip nbn_y: bias first, then the product (x = 0 / 1), activation
    u.v0 = apply_act(b + 0.f * w, act);
    u.v1 = apply_act(b + 1.f * w, act);
    u.a0 = act_d(u.v0, act);
    u.a1 = act_d(u.v1, act);
    const float mu = reinterpret_cast<const float*>(d.mean)[f];
    const float is = reinterpret_cast<const float*>(d.invstd)[f];
    u.xh0 = u.v0 * is + (-mu * is);
    u.xh1 = u.v1 * is + (-mu * is);
    // nbn.hip phase 2's output: y * gsc + (beta - mu gsc), rounded to bf16 (what the consumer GEMM would read)
    const float gsc = (d.flags & 1) ? reinterpret_cast<const float*>(d.gamma)[f] * is : is;
    const float sh = ((d.flags & 2) ? reinterpret_cast<const float*>(d.beta)[f] : 0.f) - mu * gsc;
    u.Y0 = bf2f(f2bf(u.v0 * gsc + sh));
    u.D = bf2f(f2bf(u.v1 * gsc + sh)) - u.Y0;
    return u;
}

__device__ __forceinline__ float block_sum256(float v, float* red) {
    v = warp_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

}  // namespace

// tiles: (problem, n)
__global__ __launch_bounds__(256) void bin_prep_kernel(const BinDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    __shared__ float sY0[256], sD[256], red[4];
    const int2 td = tiles[blockIdx.x];
    const BinDesc& d = descs[td.x];
    const int n = td.y, L = (int)d.L, F = (int)d.F, Nc = (int)d.Nc;
    const int t = threadIdx.x;
    if (t < F) {
        const BinUnit u = bin_unit(d, t);
        sY0[t] = u.Y0;
        sD[t] = u.D;
    }
    __syncthreads();
    const bf16_t* __restrict__ Wr = reinterpret_cast<const bf16_t*>(d.wc) + (int64_t)n * d.ldw;
    float c0 = 0.f;
    if (t < L) {
        float e = 0.f;
        const bf16_t* wp = Wr + t * F;
        for (int f = 0; f < F; ++f) {
            const float wv = bf2f(wp[f]);
            e += sD[f] * wv;
            c0 += sY0[f] * wv;
        }
        reinterpret_cast<float*>(d.E)[(int64_t)t * Nc + n] = e;
    }
    c0 = block_sum256(c0, red);
    if (t == 0) reinterpret_cast<float*>(d.C0)[n] = c0;
}

// tiles: (problem, first row / 32)
constexpr int BIN_ROWS = 32;
__global__ __launch_bounds__(256) void bin_fwd_kernel(const BinDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    __shared__ float sg[BIN_ROWS * 256];
    const int2 td = tiles[blockIdx.x];
    const BinDesc& d = descs[td.x];
    const int L = (int)d.L, Nc = (int)d.Nc, M = (int)d.B;
    const int m0 = td.y * BIN_ROWS, nr = min(BIN_ROWS, M - m0);
    const bf16_t* __restrict__ g = reinterpret_cast<const bf16_t*>(d.g);
    for (int i = threadIdx.x; i < nr * L; i += 256) sg[i] = bf2f(g[(int64_t)m0 * L + i]);
    __syncthreads();
    const int n = threadIdx.x;
    if (n >= Nc) return;
    const float* __restrict__ E = reinterpret_cast<const float*>(d.E);
    const float c0 = reinterpret_cast<const float*>(d.C0)[n];
    float* __restrict__ slab = reinterpret_cast<float*>(d.slab);
    for (int r = 0; r < nr; ++r) {
        float acc = c0;
        for (int p = 0; p < L; ++p) acc += sg[r * L + p] * E[(int64_t)p * Nc + n];
        slab[(int64_t)(m0 + r) * Nc + n] = acc;
    }
}

// tiles: (problem, position)
__global__ __launch_bounds__(256) void bin_s_kernel(const BinDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    __shared__ float red[4];
    const int2 td = tiles[blockIdx.x];
    const BinDesc& d = descs[td.x];
    const int F = (int)d.F, Nc = (int)d.Nc, L = (int)d.L, M = (int)d.B, p = td.y;
    const int f = threadIdx.x;
    // N1[p]: the ones at position p over the batch (fixed-order block sum)
    const bf16_t* __restrict__ g = reinterpret_cast<const bf16_t*>(d.g);
    float c = 0.f;
    for (int m = threadIdx.x; m < M; m += 256) c += bf2f(g[(int64_t)m * L + p]);
    const float N1 = block_sum256(c, red), N0 = (float)M - N1;
    const long long* __restrict__ Hq = reinterpret_cast<const long long*>(d.Hm);   // Q40 [Nc][L]
    const long long* __restrict__ csq = reinterpret_cast<const long long*>(d.cs);  // Q40 [Nc]
    if (p == 0 && d.dbias && f < Nc) fx_add(reinterpret_cast<long long*>(d.dbias) + f, fx_f(csq[f]));
    if (f >= F) return;
    const bf16_t* __restrict__ W = reinterpret_cast<const bf16_t*>(d.wc) + p * F + f;
    float s1 = 0.f, st = 0.f;
    for (int n = 0; n < Nc; ++n) {
        const float wv = bf2f(W[(int64_t)n * d.ldw]);
        s1 += fx_f(Hq[(int64_t)n * L + p]) * wv;
        st += fx_f(csq[n]) * wv;
    }
    const BinUnit u = bin_unit(d, f);
    const float s0 = st - s1;
    // the eight sums of gemm3.hip's GF_NBNSUM epilogue over the column's B rows (x = g in {0, 1}):
    //   [0] dy  [1] dy xhat  [2] a dy  [3] a xhat  [4] a  [5] a x dy  [6] a x xhat  [7] a x
    float* __restrict__ out = reinterpret_cast<float*>(d.part) + ((int64_t)p * F + f) * NBN_NSUM;
    const float4 lo = make_float4(st, u.xh0 * s0 + u.xh1 * s1, u.a0 * s0 + u.a1 * s1,
                                  u.a0 * u.xh0 * N0 + u.a1 * u.xh1 * N1);
    const float4 hi = make_float4(u.a0 * N0 + u.a1 * N1, u.a1 * s1, u.a1 * u.xh1 * N1, u.a1 * N1);
    *reinterpret_cast<float4*>(out) = lo;
    *reinterpret_cast<float4*>(out + 4) = hi;
}

// tiles: (problem, n).  MM: Adam moment storage (common.h)
template <int MM>
__device__ __forceinline__ void bin_wg_row(const BinDesc& d, int n, const float* sY0, const float* sD) {
    const int L = (int)d.L, F = (int)d.F, W = L * F;
    const float csn = fx_f(reinterpret_cast<const long long*>(d.cs)[n]);
    const long long* __restrict__ Hq = reinterpret_cast<const long long*>(d.Hm) + (int64_t)n * L;   // Q40 [Nc][L]
    long long* __restrict__ out = reinterpret_cast<long long*>(d.dw) + (int64_t)n * d.ldw;
    if (!d.adam) {
        for (int j = threadIdx.x; j < W; j += 256) {
            const int p = j / F, f = j - p * F;
            out[j] = fx_q(sY0[f] * csn + sD[f] * fx_f(Hq[p]));
        }
        return;
    }
    const AdamCtx ac = *reinterpret_cast<const AdamCtx*>(d.adam);
    const int64_t e0 = out - reinterpret_cast<const long long*>(ac.g);
    float* __restrict__ P = reinterpret_cast<float*>(ac.p);
    void* __restrict__ Mo = reinterpret_cast<void*>(ac.m);
    void* __restrict__ Vo = reinterpret_cast<void*>(ac.v);
    bf16_t* __restrict__ Pb = reinterpret_cast<bf16_t*>(ac.pbf);
    const float lr_t = *reinterpret_cast<const float*>(ac.lr_t);
    const int64_t* __restrict__ org_off = reinterpret_cast<const int64_t*>(ac.org_off);
    int* __restrict__ diverged = reinterpret_cast<int*>(ac.diverged);
    const int norg = (int)ac.norg;
    for (int j = threadIdx.x; j < W; j += 256) {
        const int p = j / F, f = j - p * F;
        const float gq = fx_f(fx_q(sY0[f] * csn + sD[f] * fx_f(Hq[p])));   // as the Q40 arena would hold it
        const int64_t e = e0 + j;
        if (SERANN_DIVERGE_CHECK && org_off != nullptr && fabsf(gq) > FX_DIVERGE) flag_diverged(org_off, diverged, norg, e);
        float p_ = P[e], m_ = m_ld<MM>(Mo, e), v_ = v_ld<MM>(Vo, e);
        adam_elem(p_, m_, v_, gq, lr_t, ac.b1, ac.b2, ac.eps);
        P[e] = p_;
        m_st<MM>(Mo, e, m_);
        v_st<MM>(Vo, e, v_);
        Pb[e] = f2bf(p_);
    }
}

__global__ __launch_bounds__(256) void bin_wg_kernel(const BinDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    __shared__ float sY0[256], sD[256];
    const int2 td = tiles[blockIdx.x];
    const BinDesc& d = descs[td.x];
    const int t = threadIdx.x;
    if (t < (int)d.F) {
        const BinUnit u = bin_unit(d, t);
        sY0[t] = u.Y0;
        sD[t] = u.D;
    }
    __syncthreads();
    if (d.adam && reinterpret_cast<const AdamCtx*>(d.adam)->mode == MOM_16)
        bin_wg_row<MOM_16>(d, td.y, sY0, sD);
    else
        bin_wg_row<MOM_F32>(d, td.y, sY0, sD);
}

void launch_bin(int phase, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    const dim3 grid((unsigned)ntiles), block(256);
    hipStream_t s = as_stream(stream);
    const BinDesc* dp = as_ptr<const BinDesc>(descs);
    const int2* tp = as_ptr<const int2>(tiles);
    switch (phase) {
        case 0: hipLaunchKernelGGL(bin_prep_kernel, grid, block, 0, s, dp, tp); break;
        case 1: hipLaunchKernelGGL(bin_fwd_kernel, grid, block, 0, s, dp, tp); break;
        case 3: hipLaunchKernelGGL(bin_s_kernel, grid, block, 0, s, dp, tp); break;
        case 4: hipLaunchKernelGGL(bin_wg_kernel, grid, block, 0, s, dp, tp); break;
        default: throw std::runtime_error("bin: unknown phase " + std::to_string(phase));
    }
    SERANN_CHECK(hipGetLastError());
}
