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
//   bin_prep  per (problem, n): Y0, D; the row's W staged through LDS in whole positions; E[.][n], C0[n]
//   bin_fwd   per (problem, 32 rows): the slice's fp32 partial of out into its split-K workspace slot; each thread
//             holds its column's 32 accumulators and reads E[p][n] once per position
//   (H and cs: one Dense WGRAD launch of the existing gemm3 kernel, dW = dZ^T g with dZ's column sums as the "bias
//    gradient", in Q40 fixed point into the step's zeroed workspace -- the planner adds it, K = B rows)
//   bin_sw    per (problem, 64 or 256 slice columns j = pF + f): one pass down the columns (4 waves over the Nc rows) reads each
//             weight once for S1 / St and, as the element's sole writer, stores its Q40 gradient or applies
//             Keras-Adam in place; then N1 and the 8 sums into NbnDesc::part slot 0 (nbn phase 6 finishes them)
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

// tiles: (problem, n).  The row's weights reach LDS a pass of whole positions at a time (8-B loads, all in
// flight, when the row is 8-B aligned); then four lanes per position (f = q, q + 4, ...) form E, their partials
// meeting in a fixed-order pair exchange, and every lane adds its elements' Y0 terms to C0
constexpr int BIN_STAGE = 8192;
__global__ __launch_bounds__(256) void bin_prep_kernel(const BinDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    __shared__ float sY0[256], sD[256], red[4];
    __shared__ __attribute__((aligned(16))) bf16_t sw[BIN_STAGE];
    const int2 td = tiles[blockIdx.x];
    const BinDesc& d = descs[td.x];
    const int n = td.y, L = (int)d.L, F = (int)d.F, Nc = (int)d.Nc;
    const int t = threadIdx.x;
    if (t < F) {
        const BinUnit u = bin_unit(d, t);
        sY0[t] = u.Y0;
        sD[t] = u.D;
    }
    const bf16_t* __restrict__ Wr = reinterpret_cast<const bf16_t*>(d.wc) + (int64_t)n * d.ldw;
    const bool vec = (reinterpret_cast<uintptr_t>(Wr) & 7) == 0;
    float* __restrict__ E = reinterpret_cast<float*>(d.E);
    const int ppass = (BIN_STAGE / F) & ~3;          // positions per pass (>= 32; a multiple of 4 keeps 8-B alignment)
    const int q = t & 3, pl = t >> 2;
    float c0 = 0.f;
    for (int p0 = 0; p0 < L; p0 += ppass) {
        const int np = min(ppass, L - p0), j0 = p0 * F, nj = np * F;
        __syncthreads();                              // (sY0 / sD written; the previous pass's readers done)
        if (vec) {
            const uint2* __restrict__ src = reinterpret_cast<const uint2*>(Wr + j0);
            const int n4 = nj >> 2;
#pragma unroll 8
            for (int i = t; i < n4; i += 256) reinterpret_cast<uint2*>(sw)[i] = src[i];
            for (int i = 4 * n4 + t; i < nj; i += 256) sw[i] = Wr[j0 + i];
        } else {
#pragma unroll 8
            for (int i = t; i < nj; i += 256) sw[i] = Wr[j0 + i];
        }
        __syncthreads();
        for (int pp = pl; pp < np; pp += 64) {        // the four lanes of a position share pp (same wave)
            const bf16_t* wp = sw + pp * F;
            float e = 0.f;
            for (int f = q; f < F; f += 4) {
                const float wv = bf2f(wp[f]);
                e = fmaf(sD[f], wv, e);
                c0 = fmaf(sY0[f], wv, c0);
            }
            e += __shfl_xor(e, 1, 64);
            e += __shfl_xor(e, 2, 64);
            if (q == 0) E[(int64_t)(p0 + pp) * Nc + n] = e;
        }
    }
    c0 = block_sum256(c0, red);
    if (t == 0) reinterpret_cast<float*>(d.C0)[n] = c0;
}

// tiles: (problem, first row / 32)
constexpr int BIN_ROWS = 32;
__global__ __launch_bounds__(256) void bin_fwd_kernel(const BinDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    __shared__ float sg[256 * BIN_ROWS];             // g transposed: [position][row]
    const int2 td = tiles[blockIdx.x];
    const BinDesc& d = descs[td.x];
    const int L = (int)d.L, Nc = (int)d.Nc, M = (int)d.B;
    const int m0 = td.y * BIN_ROWS, nr = min(BIN_ROWS, M - m0);
    const bf16_t* __restrict__ g = reinterpret_cast<const bf16_t*>(d.g) + (int64_t)m0 * L;
    for (int i = threadIdx.x; i < BIN_ROWS * L; i += 256) {
        const int r = i / L, p = i - r * L;
        sg[p * BIN_ROWS + r] = r < nr ? bf2f(g[i]) : 0.f;
    }
    __syncthreads();
    const float* __restrict__ E = reinterpret_cast<const float*>(d.E);
    float* __restrict__ slab = reinterpret_cast<float*>(d.slab) + (int64_t)m0 * Nc;
    for (int n = threadIdx.x; n < Nc; n += 256) {
        const float c0 = reinterpret_cast<const float*>(d.C0)[n];
        float acc[BIN_ROWS];
#pragma unroll
        for (int r = 0; r < BIN_ROWS; ++r) acc[r] = c0;
        for (int p = 0; p < L; ++p) {
            const float e = E[(int64_t)p * Nc + n];
            const float4* gp = reinterpret_cast<const float4*>(sg + p * BIN_ROWS);
#pragma unroll
            for (int q = 0; q < BIN_ROWS / 4; ++q) {
                const float4 gv = gp[q];
                acc[4 * q + 0] += gv.x * e;
                acc[4 * q + 1] += gv.y * e;
                acc[4 * q + 2] += gv.z * e;
                acc[4 * q + 3] += gv.w * e;
            }
        }
#pragma unroll
        for (int r = 0; r < BIN_ROWS; ++r)
            if (r < nr) slab[(int64_t)r * Nc + n] = acc[r];
    }
}

// tiles: (problem, (64 V-column block) * ns + split): lane -> columns j = pF + f .. + V - 1, wave -> rows
// n = r0 + wave, r0 + wave + 4, ... of the split's row range [r0, r1)  V = 4 (BIN_VEC4: 16-B fp32 / 8-B 16-bit accesses) when the slice's columns, row stride and arena
// offset are multiples of 4 and F >= 4 (a lane's columns span at most two positions), else V = 1.
// MM: Adam moment storage (common.h).  Explicit fmaf: the store and the fused-Adam branches must round alike (the
// arena pass and the in-place update see the same gradient)
#ifndef SERANN_BIN_UNROLL
#define SERANN_BIN_UNROLL 2
#endif
constexpr int BIN_NL = 4, BIN_UNROLL = SERANN_BIN_UNROLL, BIN_VEC4 = 4;
__device__ __forceinline__ float bin_grad(float Y0, float Dd, float c, float h) { return fmaf(Dd, h, Y0 * c); }

template <int V> __device__ __forceinline__ void ldv_bf(const bf16_t* p, float* x) {
    if constexpr (V == 4) {
        const uint2 u = *reinterpret_cast<const uint2*>(p);
        x[0] = __uint_as_float(u.x << 16); x[1] = __uint_as_float(u.x & 0xffff0000u);
        x[2] = __uint_as_float(u.y << 16); x[3] = __uint_as_float(u.y & 0xffff0000u);
    } else {
        x[0] = bf2f(p[0]);
    }
}
template <int V> __device__ __forceinline__ void ldv_f(const float* p, float* x) {
    if constexpr (V == 4) { const float4 u = *reinterpret_cast<const float4*>(p); x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w; }
    else x[0] = p[0];
}
template <int MM, int V> __device__ __forceinline__ void ldv_m(const void* b, int64_t e, float* x, bool second) {
    if constexpr (V == 4) {
        const float4 u = second ? v_ld4<MM>(b, e) : m_ld4<MM>(b, e);
        x[0] = u.x; x[1] = u.y; x[2] = u.z; x[3] = u.w;
    } else {
        x[0] = second ? v_ld<MM>(b, e) : m_ld<MM>(b, e);
    }
}

template <int MM, int V>
__device__ __forceinline__ void bin_sw_cols(const BinDesc& d, int j, int nb, int Nc, const int* pc, const float* Y0,
                                            const float* Dd, float* s1, float* st) {
    const int L = (int)d.L;
    const int64_t ldw = d.ldw;
    const bf16_t* __restrict__ W = reinterpret_cast<const bf16_t*>(d.wc) + j;
    const long long* __restrict__ Hq = reinterpret_cast<const long long*>(d.Hm);       // Q40 [Nc][L]
    const long long* __restrict__ csq = reinterpret_cast<const long long*>(d.cs);      // Q40 [Nc]
    long long* __restrict__ out = reinterpret_cast<long long*>(d.dw) + j;
    // a lane's columns lie in positions pc[0] and pc[0] + 1 (F >= V)
    const int pa = pc[0], pb = min(pc[0] + 1, L - 1);
    if (!d.adam) {
        for (int n = nb; n < Nc; n += BIN_NL) {
            const float ha = fx_f(Hq[(int64_t)n * L + pa]), hb = fx_f(Hq[(int64_t)n * L + pb]), c = fx_f(csq[n]);
            float w[V];
            ldv_bf<V>(W + n * ldw, w);
#pragma unroll
            for (int k = 0; k < V; ++k) {
                const float h = pc[k] == pa ? ha : hb;
                s1[k] = fmaf(h, w[k], s1[k]);
                st[k] = fmaf(c, w[k], st[k]);
                out[n * ldw + k] = fx_q(bin_grad(Y0[k], Dd[k], c, h));
            }
        }
        return;
    }
    const AdamCtx ac = *reinterpret_cast<const AdamCtx*>(d.adam);
    const int64_t e0 = out - reinterpret_cast<const long long*>(ac.g);
    float* __restrict__ P = reinterpret_cast<float*>(ac.p) + e0;
    bf16_t* __restrict__ Pb = reinterpret_cast<bf16_t*>(ac.pbf) + e0;
    const float lr_t = *reinterpret_cast<const float*>(ac.lr_t);
    const int64_t* __restrict__ org_off = reinterpret_cast<const int64_t*>(ac.org_off);
    int* __restrict__ diverged = reinterpret_cast<int*>(ac.diverged);
    const int norg = (int)ac.norg;
    const float b1 = ac.b1, b2 = ac.b2, eps = ac.eps;
    void* __restrict__ Mo = reinterpret_cast<void*>(ac.m);
    void* __restrict__ Vo = reinterpret_cast<void*>(ac.v);
    for (int n0 = nb; n0 < Nc; n0 += BIN_NL * BIN_UNROLL) {
        float w[BIN_UNROLL][V], p_[BIN_UNROLL][V], m_[BIN_UNROLL][V], v_[BIN_UNROLL][V];
        float ha[BIN_UNROLL], hb[BIN_UNROLL], c[BIN_UNROLL];
#pragma unroll
        for (int u = 0; u < BIN_UNROLL; ++u) {                 // all loads of the group first
            const int n = min(n0 + u * BIN_NL, Nc - 1);
            const int64_t o = n * ldw;
            ldv_bf<V>(W + o, w[u]);
            ldv_f<V>(P + o, p_[u]);
            ldv_m<MM, V>(Mo, e0 + o, m_[u], false);
            ldv_m<MM, V>(Vo, e0 + o, v_[u], true);
            ha[u] = fx_f(Hq[(int64_t)n * L + pa]);
            hb[u] = fx_f(Hq[(int64_t)n * L + pb]);
            c[u] = fx_f(csq[n]);
        }
#pragma unroll
        for (int u = 0; u < BIN_UNROLL; ++u) {
            if (n0 + u * BIN_NL >= Nc) break;
            const int64_t o = (int64_t)(n0 + u * BIN_NL) * ldw;
#pragma unroll
            for (int k = 0; k < V; ++k) {
                const float h = pc[k] == pa ? ha[u] : hb[u];
                s1[k] = fmaf(h, w[u][k], s1[k]);
                st[k] = fmaf(c[u], w[u][k], st[k]);
                const float gq = fx_f(fx_q(bin_grad(Y0[k], Dd[k], c[u], h)));   // as the Q40 arena would hold it
                if (SERANN_DIVERGE_CHECK && org_off != nullptr && fabsf(gq) > FX_DIVERGE)
                    flag_diverged(org_off, diverged, norg, e0 + o + k);
                adam_elem(p_[u][k], m_[u][k], v_[u][k], gq, lr_t, b1, b2, eps);
            }
            if constexpr (V == 4) {
                *reinterpret_cast<float4*>(P + o) = make_float4(p_[u][0], p_[u][1], p_[u][2], p_[u][3]);
                m_st4<MM>(Mo, e0 + o, make_float4(m_[u][0], m_[u][1], m_[u][2], m_[u][3]));
                v_st4<MM>(Vo, e0 + o, make_float4(v_[u][0], v_[u][1], v_[u][2], v_[u][3]));
                *reinterpret_cast<uint2*>(Pb + o) = make_uint2(f2bf2(p_[u][0], p_[u][1]), f2bf2(p_[u][2], p_[u][3]));
            } else {
                P[o] = p_[u][0];
                m_st<MM>(Mo, e0 + o, m_[u][0]);
                v_st<MM>(Vo, e0 + o, v_[u][0]);
                Pb[o] = f2bf(p_[u][0]);
            }
        }
    }
}

template <int V>
__device__ __forceinline__ void bin_sw_block(const BinDesc& d, int jb, int sp) {
    constexpr int COLS = 64 * V;
    __shared__ float red[256], sN1[256], sS1[BIN_NL][COLS], sSt[BIN_NL][COLS];
    const int F = (int)d.F, Nc = (int)d.Nc, L = (int)d.L, M = (int)d.B, W = L * F;
    const int t = threadIdx.x, lane = t & 63;
    const int nl = __builtin_amdgcn_readfirstlane(t >> 6);   // wave-uniform: row indices and cs in scalar registers
    const int j0 = jb * COLS, j = j0 + lane * V;
    const int ns = (int)d.ns, r0 = (int)((int64_t)sp * Nc / ns), r1 = (int)((int64_t)(sp + 1) * Nc / ns);
    if (jb == 0 && sp == 0 && d.dbias) {             // the consumer's bias gradient: cs, once per problem
        const long long* __restrict__ csq = reinterpret_cast<const long long*>(d.cs);
        for (int n = t; n < Nc; n += 256) fx_add(reinterpret_cast<long long*>(d.dbias) + n, fx_f(csq[n]));
    }
    // N1 of the block's positions [pl, pl + np): thread (mi, pi) sums rows mi, mi + nm, ... of position pl + pi
    const int pl = j0 / F, np = min(L - 1, (j0 + COLS - 1) / F) - pl + 1, nm = 256 / np;
    if (sp == 0) {                                    // (block-uniform)
        const bf16_t* __restrict__ g = reinterpret_cast<const bf16_t*>(d.g) + pl;
        const int pi = t % np, mi = t / np;
        float c = 0.f;
        if (mi < nm)
            for (int m = mi; m < M; m += nm) c += bf2f(g[(int64_t)m * L + pi]);
        red[t] = c;
        __syncthreads();
        if (t < np) {
            float s = 0.f;
            for (int k = 0; k < nm; ++k) s += red[k * np + t];
            sN1[t] = s;
        }
    }
    int pc[V];
    float Y0[V], Dd[V], s1[V], st[V];
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const int jc = min(j + k, W - 1);
        pc[k] = jc / F;
        const BinUnit u = bin_unit(d, jc - pc[k] * F);     // (recomputed for the sums: fewer live registers)
        Y0[k] = u.Y0;
        Dd[k] = u.D;
        s1[k] = st[k] = 0.f;
    }
    if (j < W) {
        if (d.adam && reinterpret_cast<const AdamCtx*>(d.adam)->mode == MOM_16)
            bin_sw_cols<MOM_16, V>(d, j, r0 + nl, r1, pc, Y0, Dd, s1, st);
        else
            bin_sw_cols<MOM_F32, V>(d, j, r0 + nl, r1, pc, Y0, Dd, s1, st);
    }
#pragma unroll
    for (int k = 0; k < V; ++k) {
        sS1[nl][lane * V + k] = s1[k];
        sSt[nl][lane * V + k] = st[k];
    }
    __syncthreads();
    if (nl != 0) return;
#pragma unroll
    for (int k = 0; k < V; ++k) {
        const int c = lane * V + k;
        if (j + k >= W) break;
        const float S1 = ((sS1[0][c] + sS1[1][c]) + sS1[2][c]) + sS1[3][c];
        const float St = ((sSt[0][c] + sSt[1][c]) + sSt[2][c]) + sSt[3][c];
        // (the count terms once: in split 0's slot; the S terms are linear, so the slots add up in phase 6)
        const float N1 = sp == 0 ? sN1[pc[k] - pl] : 0.f, N0 = sp == 0 ? (float)M - sN1[pc[k] - pl] : 0.f;
        const float s0 = St - S1;
        const BinUnit q = bin_unit(d, j + k - pc[k] * F);
        // the eight sums of gemm3.hip's GF_NBNSUM epilogue over the column's B rows (x = g in {0, 1}):
        //   [0] dy  [1] dy xhat  [2] a dy  [3] a xhat  [4] a  [5] a x dy  [6] a x xhat  [7] a x
        float* __restrict__ o = reinterpret_cast<float*>(d.part) + ((int64_t)sp * W + j + k) * NBN_NSUM;
        *reinterpret_cast<float4*>(o) = make_float4(St, q.xh0 * s0 + q.xh1 * S1, q.a0 * s0 + q.a1 * S1,
                                                    q.a0 * q.xh0 * N0 + q.a1 * q.xh1 * N1);
        *reinterpret_cast<float4*>(o + 4) = make_float4(q.a0 * N0 + q.a1 * N1, q.a1 * S1, q.a1 * q.xh1 * N1, q.a1 * N1);
    }
}

__global__ __launch_bounds__(256) void bin_sw_kernel(const BinDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const BinDesc& d = descs[td.x];
    const int ns = (int)d.ns, jb = td.y / ns;
    if (d.flags & BIN_VEC4)
        bin_sw_block<4>(d, jb, td.y - jb * ns);
    else
        bin_sw_block<1>(d, jb, td.y - jb * ns);
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
        case 3: hipLaunchKernelGGL(bin_sw_kernel, grid, block, 0, s, dp, tp); break;
        default: throw std::runtime_error("bin: unknown phase " + std::to_string(phase));
    }
    SERANN_CHECK(hipGetLastError());
}
