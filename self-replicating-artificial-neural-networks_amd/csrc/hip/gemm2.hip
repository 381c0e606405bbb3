// Grouped implicit-GEMM convolution, v2 (CDNA4 MFMA), the engine's default path.
//
// FWD / DGRAD -- "direct fragment" kernel.  A wave owns 32 output rows x BN columns; its MFMA operand
// fragments are loaded straight from global memory into VGPRs (no LDS, no barriers): lane l of
// mfma_f32_16x16x32_bf16 needs 8 consecutive reduction elements of one row, which for an NHWC
// activation (or a [N][K] weight) are 16 contiguous bytes whenever the 8 elements stay inside one
// pixel's channel vector (always for 1x1 / Dense problems).  gfx950 serves 16-B loads at any 2-B
// alignment (measured: scripts/micro/unaligned.hip), so odd channel counts keep the vector path; only
// chunks that straddle a pixel fall back to element gathers.  The next k-step's fragments are
// prefetched into registers while the current MFMAs run.  Weights ([N][K], L2-resident) are read by
// all 4 waves of a block, i.e. from L1.
//   FWD   : Y[m][f]  = act(im2col(X)[m][k] . Wm[f][k] + b[f])
//   DGRAD : dX[m][c] = sum_{k'=(kh,kw,f)} dZ[b,(ih-kh)/SH,(iw-kw)/SW,f] . Wt[c][k']     (Wt: transposed
//           weights [C][KH][KW][F], produced once per step by transpose_weights_kernel)
// WGRAD -- LDS kernel: both operands are naturally m-major (m = reduction index), so tiles are staged
// in their natural layouts with 16-B writes and the MFMA fragments are read with the CDNA4 transposing
// LDS read ds_read_b64_tr_b16 (two per fragment).  Split-K over m, fp32 atomics into the gradient arena.
#include "common.h"
#include "serann_hip.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;

namespace {

union Frag {
    uint4 u;
    bf16_t h[8];
    bf16x8_t v;
};

struct G2 {
    int H, W, C, OH, OW, F, KH, KW, SH, SW, M, N, K, act, flags;
};

__device__ __forceinline__ G2 geo2(const GemmDesc& d) {
    G2 g;
    g.H = (int)d.H; g.W = (int)d.W; g.C = (int)d.C; g.OH = (int)d.OH; g.OW = (int)d.OW; g.F = (int)d.F;
    g.KH = (int)d.KH; g.KW = (int)d.KW; g.SH = (int)d.SH; g.SW = (int)d.SW;
    g.M = (int)d.M; g.N = (int)d.N; g.K = (int)d.K; g.act = (int)d.act; g.flags = (int)d.flags;
    return g;
}

// dZ = dY * act'(Y): the activation backward fused into the loads of the output gradient (the
// separate act_bwd pass of v1 is gone); Y is the layer's post-activation output, same layout as dY.
__device__ __forceinline__ uint4 act_grad8(uint4 dy, const bf16_t* __restrict__ y, int64_t off, int act, int n) {
    if (act == ACT_LINEAR) return dy;
    Frag g, yv, out;
    g.u = dy;
    if (n == 8) {
        yv.u = *reinterpret_cast<const uint4*>(y + off);
    } else {
        yv.u = make_uint4(0, 0, 0, 0);
        for (int j = 0; j < n; ++j) yv.h[j] = y[off + j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) out.h[j] = f2bf(bf2f(g.h[j]) * act_grad_from_y(bf2f(yv.h[j]), act));
    return out.u;
}

// ---- FWD A fragment: im2col row (pixel base `base`), reduction index k..k+7 -----------------------
__device__ __forceinline__ uint4 fwd_a(const bf16_t* __restrict__ x, const G2& g, bool rowok, int base, int k) {
    Frag f;
    f.u = make_uint4(0, 0, 0, 0);
    if (!rowok || k >= g.K) return f.u;
    const int pix = k / g.C;
    const int ci = k - pix * g.C;
    if (ci + 8 <= g.C) {                               // inside one pixel: contiguous 16 B
        const int kh = pix / g.KW, kw = pix - (pix / g.KW) * g.KW;
        f.u = *reinterpret_cast<const uint4*>(x + base + (kh * g.W + kw) * g.C + ci);
        return f.u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kk = k + j;
        if (kk < g.K) {
            const int p = kk / g.C;
            const int c = kk - p * g.C;
            const int kh = p / g.KW, kw = p - (p / g.KW) * g.KW;
            f.h[j] = x[base + (kh * g.W + kw) * g.C + c];
        }
    }
    return f.u;
}

// ---- DGRAD A fragment: dZ gathered at input pixel (b, ih, iw), k' = (kh*KW+kw)*F + f ------------------
__device__ __forceinline__ uint4 dgrad_a(const bf16_t* __restrict__ dz, const bf16_t* __restrict__ y, const G2& g,
                                         bool rowok, int b, int ih, int iw, int k) {
    Frag fr;
    fr.u = make_uint4(0, 0, 0, 0);
    if (!rowok || k >= g.K) return fr.u;
    const int pix = k / g.F;
    const int f = k - pix * g.F;
    if (f + 8 <= g.F) {
        const int kh = pix / g.KW, kw = pix - (pix / g.KW) * g.KW;
        const int ohn = ih - kh, own = iw - kw;
        if (ohn < 0 || own < 0) return fr.u;
        const int oh = ohn / g.SH, ow = own / g.SW;
        if (oh * g.SH != ohn || ow * g.SW != own || oh >= g.OH || ow >= g.OW) return fr.u;
        const int64_t off = ((int64_t)(b * g.OH + oh) * g.OW + ow) * g.F + f;
        return act_grad8(*reinterpret_cast<const uint4*>(dz + off), y, off, g.act, 8);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int kk = k + j;
        if (kk >= g.K) break;
        const int p = kk / g.F;
        const int ff = kk - p * g.F;
        const int kh = p / g.KW, kw = p - (p / g.KW) * g.KW;
        const int ohn = ih - kh, own = iw - kw;
        if (ohn < 0 || own < 0) continue;
        const int oh = ohn / g.SH, ow = own / g.SW;
        if (oh * g.SH != ohn || ow * g.SW != own || oh >= g.OH || ow >= g.OW) continue;
        const int64_t off = ((int64_t)(b * g.OH + oh) * g.OW + ow) * g.F + ff;
        float v = bf2f(dz[off]);
        if (g.act != ACT_LINEAR) v *= act_grad_from_y(bf2f(y[off]), g.act);
        fr.h[j] = f2bf(v);
    }
    return fr.u;
}

// ---- B fragment: row n of a [N][K] (k-contiguous) matrix ---------------------------------------------
__device__ __forceinline__ uint4 row_b(const bf16_t* __restrict__ w, int N, int K, int n, int k) {
    Frag f;
    f.u = make_uint4(0, 0, 0, 0);
    if (n >= N || k >= K) return f.u;
    const bf16_t* p = w + (int64_t)n * K + k;
    if (k + 8 <= K) {
        f.u = *reinterpret_cast<const uint4*>(p);
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (k + j < K) f.h[j] = p[j];
    }
    return f.u;
}

}  // namespace

// ==================================================================================================
// FWD / DGRAD direct kernel.  NT = BN / 16 column tiles per wave.
//   KW = false: block = 4 waves x 32 rows = 128 rows, every wave runs the whole k range.
//   KW = true : block = 32 rows; the 4 waves split the k range (k-step w, w+4, ...) and their partial
//               accumulators are summed through LDS -- for long-K / few-row problems (Dense on the
//               flattened merge, heads) whose serial k loop would otherwise be latency-bound.
template <int MODE, int NT, bool KW>
__global__ __launch_bounds__(256) void gemm_direct_kernel(const GemmDesc* __restrict__ descs,
                                                          const int4* __restrict__ tiles) {
    constexpr int BMB = KW ? 32 : 128, BNB = NT * 16;
    __shared__ float red[KW ? 3 * 2 * NT * 4 * 64 : 1];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G2 g = geo2(d);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r16 = lane & 15, kg = (lane >> 4) * 8;
    const int m_w = td.y * BMB + (KW ? 0 : wave * 32);
    const bf16_t* __restrict__ Yact = reinterpret_cast<const bf16_t*>(d.aux);
    const int n0 = td.z * BNB;
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;
    const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ Bw = reinterpret_cast<const bf16_t*>(d.b);

    // per-lane row invariants for the 2 row tiles of this wave
    int base[2], db[2], dih[2], diw[2];
    bool rowok[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int m = m_w + i * 16 + r16;
        rowok[i] = m < g.M;
        base[i] = 0; db[i] = 0; dih[i] = 0; diw[i] = 0;
        if (rowok[i]) {
            if (MODE == MODE_FWD) {
                const int ohw = g.OH * g.OW;
                const int b = m / ohw;
                const int r = m - b * ohw;
                const int oh = r / g.OW, ow = r - (r / g.OW) * g.OW;
                base[i] = ((b * g.H + oh * g.SH) * g.W + ow * g.SW) * g.C;
            } else {
                const int hw = g.H * g.W;
                db[i] = m / hw;
                const int r = m - db[i] * hw;
                dih[i] = r / g.W;
                diw[i] = r - dih[i] * g.W;
            }
        }
    }

    f32x4_t acc[2][NT];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    Frag fa[2], fb[NT];
    auto load = [&](int kt) {
        const int k = kt * 32 + kg;
#pragma unroll
        for (int i = 0; i < 2; ++i)
            fa[i].u = (MODE == MODE_FWD) ? fwd_a(A, g, rowok[i], base[i], k)
                                         : dgrad_a(A, Yact, g, rowok[i], db[i], dih[i], diw[i], k);
#pragma unroll
        for (int j = 0; j < NT; ++j) fb[j].u = row_b(Bw, g.N, g.K, n0 + j * 16 + r16, k);
    };

    const int kfirst = kt0 + (KW ? wave : 0), kstep = KW ? 4 : 1;
    if (kfirst < kt1) load(kfirst);
    for (int kt = kfirst; kt < kt1; kt += kstep) {
        Frag ca[2], cb[NT];
#pragma unroll
        for (int i = 0; i < 2; ++i) ca[i] = fa[i];
#pragma unroll
        for (int j = 0; j < NT; ++j) cb[j] = fb[j];
        if (kt + kstep < kt1) load(kt + kstep);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ca[i].v, cb[j].v, acc[i][j], 0, 0, 0);
    }
    if (KW) {
        // waves 1..3 park their partial sums in LDS, wave 0 reduces and runs the epilogue
        if (wave > 0) {
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        red[((((wave - 1) * 2 + i) * NT + j) * 4 + r) * 64 + lane] = acc[i][j][r];
        }
        __syncthreads();
        if (wave > 0) return;
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[i][j][r] += red[(((w * 2 + i) * NT + j) * 4 + r) * 64 + lane];
    }

    // epilogue: C/D layout col = lane & 15, row = (lane >> 4) * 4 + r
    const int rq = (lane >> 4) * 4;
    const float* bias = reinterpret_cast<const float*>(d.bias);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = n0 + j * 16 + r16;
        if (col >= g.N) continue;
        const float bv = (MODE == MODE_FWD && bias) ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m_w + i * 16 + rq + r;
                if (row >= g.M) continue;
                float v = acc[i][j][r];
                const int64_t off = (int64_t)row * g.N + col;
                if (MODE == MODE_FWD) {
                    v = apply_act(v + bv, g.act);
                    if (g.flags & GF_OUT_F32) {
                        reinterpret_cast<float*>(d.out)[off] = v;
                        continue;
                    }
                }
                bf16_t* o = reinterpret_cast<bf16_t*>(d.out);
                if (g.flags & GF_ACCUM) v += bf2f(o[off]);
                o[off] = f2bf(v);
            }
    }
}

// ==================================================================================================
// WGRAD: dWm[f][k] += sum_m dZ[m][f] * im2col(X)[m][k].  Tile BMF (f) x 64 (k) x 32 (m), 4 waves.
template <int BMF>
__global__ __launch_bounds__(256) void gemm_wgrad_kernel(const GemmDesc* __restrict__ descs,
                                                         const int4* __restrict__ tiles) {
    constexpr int BNK = 64, BKM = 32;
    constexpr int LDA = BMF + 8, LDB = BNK + 8;            // padded rows (elements)
    __shared__ __attribute__((aligned(16))) bf16_t As[BKM * LDA];
    __shared__ __attribute__((aligned(16))) bf16_t Bs[BKM * LDB];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G2 g = geo2(d);                 // WGRAD dims: M = F (rows), N = KH*KW*C (cols), K = B*OH*OW
    const int f0 = td.y * BMF, k0c = td.z * BNK;
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;
    const bf16_t* __restrict__ dZ = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(d.b);
    const bf16_t* __restrict__ Yact = reinterpret_cast<const bf16_t*>(d.aux);
    float* __restrict__ dbias = reinterpret_cast<float*>(d.bias);
    const bool has_bias = dbias != nullptr;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;

    // wave layout: BMF=64 -> 2x2 waves of 32x32; BMF=32 -> 1x4 waves of 32x16; BMF=16 -> 1x4 of 16x16
    constexpr int WR = (BMF == 64) ? 2 : 1;                 // waves along f
    constexpr int WC = 4 / WR;                              // waves along k
    constexpr int TF = BMF / WR / 16;                       // 16-row tiles per wave
    constexpr int TK = BNK / WC / 16;                       // 16-col tiles per wave
    const int wf = wave / WC, wk = wave % WC;

    // loaders: A rows m (32) x f (BMF): chunks of 8 f -> BMF/8 chunks per m
    constexpr int ACH = BMF / 8;
    const bool a_act = t < BKM * ACH;
    const int a_m = a_act ? t / ACH : 0, a_f = (t % ACH) * 8;
    // B rows m (32) x k (64): 8 chunks per m -> 256 threads
    const int b_m = t >> 3, b_k = (t & 7) * 8;

    Frag ra, rb;
    auto load = [&](int kt) {
        const int m0 = kt * BKM;
        ra.u = make_uint4(0, 0, 0, 0);
        if (a_act) {
            const int m = m0 + a_m;
            const int f = f0 + a_f;
            if (m < g.K) {
                const int64_t off = (int64_t)m * g.F + f;
                const bf16_t* src = dZ + off;
                const int nv = min(8, g.F - f);
                if (nv == 8) {
                    ra.u = *reinterpret_cast<const uint4*>(src);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < nv) ra.h[j] = src[j];
                }
                ra.u = act_grad8(ra.u, Yact, off, g.act, nv);
            }
        }
        rb.u = make_uint4(0, 0, 0, 0);
        const int m = m0 + b_m;
        if (m < g.K) {
            const int ohw = g.OH * g.OW;
            const int b = m / ohw;
            const int r = m - b * ohw;
            const int oh = r / g.OW, ow = r - (r / g.OW) * g.OW;
            const int base = ((b * g.H + oh * g.SH) * g.W + ow * g.SW) * g.C;
            G2 gg = g;
            gg.K = g.N;                                       // im2col width
            rb.u = fwd_a(X, gg, true, base, k0c + b_k);
        }
    };
    auto stash = [&]() {
        if (a_act) *reinterpret_cast<uint4*>(&As[a_m * LDA + a_f]) = ra.u;
        *reinterpret_cast<uint4*>(&Bs[b_m * LDB + b_k]) = rb.u;
    };

    f32x4_t acc[TF][TK];
#pragma unroll
    for (int i = 0; i < TF; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    // transposing-read addressing: lane = 16*grp + 4*q + p supplies row (mrow + q), col (col0 + 4p)
    const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;

    // bias gradient: sum_m dZ[m][f], accumulated from the A tiles by the blocks of k-column tile 0
    const bool do_bias = has_bias && td.z == 0;
    float bsum[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bsum[j] = 0.f;

    if (kt0 < kt1) load(kt0);
    for (int kt = kt0; kt < kt1; ++kt) {
        __syncthreads();
        stash();
        if (do_bias) {
#pragma unroll
            for (int j = 0; j < 8; ++j) bsum[j] += bf2f(ra.h[j]);
        }
        __syncthreads();
        if (kt + 1 < kt1) load(kt + 1);
        Frag fa[TF], fbk[TK];
#pragma unroll
        for (int i = 0; i < TF; ++i) {
            const int col = wf * (BMF / WR) + i * 16 + 4 * p;
            const int mr = grp * 8 + q;
            s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(&As[mr * LDA + col]));
            s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(&As[(mr + 4) * LDA + col]));
#pragma unroll
            for (int e = 0; e < 4; ++e) { fa[i].h[e] = (bf16_t)lo[e]; fa[i].h[4 + e] = (bf16_t)hi[e]; }
        }
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            const int col = wk * (BNK / WC) + j * 16 + 4 * p;
            const int mr = grp * 8 + q;
            s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(&Bs[mr * LDB + col]));
            s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
                (__attribute__((address_space(3))) s16x4_t*)(&Bs[(mr + 4) * LDB + col]));
#pragma unroll
            for (int e = 0; e < 4; ++e) { fbk[j].h[e] = (bf16_t)lo[e]; fbk[j].h[4 + e] = (bf16_t)hi[e]; }
        }
#pragma unroll
        for (int i = 0; i < TF; ++i)
#pragma unroll
            for (int j = 0; j < TK; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fbk[j].v, acc[i][j], 0, 0, 0);
    }

    if (do_bias) {
        // lanes of one wave holding the same f chunk differ in the bits >= log2(ACH): butterfly-reduce them
#pragma unroll
        for (int xo = ACH; xo < 64; xo <<= 1)
#pragma unroll
            for (int j = 0; j < 8; ++j) bsum[j] += __shfl_xor(bsum[j], xo, 64);
        if (a_act && lane < ACH) {
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (f0 + a_f + j < g.F) atomicAdd(dbias + f0 + a_f + j, bsum[j]);
        }
    }
    const int c16 = lane & 15, rq = (lane >> 4) * 4;
    float* out = reinterpret_cast<float*>(d.out);
#pragma unroll
    for (int i = 0; i < TF; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            const int col = k0c + wk * (BNK / WC) + j * 16 + c16;
            if (col >= g.N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = f0 + wf * (BMF / WR) + i * 16 + rq + r;
                if (row < g.M) atomicAdd(out + (int64_t)row * g.N + col, acc[i][j][r]);
            }
        }
}

// ==================================================================================================
// Transposed bf16 weights for DGRAD: Wt[c][kh][kw][f] = Wm[f][kh][kw][c], grouped over problems.
struct TransDesc { int64_t src, dst, F, P, C; };   // P = KH*KW

__global__ __launch_bounds__(256) void transpose_weights_kernel(const TransDesc* __restrict__ descs,
                                                                const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const TransDesc& d = descs[td.x];
    const int64_t total = d.F * d.P * d.C;
    const bf16_t* src = reinterpret_cast<const bf16_t*>(d.src);
    bf16_t* dst = reinterpret_cast<bf16_t*>(d.dst);
    const int64_t e0 = (int64_t)td.y * 4096;
    for (int64_t e = e0 + threadIdx.x; e < min(total, e0 + 4096); e += blockDim.x) {
        // e indexes the destination [c][p][f]
        const int64_t f = e % d.F;
        const int64_t rest = e / d.F;
        const int64_t pp = rest % d.P;
        const int64_t c = rest / d.P;
        dst[e] = src[(f * d.P + pp) * d.C + c];
    }
}

void launch_gemm2(int mode, int variant, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipStream_t s = as_stream(stream);
    const GemmDesc* dp = as_ptr<const GemmDesc>(descs);
    const int4* tp = as_ptr<const int4>(tiles);
    dim3 grid((unsigned)ntiles), block(256);
    if (mode == MODE_WGRAD) {
        if (variant == 16) hipLaunchKernelGGL(gemm_wgrad_kernel<16>, grid, block, 0, s, dp, tp);
        else if (variant == 32) hipLaunchKernelGGL(gemm_wgrad_kernel<32>, grid, block, 0, s, dp, tp);
        else hipLaunchKernelGGL(gemm_wgrad_kernel<64>, grid, block, 0, s, dp, tp);
    } else {
        const bool kw = variant >= 1000;
        const int bn = variant % 1000;
#define SERANN_DIRECT(M_, NT_, KW_) hipLaunchKernelGGL((gemm_direct_kernel<M_, NT_, KW_>), grid, block, 0, s, dp, tp)
        if (mode == MODE_FWD) {
            if (kw) { if (bn == 16) SERANN_DIRECT(MODE_FWD, 1, true); else if (bn == 32) SERANN_DIRECT(MODE_FWD, 2, true);
                      else SERANN_DIRECT(MODE_FWD, 4, true); }
            else    { if (bn == 16) SERANN_DIRECT(MODE_FWD, 1, false); else if (bn == 32) SERANN_DIRECT(MODE_FWD, 2, false);
                      else SERANN_DIRECT(MODE_FWD, 4, false); }
        } else {
            if (kw) { if (bn == 16) SERANN_DIRECT(MODE_DGRAD, 1, true); else if (bn == 32) SERANN_DIRECT(MODE_DGRAD, 2, true);
                      else SERANN_DIRECT(MODE_DGRAD, 4, true); }
            else    { if (bn == 16) SERANN_DIRECT(MODE_DGRAD, 1, false); else if (bn == 32) SERANN_DIRECT(MODE_DGRAD, 2, false);
                      else SERANN_DIRECT(MODE_DGRAD, 4, false); }
        }
#undef SERANN_DIRECT
    }
    SERANN_CHECK(hipGetLastError());
}

void launch_transpose_weights(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(transpose_weights_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const TransDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}
