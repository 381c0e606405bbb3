// Grouped implicit-GEMM convolution on CDNA4 MFMA (K01/K02/K04/K07/K09/K10/K11).
//
// Every trainable SeRANN layer -- Dense on the last axis, Conv2D, Conv1D and the two heads -- is an
// NHWC 'valid' convolution (H,W,C) --(KH,KW,SH,SW)--> (OH,OW,F); a Dense layer is the 1x1 case.
// One launch processes one (level, mode) group of *different* problems from many organisms: the
// host builds a tile table (problem, m-tile, n-tile, k-range) and every workgroup looks its tile up,
// so heterogeneous shapes share one launch and fill the 256 CUs.
//
// Modes (weights are stored output-major, Wm[F][KH][KW][C], i.e. [N][K] for the forward GEMM):
//   FWD   : Y[m][f]      = act( sum_k im2col(X)[m][k] * Wm[f][k] + bias[f] )      M=B*OH*OW, N=F, K=KH*KW*C
//   DGRAD : dX[m'][c]    = sum_{kh,kw,f} dZ[b, (ih-kh)/SH, (iw-kw)/SW, f] * Wm[f][kh][kw][c]
//                                                                                 M=B*H*W,   N=C, K=KH*KW*F
//   WGRAD : dWm[f][k]   += sum_m dZ[m][f] * im2col(X)[m][k]                        M=F, N=KH*KW*C, K=B*OH*OW
//           (split-K over m; fp32 atomic accumulation into the gradient arena, zeroed by Adam)
//
// Tile 64x64x32, 256 threads = 4 waves (2x2), each wave 32x32 = 2x2 mfma_f32_16x16x32_bf16 tiles,
// fp32 accumulation.  Operand tiles are staged k-contiguous in LDS ([64][40] bf16: 80-B rows make
// the 16-lane ds_read_b128 fragment reads conflict-free); the next k-tile is prefetched into
// registers while the MFMAs run.  Operand fetch uses 16-B vectors whenever 8 consecutive reduction
// elements are contiguous (flags GF_VEC_A/GF_VEC_B), and per-element gathers otherwise (C=1 inputs,
// odd channel counts).
#include "common.h"
#include "serann_hip.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

namespace {

constexpr int BM = 64, BN = 64, BK = 32, LDSK = BK + 8;

struct Geo {
    int H, W, C, OH, OW, F, KH, KW, SH, SW, M, N, K, act, flags;
};

__device__ __forceinline__ Geo load_geo(const GemmDesc& d) {
    Geo g;
    g.H = (int)d.H; g.W = (int)d.W; g.C = (int)d.C; g.OH = (int)d.OH; g.OW = (int)d.OW; g.F = (int)d.F;
    g.KH = (int)d.KH; g.KW = (int)d.KW; g.SH = (int)d.SH; g.SW = (int)d.SW;
    g.M = (int)d.M; g.N = (int)d.N; g.K = (int)d.K; g.act = (int)d.act; g.flags = (int)d.flags;
    return g;
}

union Pack8 {
    uint4 v;
    bf16_t h[8];
};

// ---- FWD operand fetchers --------------------------------------------------------------------
// im2col element offset of reduction index k for a row with pixel base 'base' (b, oh*SH, ow*SW)
__device__ __forceinline__ int im2col_koff(const Geo& g, int k) {
    int pix = k / g.C;
    int ci = k - pix * g.C;
    int kh = pix / g.KW;
    int kw = pix - kh * g.KW;
    return (kh * g.W + kw) * g.C + ci;
}

__device__ __forceinline__ int im2col_rowbase(const Geo& g, int m) {
    int ohw = g.OH * g.OW;
    int b = m / ohw;
    int r = m - b * ohw;
    int oh = r / g.OW;
    int ow = r - oh * g.OW;
    return ((b * g.H + oh * g.SH) * g.W + ow * g.SW) * g.C;
}

// 8 consecutive k of im2col row m (K-major chunk)
__device__ __forceinline__ uint4 fetch_im2col_kchunk(const bf16_t* __restrict__ x, const Geo& g, int m, int base,
                                                     int k, bool vec) {
    Pack8 p;
    p.v = make_uint4(0, 0, 0, 0);
    if (m >= g.M) return p.v;
    if (vec) {
        if (k < g.K) p.v = *reinterpret_cast<const uint4*>(x + base + im2col_koff(g, k));
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            int kk = k + j;
            if (kk < g.K) p.h[j] = x[base + im2col_koff(g, kk)];
        }
    }
    return p.v;
}

// ---- DGRAD operand fetchers ------------------------------------------------------------------
// A'(m', k') = dZ[b, (ih-kh)/SH, (iw-kw)/SW, f],  k' = (kh*KW + kw)*F + f
__device__ __forceinline__ uint4 fetch_dgrad_a(const bf16_t* __restrict__ dz, const Geo& g, int b, int ih, int iw,
                                               bool mvalid, int k, bool vec) {
    Pack8 p;
    p.v = make_uint4(0, 0, 0, 0);
    if (!mvalid) return p.v;
    if (vec) {
        if (k >= g.K) return p.v;
        int pix = k / g.F;
        int f = k - pix * g.F;
        int kh = pix / g.KW, kw = pix - (pix / g.KW) * g.KW;
        int ohn = ih - kh, own = iw - kw;
        if (ohn < 0 || own < 0) return p.v;
        int oh = ohn / g.SH, ow = own / g.SW;
        if (oh * g.SH != ohn || ow * g.SW != own || oh >= g.OH || ow >= g.OW) return p.v;
        p.v = *reinterpret_cast<const uint4*>(dz + ((b * g.OH + oh) * g.OW + ow) * g.F + f);
        return p.v;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        int kk = k + j;
        if (kk >= g.K) break;
        int pix = kk / g.F;
        int f = kk - pix * g.F;
        int kh = pix / g.KW, kw = pix - (pix / g.KW) * g.KW;
        int ohn = ih - kh, own = iw - kw;
        if (ohn < 0 || own < 0) continue;
        int oh = ohn / g.SH, ow = own / g.SW;
        if (oh * g.SH != ohn || ow * g.SW != own || oh >= g.OH || ow >= g.OW) continue;
        p.h[j] = dz[((b * g.OH + oh) * g.OW + ow) * g.F + f];
    }
    return p.v;
}

}  // namespace

template <int MODE>
__global__ __launch_bounds__(256) void grouped_gemm_kernel(const GemmDesc* __restrict__ descs,
                                                           const int4* __restrict__ tiles) {
    __shared__ __attribute__((aligned(16))) bf16_t As[BM][LDSK];
    __shared__ __attribute__((aligned(16))) bf16_t Bs[BN][LDSK];

    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const Geo g = load_geo(d);
    const int m0 = td.y * BM, n0 = td.z * BN;
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;
    const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ Bp = reinterpret_cast<const bf16_t*>(d.b);
    const bool vecA = g.flags & GF_VEC_A, vecB = g.flags & GF_VEC_B;

    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int wm = wave >> 1, wn = wave & 1;

    // K-major loader coordinates (row, 8-chunk of k)
    const int kr_row = t >> 2, kr_kc = (t & 3) * 8;
    // row-major loader coordinates (k row, 8-chunk of tile rows)
    const int rm_k = t >> 3, rm_rc = (t & 7) * 8;

    // ---- per-thread invariants ---------------------------------------------------------------
    int a_base = 0;         // FWD: im2col row base for row m0+kr_row
    int dg_b = 0, dg_ih = 0, dg_iw = 0;
    bool dg_valid = false;
    if (MODE == MODE_FWD) {
        int m = m0 + kr_row;
        if (m < g.M) a_base = im2col_rowbase(g, m);
    } else if (MODE == MODE_DGRAD) {
        int m = m0 + kr_row;
        dg_valid = m < g.M;
        if (dg_valid) {
            int hw = g.H * g.W;
            dg_b = m / hw;
            int r = m - dg_b * hw;
            dg_ih = r / g.W;
            dg_iw = r - dg_ih * g.W;
        }
    }

    f32x4_t acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    uint4 ra, rb;   // register-staged next tile

    auto fetch = [&](int kt) {
        const int k0 = kt * BK;
        if (MODE == MODE_FWD) {
            ra = fetch_im2col_kchunk(A, g, m0 + kr_row, a_base, k0 + kr_kc, vecA);
            // B[k][n] = Wm[n][k]: K-major chunk of row n
            Pack8 p;
            p.v = make_uint4(0, 0, 0, 0);
            const int n = n0 + kr_row, k = k0 + kr_kc;
            if (n < g.N) {
                const bf16_t* wrow = Bp + (int64_t)n * g.K;
                if (vecB) {
                    if (k < g.K) p.v = *reinterpret_cast<const uint4*>(wrow + k);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (k + j < g.K) p.h[j] = wrow[k + j];
                }
            }
            rb = p.v;
        } else if (MODE == MODE_DGRAD) {
            ra = fetch_dgrad_a(A, g, dg_b, dg_ih, dg_iw, dg_valid, k0 + kr_kc, vecA);
            // B'(k', n'=c) = Wm[f][kh][kw][c]; row-major chunk: k' fixed, 8 consecutive c
            Pack8 p;
            p.v = make_uint4(0, 0, 0, 0);
            const int k = k0 + rm_k, c = n0 + rm_rc;
            if (k < g.K) {
                const int pix = k / g.F;
                const int f = k - pix * g.F;
                const int wk = g.KH * g.KW * g.C;
                const bf16_t* src = Bp + (int64_t)f * wk + pix * g.C;
                if (vecB && c + 8 <= g.N) {
                    p.v = *reinterpret_cast<const uint4*>(src + c);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (c + j < g.N) p.h[j] = src[c + j];
                }
            }
            rb = p.v;
        } else {
            // WGRAD: A''(f, m) = dZ[m][f]  (row-major chunk: m fixed, 8 consecutive f)
            Pack8 pa;
            pa.v = make_uint4(0, 0, 0, 0);
            const int m = k0 + rm_k;
            if (m < g.K) {
                const int f = m0 + rm_rc;
                const bf16_t* src = A + (int64_t)m * g.F;
                if (vecA && f + 8 <= g.M) {
                    pa.v = *reinterpret_cast<const uint4*>(src + f);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (f + j < g.M) pa.h[j] = src[f + j];
                }
            }
            ra = pa.v;
            // B''(m, k) = im2col(X)[m][k]  (row-major chunk: m fixed, 8 consecutive k)
            Pack8 pb;
            pb.v = make_uint4(0, 0, 0, 0);
            if (m < g.K) {
                const int base = im2col_rowbase(g, m);   // note: here g.M/g.N/g.K are the WGRAD dims
                const int kk = n0 + rm_rc;
                if (vecB && kk + 8 <= g.N) {
                    int pix = kk / g.C;
                    int ci = kk - pix * g.C;
                    int kh = pix / g.KW, kw = pix - (pix / g.KW) * g.KW;
                    pb.v = *reinterpret_cast<const uint4*>(Bp + base + (kh * g.W + kw) * g.C + ci);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        int q = kk + j;
                        if (q < g.N) {
                            int pix = q / g.C;
                            int ci = q - pix * g.C;
                            int kh = pix / g.KW, kw = pix - (pix / g.KW) * g.KW;
                            pb.h[j] = Bp[base + (kh * g.W + kw) * g.C + ci];
                        }
                    }
                }
            }
            rb = pb.v;
        }
    };

    auto stash = [&]() {
        if (MODE == MODE_FWD) {
            *reinterpret_cast<uint4*>(&As[kr_row][kr_kc]) = ra;
            *reinterpret_cast<uint4*>(&Bs[kr_row][kr_kc]) = rb;
        } else if (MODE == MODE_DGRAD) {
            *reinterpret_cast<uint4*>(&As[kr_row][kr_kc]) = ra;
            Pack8 p;
            p.v = rb;
#pragma unroll
            for (int j = 0; j < 8; ++j) Bs[rm_rc + j][rm_k] = p.h[j];
        } else {
            Pack8 pa, pb;
            pa.v = ra;
            pb.v = rb;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                As[rm_rc + j][rm_k] = pa.h[j];
                Bs[rm_rc + j][rm_k] = pb.h[j];
            }
        }
    };

    if (kt0 < kt1) fetch(kt0);
    for (int kt = kt0; kt < kt1; ++kt) {
        __syncthreads();
        stash();
        __syncthreads();
        if (kt + 1 < kt1) fetch(kt + 1);
        const int fr = lane & 15, fk = (lane >> 4) * 8;
        bf16x8_t af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
            af[i] = *reinterpret_cast<const bf16x8_t*>(&As[wm * 32 + i * 16 + fr][fk]);
#pragma unroll
        for (int j = 0; j < 2; ++j)
            bfr[j] = *reinterpret_cast<const bf16x8_t*>(&Bs[wn * 32 + j * 16 + fr][fk]);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }

    // ---- epilogue ------------------------------------------------------------------------------
    const int col_l = lane & 15, row_q = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = m0 + wm * 32 + i * 16 + row_q + r;
                const int col = n0 + wn * 32 + j * 16 + col_l;
                if (row >= g.M || col >= g.N) continue;
                float v = acc[i][j][r];
                const int64_t off = (int64_t)row * g.N + col;
                if (MODE == MODE_FWD) {
                    if (d.bias) v += reinterpret_cast<const float*>(d.bias)[col];
                    v = apply_act(v, g.act);
                    if (g.flags & GF_OUT_F32) {
                        reinterpret_cast<float*>(d.out)[off] = v;
                    } else {
                        bf16_t* o = reinterpret_cast<bf16_t*>(d.out);
                        if (g.flags & GF_ACCUM) v += bf2f(o[off]);
                        o[off] = f2bf(v);
                    }
                } else if (MODE == MODE_DGRAD) {
                    bf16_t* o = reinterpret_cast<bf16_t*>(d.out);
                    if (g.flags & GF_ACCUM) v += bf2f(o[off]);
                    o[off] = f2bf(v);
                } else {
                    atomicAdd(reinterpret_cast<float*>(d.out) + off, v);
                }
            }
}

void launch_grouped_gemm(int mode, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipStream_t s = as_stream(stream);
    const GemmDesc* dp = as_ptr<const GemmDesc>(descs);
    const int4* tp = as_ptr<const int4>(tiles);
    dim3 grid((unsigned)ntiles), block(256);
    if (mode == MODE_FWD)
        hipLaunchKernelGGL(grouped_gemm_kernel<MODE_FWD>, grid, block, 0, s, dp, tp);
    else if (mode == MODE_DGRAD)
        hipLaunchKernelGGL(grouped_gemm_kernel<MODE_DGRAD>, grid, block, 0, s, dp, tp);
    else
        hipLaunchKernelGGL(grouped_gemm_kernel<MODE_WGRAD>, grid, block, 0, s, dp, tp);
    SERANN_CHECK(hipGetLastError());
}
