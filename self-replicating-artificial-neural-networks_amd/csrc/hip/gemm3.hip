// Grouped implicit-GEMM convolution, v3 (CDNA4 MFMA) -- the engine's default path.
//
// Measured bottleneck of v2 (gemm2.hip): the im2col / col2im address math, not the MFMAs.  v2
// decomposed every 8-element reduction chunk with two runtime integer divisions (k / C, pix / KW;
// ~20 VALU instructions each -- CDNA has no integer divider) and 64-bit flat addresses, so a
// 16-column tile issued ~10x more VALU cycles than MFMA cycles.  v3:
//  * divisions by problem constants are host-computed magic multiplies (GemmDesc::dv*):
//    q = (umulhi(n, mul) + n) >> shift;
//  * operands are read with raw BUFFER loads: base address and extent in SGPRs (one resource per
//    operand), 32-bit byte offsets per lane, and hardware range checking -- an out-of-range offset
//    returns zeros, which is how invalid DGRAD taps, padded rows and tensor tails are zeroed without
//    selects or branches;
//  * the reduction chunk (kh, kw, c) is decomposed once per lane and k-step and shared by the RT
//    row tiles of the wave (RT = 4: every weight fragment feeds 4 MFMAs), and the k loop is a
//    two-register-set software pipeline (no fragment copies);
//  * chunks are classified by contiguity: the 8 elements are contiguous in memory whenever they stay
//    inside one receptive-field row (KW*C elements); only chunks that wrap to the next kernel row are
//    spliced from a second 16-B load.  Problems with KW*C < 8 (FWD/WGRAD) or F % 8 != 0 on a
//    KHxKW > 1 kernel (DGRAD) -- tiny and rare (mutants) -- use the GEN=true instantiation with
//    element gathers, so the common kernel carries no gather code.
//   FWD   : Y[m][f]  = act(im2col(X)[m][k] . Wm[f][k] + b[f])
//   DGRAD : dX[m][c] = sum_{k'=(kh,kw,f)} dZ[b,(ih-kh)/SH,(iw-kw)/SW,f] . Wt[c][k']
//   WGRAD : dWm[f][k] += sum_m dZ[m][f] . im2col(X)[m][k]      (LDS tiles, transposing LDS reads,
//           64 rows of m per barrier pair, Q40 fixed-point atomics into the gradient arena for split-m)
// dZ = dY * act'(Y) is formed on the fly from the layer output Y (GemmDesc::aux) in DGRAD / WGRAD.
#include <type_traits>

#include "common.h"
#include "serann_hip.h"

#ifndef WG_NSETS
// WGRAD register sets in flight (build-time A/B knob).  One set: 127 VGPRs, 3 waves per SIMD; two sets (the
// round-2 choice): 183 + 36 AGPRs, 2 waves -- one set measured 5.6 vs 5.9 ms (ancestor) and 13.7 vs 13.9 ms
// (generation-3 mix, 4 stream groups) per step (profiles/r4/ab_wgrad_nsets1.txt)
#define WG_NSETS 1
#endif
#ifndef WG_WAVES_PER_EU
#define WG_WAVES_PER_EU 0   // WGRAD occupancy target (build-time A/B knob; 0: the compiler's choice)
#endif
#if WG_WAVES_PER_EU > 0
#define WG_OCC __attribute__((amdgpu_waves_per_eu(WG_WAVES_PER_EU)))
#else
#define WG_OCC
#endif
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;
typedef __attribute__((ext_vector_type(4))) short s16x4_t;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

namespace {

union Frag {
    uint4 u;
    u32x4_t q;
    uint32_t w[4];
    bf16_t h[8];
    bf16x8_t v;
};

// ---- buffer resources ------------------------------------------------------------------------
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int OOB = 0x7ffffff0;                 // byte offset beyond every extent: loads return 0

// Range checking is per load instruction: a 16-B load that crosses num_records returns zeros as a
// whole, so every extent carries 16 B of slack (the engine allocates >= 64 B of slack behind every
// tensor it hands to these kernels; the over-read bytes are masked by splice()).
__device__ __forceinline__ rsrc_t mkrsrc(int64_t ptr, int64_t bytes) {
    bytes = bytes > 0 ? bytes + 16 : 0;
    const int n = bytes > 0x7fff0000LL ? 0x7fff0000 : (int)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(ptr), (short)0, n, 0x00020000);
}
__device__ __forceinline__ uint4 bl16(rsrc_t r, int elem) {       // 8 bf16 at element offset (<0: zeros)
    Frag f;
    f.q = __builtin_amdgcn_raw_buffer_load_b128(r, elem < 0 ? OOB : elem * 2, 0, 0);
    return f.u;
}
__device__ __forceinline__ uint4 bl16b(rsrc_t r, int byteoff) {   // 8 bf16 at a byte offset (OOB: zeros)
    Frag f;
    f.q = __builtin_amdgcn_raw_buffer_load_b128(r, byteoff, 0, 0);
    return f.u;
}
__device__ __forceinline__ bf16_t bl1(rsrc_t r, int elem) {
    return __builtin_amdgcn_raw_buffer_load_b16(r, elem * 2, 0, 0);
}

// ---- fast division ---------------------------------------------------------------------------
struct Div {
    uint32_t mul, sh;
};
__device__ __forceinline__ Div mkdiv(int64_t packed) {
    Div d;
    d.mul = (uint32_t)(packed & 0xffffffffLL);
    d.sh = (uint32_t)((packed >> 32) & 0xff);
    return d;
}
__device__ __forceinline__ int fdiv(int n, const Div& d) {
    return (int)((__umulhi((uint32_t)n, d.mul) + (uint32_t)n) >> d.sh);
}

struct G3 {
    int H, W, C, OH, OW, F, KH, KW, SH, SW, M, N, K, act, flags;
    Div dC, dKW, dOW, dOHW, dF, dW, dHW, dSH, dSW;
};

__device__ __forceinline__ G3 geo3(const GemmDesc& d) {
    G3 g;
    g.H = (int)d.H; g.W = (int)d.W; g.C = (int)d.C; g.OH = (int)d.OH; g.OW = (int)d.OW; g.F = (int)d.F;
    g.KH = (int)d.KH; g.KW = (int)d.KW; g.SH = (int)d.SH; g.SW = (int)d.SW;
    g.M = (int)d.M; g.N = (int)d.N; g.K = (int)d.K; g.act = (int)d.act; g.flags = (int)d.flags;
    g.dC = mkdiv(d.dvC); g.dKW = mkdiv(d.dvKW); g.dOW = mkdiv(d.dvOW); g.dOHW = mkdiv(d.dvOHW);
    g.dF = mkdiv(d.dvF); g.dW = mkdiv(d.dvW); g.dHW = mkdiv(d.dvHW); g.dSH = mkdiv(d.dvSH); g.dSW = mkdiv(d.dvSW);
    return g;
}

// elements j < s from lo, j >= s from hi (s <= 0: all hi, s >= 8: all lo)
__device__ __forceinline__ uint4 splice(uint4 lo, uint4 hi, int s) {
    Frag a, b, r;
    a.u = lo;
    b.u = hi;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const int e0 = 2 * w;
        const uint32_t mixed = (a.w[w] & 0xffffu) | (b.w[w] & 0xffff0000u);
        r.w[w] = (e0 + 1 < s) ? a.w[w] : ((e0 >= s) ? b.w[w] : mixed);
    }
    return r.u;
}

// dZ = dY * act'(Y) on 8 bf16 lanes.  ReLU (the common case) is exact bit logic on 32-bit words
// holding two bf16 lanes -- act' = [Y > 0] -- about six VALU ops per pair instead of two float
// conversions, a select, a multiply and a round-to-nearest per element.  Sigmoid keeps the float path.
// BITS = false keeps the all-float form: the direct-fragment DGRAD kernel measured ~25 % slower with
// the bit form (its register allocation changes), the LDS-tiled and WGRAD kernels faster.
template <bool BITS = true>
__device__ __forceinline__ uint4 mul_act_grad(uint4 dy, uint4 yv, int act) {
    Frag g, y, out;
    g.u = dy;
    y.u = yv;
    if (BITS && act == ACT_RELU) {
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            // per 16-bit half h: low15 + 0x7fff carries into bit 15 iff low15 != 0 (never past it), so
            // bit 15 of t & ~h marks a positive non-zero bf16; (bits >> 15) * 0xffff widens the two
            // marks to two 16-bit lane masks (24-bit multiply: at most 0x10001 * 0xffff)
            const uint32_t yw = y.w[w];
            const uint32_t t = (yw & 0x7fff7fffu) + 0x7fff7fffu;
            const uint32_t pos = (t & ~yw & 0x80008000u) >> 15;
            out.w[w] = g.w[w] & __umul24(pos, 0xffffu);
        }
        return out.u;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) out.h[j] = f2bf(bf2f(g.h[j]) * act_grad_from_y(bf2f(y.h[j]), act));
    return out.u;
}

// Two transposing LDS reads (rows r and r + 4 of a 16-column quad) -> one MFMA fragment.  A vector
// shuffle + bit cast: no per-element moves (an element-wise copy through bf16_t left v_bfi no-ops in
// the MFMA loops).
typedef __attribute__((ext_vector_type(8))) short s16x8_t;
__device__ __forceinline__ bf16x8_t tr_frag(const bf16_t* lo_p, const bf16_t* hi_p) {
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(lo_p));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4_t*)(hi_p));
    const s16x8_t v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8_t, v);
}

// XOR swizzle of an unpadded m-major LDS tile with NB 32-B blocks (16 bf16) per row, read by tr_frag
// (ds_read_b64_tr_b16: two 32-lane groups, each 8 rows {0-3, 8-11} (+4, + 32 per sub-step) x 32 B of one
// column block).  Block L = row * NB + col / 16 moves inside its aligned 256-B group (8 blocks) by a
// function of the group index only (a bijection): the 8 rows of a read group land on the 8 distinct
// 32-B bank blocks of the 256-B bank row, and the 16-B staging stores of 8 consecutive lanes (an aligned
// quad of blocks) keep distinct 128-B bank windows.  Per-NB masks from an exhaustive search over linear
// maps of the group bits (padding rows to 72 / 136 elements, as before, left 2-way conflicts).
template <int NB>
__device__ __forceinline__ int tr_swz_h(int G) {
    static_assert(NB == 1 || NB == 2 || NB == 4 || NB == 6 || NB == 8 || NB == 10 || NB == 12 || NB == 16,
                  "tr_swz: no conflict-free map searched for this row width");
    if constexpr (NB == 1) return (G & 1) << 2;
    else if constexpr (NB == 2 || NB == 6 || NB == 10) return (G >> 1) & 1;
    else if constexpr (NB == 4 || NB == 12) return (G & 1) | ((G >> 1) & 2);
    else if constexpr (NB == 8) return (G & 3) | ((G >> 1) & 4);
    else return ((G >> 1) & 3) | ((G >> 2) & 4);
}
template <int NB>
__device__ __forceinline__ int tr_swz(int row, int col) {
    const int L = row * NB + (col >> 4);
    return ((L ^ tr_swz_h<NB>(L >> 3)) << 4) | (col & 15);
}
// The same map as seen by a lane-linear writer (LDS-DMA: lane i of a wave instruction writes 16-B piece q0 + i):
// physical 16-B piece q holds logical (row, 8-column piece) of block L = P ^ h(P >> 3), P = q >> 1 (the XOR
// only touches the low 3 bits of the block index, so it is its own inverse within the 256-B group)
template <int NB>
__device__ __forceinline__ void tr_swz_piece(int q, int& row, int& col) {
    const int P = q >> 1;
    const int L = P ^ tr_swz_h<NB>(P >> 3);
    row = L / NB;
    col = (L - row * NB) * 16 + (q & 1) * 8;
}

// ---- im2col chunk (FWD A operand, WGRAD B operand) -------------------------------------------
// Per-lane decomposition of the reduction chunk starting at k = (kh, kw, c).
struct KChunk {
    int poff;     // element offset of (kh, kw, c) relative to the receptive field's top-left pixel
    int run;      // elements usable from poff (>= 8: the whole chunk)
    int noff;     // next kernel row's first element minus run (splice source); < 0: none (zeros)
};

__device__ __forceinline__ KChunk im2col_chunk(const G3& g, int k) {
    KChunk r;
    const int rem = g.K - k;
    const int kk = min(k, g.K - 1);
    const int pix = fdiv(kk, g.dC);
    const int c = kk - pix * g.C;
    const int kh = fdiv(pix, g.dKW);
    const int kw = pix - kh * g.KW;
    const int rowrun = (g.KW - kw) * g.C - c;            // elements left in this kernel row
    const bool flat = g.W == g.KW || rowrun >= 8;         // kernel rows adjacent in memory, or no wrap
    r.poff = (kh * g.W + kw) * g.C + c;
    r.run = rem <= 0 ? 0 : (flat ? min(8, rem) : rowrun);
    r.noff = (!flat && kh + 1 < g.KH) ? (kh + 1) * g.W * g.C - rowrun : -1;
    return r;
}

// the chunk's 8 elements for the receptive field at `base` (GEN: KW*C < 8 problems gather)
template <bool GEN>
__device__ __forceinline__ uint4 im2col_load(rsrc_t x, const G3& g, int base, const KChunk& kc, int k) {
    uint4 lo = bl16(x, base + kc.poff);
    if (kc.run < 8) {                                      // K tail / kernel-row wrap (divergent, rare)
        if (GEN && g.KW * g.C < 8) {
            Frag f;
            f.u = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int kk = k + j;
                if (kk < g.K) {
                    const int p = fdiv(kk, g.dC);
                    const int c = kk - p * g.C;
                    const int kh = fdiv(p, g.dKW);
                    const int kw = p - kh * g.KW;
                    f.h[j] = bl1(x, base + (kh * g.W + kw) * g.C + c);
                }
            }
            lo = f.u;
        } else {
            const uint4 hi = kc.noff >= 0 ? bl16(x, base + kc.noff) : make_uint4(0, 0, 0, 0);
            lo = splice(lo, hi, kc.run);
        }
    }
    return lo;
}

// ---- coalesced epilogue ------------------------------------------------------------------------
// A wave's accumulator tile covers rows [row0, row0 + nrows) x ALL N columns of a row-major [M][N]
// bf16 output, i.e. one contiguous range of memory.  The MFMA C layout gives each lane 4 rows of one
// column (2-byte scattered stores), so the tile is first written to LDS in the output's own layout
// (row stride N) and then streamed out with 16-B stores (read-modify-write for GF_ACCUM).  row0 * N
// is a multiple of 16 elements for every caller (row0 is a multiple of 32), so the 16-B chunks are
// aligned.
template <int RT, int NT>
__device__ __forceinline__ void wave_store_rows(bf16_t* __restrict__ st, bf16_t* __restrict__ out, int64_t row0,
                                                int nrows, int N, bool accum, const f32x4_t (&acc)[RT][NT],
                                                const float* __restrict__ bias, int act, int lane) {
    const int r16 = lane & 15, rq = (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = j * 16 + r16;
        if (col >= N) continue;
        const float bv = bias ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = i * 16 + rq + r;
                st[row * N + col] = f2bf(apply_act(acc[i][j][r] + bv, act));
            }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int total = nrows * N;
    const int nvec = total >> 3;
    bf16_t* __restrict__ dst = out + row0 * N;
    for (int v = lane; v < nvec; v += 64) {
        Frag f;
        f.u = *reinterpret_cast<const uint4*>(&st[v * 8]);
        if (accum) {
            Frag o;
            o.u = *reinterpret_cast<const uint4*>(&dst[v * 8]);
#pragma unroll
            for (int e = 0; e < 8; ++e) f.h[e] = f2bf(bf2f(f.h[e]) + bf2f(o.h[e]));
        }
        *reinterpret_cast<uint4*>(&dst[v * 8]) = f.u;
    }
    for (int e = nvec * 8 + lane; e < total; e += 64) {
        float v = bf2f(st[e]);
        if (accum) v += bf2f(dst[e]);
        dst[e] = f2bf(v);
    }
}

}  // namespace


// GF_BNUSTAT (FWD epilogues of the conv-halo, direct, LDS-tiled and shared-input kernels): this output feeds a
// BatchNormalization -- accumulate its phase-0 statistics here, unshifted (K = 0: sum x and sum x^2 of the stored bf16
// values; the BN's flag 512 makes phase 2 finish them in double).  The per-wave partials are fp32 sums of at most
// RT * 16 values before they reach the fixed-point workspace, so E[x^2] - mean^2 keeps ~2^-24 relative error of
// E[x^2]: channels with |mean| >> std lose that much of their variance (tests/test_gpu_kernels.py::
// test_fwd_epilogue_bn_statistics checks both sums against the stored outputs' at |mean| > std; phase 0's shifted
// sums remain the path for outputs that do not take this epilogue).  A
// wave's rows of each accumulator column are summed in fp32 in a fixed order, the waves' partials meet in LDS in
// wave order, and the block adds them to its stripe of the wide fixed-point workspace d.aux: one atomic pair per
// column and sum per block (deterministic).  The block's 4 waves cover WG column groups of NT * 16 columns (wave w:
// group w % WG, at column colblk + (w % WG) * NT * 16); red holds 4 x 2 x WG * NT * 16 floats.  Contains a barrier:
// every thread of the block calls it.
template <int RT, int NT, int WG, typename RowOk>
__device__ __forceinline__ void bn_ustat_flush(const GemmDesc& d, const f32x4_t (&acc)[RT][NT], RowOk row_ok,
                                               int colblk, int ncols, const float* __restrict__ bias, int act,
                                               float* red, int wave, int lane, int C) {
    constexpr int WC = NT * 16, BC = WG * WC;
    const int r16 = lane & 15, rq = (lane >> 4) * 4;
    const int coff = (wave % WG) * WC;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = colblk + coff + j * 16 + r16;
        const float bv = (bias && col < ncols) ? bias[col] : 0.f;
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (row_ok(i, rq + r)) {
                    const float v = bf2f(f2bf(apply_act(acc[i][j][r] + bv, act)));
                    s1 += v;
                    s2 += v * v;
                }
            }
        s1 += __shfl_xor(s1, 16, 64);
        s2 += __shfl_xor(s2, 16, 64);
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (lane < 16) {
            red[(wave * 2 + 0) * BC + coff + j * 16 + lane] = s1;
            red[(wave * 2 + 1) * BC + coff + j * 16 + lane] = s2;
        }
    }
    __syncthreads();
    long long* ws = reinterpret_cast<long long*>(d.aux) + (blockIdx.x % BN_WS_STRIPES) * 4 * C;
    for (int e = threadIdx.x; e < 2 * BC; e += blockDim.x) {
        const int which = e / BC, cl = e - which * BC;
        const int col = colblk + cl;
        if (col >= ncols) continue;
        float v = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w)
            if (w % WG == cl / WC) v += red[(w * 2 + which) * BC + cl];
        fxw_add(ws + 2 * (which * C + col), v);
    }
}

// ==================================================================================================
// FWD / DGRAD direct-fragment kernel.  NT = BN/16 column tiles, RT = 16-row tiles per wave.
//   KW = false: block = 4 waves x RT*16 rows; every wave runs the whole k range.
//   KW = true : block = RT*16 rows; the 4 waves split the k range (k-steps w, w+4, ...) and reduce
//               their accumulators through LDS -- for few-row / long-K problems (merged Dense, heads).
template <int MODE, int NT, int RT, bool KW, bool GEN, bool SK = false>
// Occupancy request by tile size (NT x RT 16-column x 64-row fragments per wave): without it the compiler parks
// accumulators in AGPRs and settles one wave per SIMD lower (e.g. <1, 8, 2>: 138 + 128 registers, 1 wave; with
// it 202, 2 waves; no spills).  Generation-3 mix: 13.73 -> 13.65 ms per step (profiles/r4/ab_direct_occupancy.txt)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NT * RT >= 16 ? 2 : (NT * RT >= 8 ? 3 : 4))))
void g3_direct_kernel(const GemmDesc* __restrict__ descs,
                                                        const int4* __restrict__ tiles) {
    constexpr int WROWS = RT * 16;
    constexpr int BMB = KW ? WROWS : 4 * WROWS, BNB = NT * 16;
    // KW: cross-wave reduction buffer (re-used by wave 0 as the output staging tile);
    // otherwise one output staging tile per wave
    constexpr int RED = KW ? 3 * RT * NT * 4 * 64 : 1;
    constexpr int STAGE = KW ? 1 : 4 * WROWS * BNB;
    __shared__ __attribute__((aligned(16))) float red[RED];
    __shared__ __attribute__((aligned(16))) bf16_t ostage[STAGE];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G3 g = geo3(d);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r16 = lane & 15, kg = (lane >> 4) * 8;
    const int m_w = td.y * BMB + (KW ? 0 : wave * WROWS);
    const int n0 = td.z * BNB;
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;

    // operand extents (elements): FWD A = X[B][H][W][C], DGRAD A = dZ (and Y) [B][OH][OW][F]
    int64_t a_elems;
    if (MODE == MODE_FWD) a_elems = (int64_t)(g.M / (g.OH * g.OW)) * g.H * g.W * g.C;
    else a_elems = (int64_t)(g.M / (g.H * g.W)) * g.OH * g.OW * g.F;
    const rsrc_t rA = mkrsrc(d.a, a_elems * 2);
    const rsrc_t rY = mkrsrc(d.aux, d.aux ? a_elems * 2 : 0);
    const rsrc_t rB = mkrsrc(d.b, (int64_t)g.N * g.K * 2);

    // per-lane row invariants.  Rows >= M only feed accumulator rows that are never stored.
    int base[RT], rb[RT], rih[RT], riw[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        int m = m_w + i * 16 + r16;
        if (m >= g.M) m = 0;
        if (MODE == MODE_FWD) {
            const int b = fdiv(m, g.dOHW);
            const int r = m - b * (g.OH * g.OW);
            const int oh = fdiv(r, g.dOW);
            const int ow = r - oh * g.OW;
            base[i] = ((b * g.H + oh * g.SH) * g.W + ow * g.SW) * g.C;
            rb[i] = rih[i] = riw[i] = 0;
        } else {
            const int b = fdiv(m, g.dHW);
            const int r = m - b * (g.H * g.W);
            rb[i] = b * g.OH;
            rih[i] = fdiv(r, g.dW);
            riw[i] = r - rih[i] * g.W;
            base[i] = 0;
        }
    }
    // B rows: columns n >= N only feed output columns that are never stored (clamped)
    int brow[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) brow[j] = min(n0 + j * 16 + r16, g.N - 1) * g.K;

    f32x4_t acc[RT][NT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    auto load = [&](Frag (&fa)[RT], Frag (&fb)[NT], int kt) {
        const int k = kt * 32 + kg;
        if (MODE == MODE_FWD) {
            const KChunk kc = im2col_chunk(g, k);
#pragma unroll
            for (int i = 0; i < RT; ++i) fa[i].u = im2col_load<GEN>(rA, g, base[i], kc, k);
        } else {
            // k' = (kh*KW + kw)*F + f
            const int rem = g.K - k;
            const int kc = min(k, g.K - 1);
            const int pix = fdiv(kc, g.dF);
            const int f = kc - pix * g.F;
            const int kh = fdiv(pix, g.dKW);
            const int kw = pix - kh * g.KW;
            const int run = rem <= 0 ? 0 : min(8, g.F - f);   // contiguous problems: F%8==0 or 1x1
            if (!GEN || g.F - f >= 8 || g.KH * g.KW == 1) {
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    const int ohn = rih[i] - kh, own = riw[i] - kw;
                    int oh = ohn, ow = own;
                    bool ok = ohn >= 0 && own >= 0;
                    if (g.SH != 1) { oh = fdiv(max(ohn, 0), g.dSH); ok = ok && oh * g.SH == ohn; }
                    if (g.SW != 1) { ow = fdiv(max(own, 0), g.dSW); ok = ok && ow * g.SW == own; }
                    ok = ok && oh < g.OH && ow < g.OW;
                    const int off = ok ? ((rb[i] + oh) * g.OW + ow) * g.F + f : -1;
                    uint4 v = bl16(rA, off);
                    if (g.act != ACT_LINEAR) v = mul_act_grad<false>(v, bl16(rY, off), g.act);
                    fa[i].u = v;
                }
                if (run < 8) {
#pragma unroll
                    for (int i = 0; i < RT; ++i) fa[i].u = splice(fa[i].u, make_uint4(0, 0, 0, 0), run);
                }
            } else {
#pragma unroll
                for (int i = 0; i < RT; ++i) {
                    Frag t;
                    t.u = make_uint4(0, 0, 0, 0);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        const int kk = k + j;
                        if (kk >= g.K) continue;
                        const int p = fdiv(kk, g.dF);
                        const int ff = kk - p * g.F;
                        const int kh2 = fdiv(p, g.dKW);
                        const int kw2 = p - kh2 * g.KW;
                        const int ohn = rih[i] - kh2, own = riw[i] - kw2;
                        int oh = ohn, ow = own;
                        bool ok = ohn >= 0 && own >= 0;
                        if (g.SH != 1) { oh = fdiv(max(ohn, 0), g.dSH); ok = ok && oh * g.SH == ohn; }
                        if (g.SW != 1) { ow = fdiv(max(own, 0), g.dSW); ok = ok && ow * g.SW == own; }
                        ok = ok && oh < g.OH && ow < g.OW;
                        if (!ok) continue;
                        const int off = ((rb[i] + oh) * g.OW + ow) * g.F + ff;
                        float v = bf2f(bl1(rA, off));
                        if (g.act != ACT_LINEAR) v *= act_grad_from_y(bf2f(bl1(rY, off)), g.act);
                        t.h[j] = f2bf(v);
                    }
                    fa[i] = t;
                }
            }
        }
        const int kb = min(k, g.K);
#pragma unroll
        for (int j = 0; j < NT; ++j) fb[j].u = bl16(rB, brow[j] + kb);
        if (k + 8 > g.K) {
#pragma unroll
            for (int j = 0; j < NT; ++j) fb[j].u = splice(fb[j].u, make_uint4(0, 0, 0, 0), g.K - k);
        }
    };
    auto mma = [&](const Frag (&fa)[RT], const Frag (&fb)[NT]) {
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
    };

    if (SK) {
        // K <= 32: one k step, one fragment set (fewer registers -> more resident waves for the
        // store-bound small-K layers)
        Frag fa0[RT], fb0[NT];
        if (kt0 < kt1) {
            load(fa0, fb0, kt0);
            mma(fa0, fb0);
        }
    } else {
        // two-register-set software pipeline: fragments of step s+1 load while step s multiplies.  The
        // loop body is branch-free so the accumulators stay in place (no AGPR shuffles at the latch).
        const int kstep = KW ? 4 : 1;
        const int kfirst = kt0 + (KW ? wave : 0);
        const int nsteps = kfirst < kt1 ? (kt1 - kfirst + kstep - 1) / kstep : 0;
        Frag fa0[RT], fb0[NT], fa1[RT], fb1[NT];
        if (nsteps > 0) load(fa0, fb0, kfirst);
        int st = 0;
        for (; st + 2 < nsteps; st += 2) {
            load(fa1, fb1, kfirst + (st + 1) * kstep);
            mma(fa0, fb0);
            load(fa0, fb0, kfirst + (st + 2) * kstep);
            mma(fa1, fb1);
        }
        if (st + 1 < nsteps) {
            load(fa1, fb1, kfirst + (st + 1) * kstep);
            mma(fa0, fb0);
            mma(fa1, fb1);
        } else if (st < nsteps) {
            mma(fa0, fb0);
        }
    }

    if (KW) {
        if (wave > 0) {
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        red[((((wave - 1) * RT + i) * NT + j) * 4 + r) * 64 + lane] = acc[i][j][r];
        }
        __syncthreads();
        if (wave > 0) return;
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        acc[i][j][r] += red[(((w * RT + i) * NT + j) * 4 + r) * 64 + lane];
    }

    // epilogue: one contiguous output range per wave when the block spans all N columns
    const float* bias = reinterpret_cast<const float*>(d.bias);
    if constexpr (MODE == MODE_FWD && !KW) {
        if (g.flags & GF_BNUSTAT) {
            __shared__ float bnred[4 * 2 * BNB];
            bn_ustat_flush<RT, NT, 1>(d, acc, [&](int i, int rr) { return m_w + i * 16 + rr < g.M; }, n0, g.N, bias,
                                      g.act, bnred, wave, lane, g.N);
        }
    }
    if (n0 == 0 && g.N <= BNB && !(g.flags & GF_OUT_F32)) {
        const int nrows = min(WROWS, g.M - m_w);
        if (nrows > 0) {
            bf16_t* st = KW ? reinterpret_cast<bf16_t*>(red) : &ostage[wave * WROWS * BNB];
            wave_store_rows<RT, NT>(st, reinterpret_cast<bf16_t*>(d.out), m_w, nrows, g.N,
                                    (g.flags & GF_ACCUM) != 0, acc, MODE == MODE_FWD ? bias : nullptr,
                                    MODE == MODE_FWD ? g.act : ACT_LINEAR, lane);
        }
        return;
    }
    // C/D layout col = lane & 15, row = (lane >> 4) * 4 + r
    const int rq = (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = n0 + j * 16 + r16;
        if (col >= g.N) continue;
        const float bv = (MODE == MODE_FWD && bias) ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < RT; ++i)
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

template <int N>
__device__ __forceinline__ void wait_vmcnt() {       // s_waitcnt vmcnt(N) only (gfx9 encoding; expcnt / lgkmcnt max)
    static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}
// Flush of a Dense / 1x1 WGRAD tile (g3_wgrad_kernel, g3_dwgrad_kernel): a lane holds rows frow0 + i * 16 + 4 * (lane / 16)
// + r and columns kcol0 + j * 16 + lane % 16 of its TF x TK accumulator tiles.  Fused Adam (sole writer), plain
// Q40 store (sole writer) or fixed-point atomics (m-split).
// Fused-Adam flush of a sole-writer WGRAD tile (GF_WSTORE | GF_ADAM): the optimizer step applied to the tile, the
// gradient quantised exactly as the Q40 arena would hold it (the arena-wide Adam pass skips these parameters).
// MM: storage of the moment arenas (common.h MOM_*).
template <int MM, int TF, int TK>
__device__ __forceinline__ void wgrad_adam_flush(const GemmDesc& d, const G3& g, f32x4_t (&acc)[TF][TK], int frow0,
                                                 int kcol0, int lane, float* stage, int wave) {
    const int c16 = lane & 15, rq = (lane >> 4) * 4;
    const long long* out = reinterpret_cast<const long long*>(d.out);
    const int ldo = d.ldo ? (int)d.ldo : g.N;
    // every AdamCtx field is read into registers here, before the first store: read through the struct inside
    // the pass loop, each field would be re-loaded after every p / m / v store the compiler cannot prove disjoint
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
    auto chk = [&](float gq, int64_t e) {            // common.h flag_diverged
        if (SERANN_DIVERGE_CHECK && org_off != nullptr && fabsf(gq) > FX_DIVERGE) flag_diverged(org_off, diverged, norg, e);
    };
    if (stage != nullptr) {
        // Row-major through LDS (stage: 2 x TR x LD floats; the k loop's tiles are dead): a lane of the
        // accumulator layout holds 4 rows x 1 column of each 16 x 16 tile, so updating in place read and wrote
        // p / m / v / pbf as 64-B quarter rows, one element per lane per instruction.  Staged, a lane takes 4
        // consecutive columns of one row: 16-B accesses, whole 256-B row segments per 16 lanes, a quarter of the
        // memory instructions.  Two rounds of two waves (the LDS holds two wave tiles).
        constexpr int TR = TF * 16, TC = TK * 16, LD = TC + 4, CG = TC / 4, RPI = 64 / CG;
        const int64_t t0 = e0 + (int64_t)frow0 * ldo + kcol0;
        const bool vec = (t0 & 3) == 0 && (ldo & 3) == 0;      // float4-aligned rows
        const int cg = lane % CG, rr = lane / CG;
        const int col = kcol0 + cg * 4;
        // Software-pipelined one row pass deep: the p / m / v loads of pass it + 1 are issued before pass it's
        // stores (different rows; the compiler cannot hoist them itself over stores through possibly aliasing
        // pointers), and every wave issues its first pass's loads before the LDS rounds, so the second round's
        // loads fly during the first.  (Issuing ALL passes' loads up front -- one round trip -- measured 30 %
        // slower on the ancestor step: those registers cost the k loop its occupancy.)
        using MT = typename std::conditional<MM == MOM_16, uint2, float4>::type;
        const bool vcol = vec && col + 4 <= g.N;
        auto ld_pass = [&](int it, float4& pp, MT& mm, MT& vv) {
            const int row = frow0 + it * RPI + rr;
            if (vcol && row < g.M) {
                const int64_t e = e0 + (int64_t)row * ldo + col;
                pp = *reinterpret_cast<const float4*>(&P[e]);
                if constexpr (MM == MOM_16) {
                    mm = *reinterpret_cast<const uint2*>(reinterpret_cast<const bf16_t*>(Mo) + e);
                    vv = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint16_t*>(Vo) + e);
                } else {
                    mm = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Mo) + e);
                    vv = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Vo) + e);
                }
            }
        };
        float4 pn;
        MT mn, vn;
        ld_pass(0, pn, mn, vn);
        for (int half = 0; half < 2; ++half) {
            __syncthreads();
            if ((wave >> 1) == half) {
                float* st = stage + (wave & 1) * TR * LD;
#pragma unroll
                for (int i = 0; i < TF; ++i)
#pragma unroll
                    for (int j = 0; j < TK; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) st[(i * 16 + rq + r) * LD + j * 16 + c16] = acc[i][j][r];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int it = 0; it < TR / RPI; ++it) {
                    float4 p4 = pn;
                    const MT mr = mn, vr = vn;
                    if (it + 1 < TR / RPI) ld_pass(it + 1, pn, mn, vn);
                    const int row = frow0 + it * RPI + rr;
                    if (row >= g.M || col >= g.N) continue;
                    const float4 gv = *reinterpret_cast<const float4*>(&st[(it * RPI + rr) * LD + cg * 4]);
                    const int64_t e = e0 + (int64_t)row * ldo + col;
                    chk(fmaxf(fmaxf(fabsf(gv.x), fabsf(gv.y)), fmaxf(fabsf(gv.z), fabsf(gv.w))), e);
                    if (vcol) {
                        float4 m4, v4;
                        if constexpr (MM == MOM_16) {
                            m4 = make_float4(__uint_as_float(mr.x << 16), __uint_as_float(mr.x & 0xffff0000u),
                                             __uint_as_float(mr.y << 16), __uint_as_float(mr.y & 0xffff0000u));
                            v4 = make_float4(log16_f(vr.x), log16_f(vr.x >> 16), log16_f(vr.y), log16_f(vr.y >> 16));
                        } else {
                            m4 = mr;
                            v4 = vr;
                        }
                        adam_elem(p4.x, m4.x, v4.x, fx_f(fx_q(gv.x)), lr_t, ac.b1, ac.b2, ac.eps);
                        adam_elem(p4.y, m4.y, v4.y, fx_f(fx_q(gv.y)), lr_t, ac.b1, ac.b2, ac.eps);
                        adam_elem(p4.z, m4.z, v4.z, fx_f(fx_q(gv.z)), lr_t, ac.b1, ac.b2, ac.eps);
                        adam_elem(p4.w, m4.w, v4.w, fx_f(fx_q(gv.w)), lr_t, ac.b1, ac.b2, ac.eps);
                        *reinterpret_cast<float4*>(&P[e]) = p4;
                        m_st4<MM>(Mo, e, m4);
                        v_st4<MM>(Vo, e, v4);
                        *reinterpret_cast<uint2*>(&Pb[e]) = make_uint2(f2bf2(p4.x, p4.y), f2bf2(p4.z, p4.w));
                    } else {
                        const float gq[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q) {
                            if (col + q >= g.N) break;
                            float p_ = P[e + q], m_ = m_ld<MM>(Mo, e + q), v_ = v_ld<MM>(Vo, e + q);
                            adam_elem(p_, m_, v_, fx_f(fx_q(gq[q])), lr_t, ac.b1, ac.b2, ac.eps);
                            P[e + q] = p_; m_st<MM>(Mo, e + q, m_); v_st<MM>(Vo, e + q, v_); Pb[e + q] = f2bf(p_);
                        }
                    }
                }
            }
        }
        return;
    }
    // per 16-row f tile i: every (p, m, v) of the lane's TK x 4 elements is loaded first, then updated
    // and stored -- element by element, each load waited behind the previous element's stores (the
    // compiler cannot move loads over stores through possibly aliasing pointers): up to 32 serial memory
    // round trips per lane in the epilogue, now TF (one batch of TK x 4 x 3 loads in flight each)
#pragma unroll
    for (int i = 0; i < TF; ++i) {
        float pv[TK][4], mv[TK][4], vv[TK][4];
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            const int col = kcol0 + j * 16 + c16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = frow0 + i * 16 + rq + r;
                if (col < g.N && row < g.M) {
                    const int64_t e = e0 + (int64_t)row * ldo + col;
                    pv[j][r] = P[e];
                    mv[j][r] = m_ld<MM>(Mo, e);
                    vv[j][r] = v_ld<MM>(Vo, e);
                }
            }
        }
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            const int col = kcol0 + j * 16 + c16;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = frow0 + i * 16 + rq + r;
                if (col < g.N && row < g.M) {
                    const int64_t e = e0 + (int64_t)row * ldo + col;
                    float p_ = pv[j][r], m_ = mv[j][r], v_ = vv[j][r];
                    chk(acc[i][j][r], e);
                    adam_elem(p_, m_, v_, fx_f(fx_q(acc[i][j][r])), lr_t, ac.b1, ac.b2, ac.eps);
                    P[e] = p_; m_st<MM>(Mo, e, m_); v_st<MM>(Vo, e, v_); Pb[e] = f2bf(p_);
                }
            }
        }
    }
}

template <int TF, int TK>
__device__ __forceinline__ void wgrad_flush(const GemmDesc& d, const G3& g, f32x4_t (&acc)[TF][TK], int frow0,
                                            int kcol0, int lane, float* stage = nullptr, int wave = 0,
                                            float* slab = nullptr) {
    const int c16 = lane & 15, rq = (lane >> 4) * 4;
    long long* out = reinterpret_cast<long long*>(d.out);     // Q40 gradient arena (common.h fx_*)
    const int ldo = d.ldo ? (int)d.ldo : g.N;        // output row stride (a column slice of a wider dW)
    if ((g.flags & (GF_WSTORE | GF_ADAM)) == (GF_WSTORE | GF_ADAM)) {
        if (reinterpret_cast<const AdamCtx*>(d.adam)->mode == MOM_16)
            wgrad_adam_flush<MOM_16, TF, TK>(d, g, acc, frow0, kcol0, lane, stage, wave);
        else
            wgrad_adam_flush<MOM_F32, TF, TK>(d, g, acc, frow0, kcol0, lane, stage, wave);
        return;
    }
    if (stage != nullptr && (slab != nullptr || (g.flags & GF_WSTORE))) {
        // sole writer (of the Q40 tile, or of this split's fp32 slab tile), plain stores: row-major through LDS as the Adam path above, a lane storing 4 consecutive
        // Q40 elements of a row (two 16-B stores) instead of one 8-B element of 4 rows x 1 column
        constexpr int TR = TF * 16, TC = TK * 16, LD = TC + 4, CG = TC / 4, RPI = 64 / CG;
        const bool vec = (reinterpret_cast<uintptr_t>(out + (int64_t)frow0 * ldo + kcol0) & 15) == 0 && (ldo & 1) == 0;
        const int cg = lane % CG, rr = lane / CG;
        for (int half = 0; half < 2; ++half) {
            __syncthreads();
            if ((wave >> 1) == half) {
                float* st = stage + (wave & 1) * TR * LD;
#pragma unroll
                for (int i = 0; i < TF; ++i)
#pragma unroll
                    for (int j = 0; j < TK; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) st[(i * 16 + rq + r) * LD + j * 16 + c16] = acc[i][j][r];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                for (int r0 = 0; r0 < TR; r0 += RPI) {
                    const int row = frow0 + r0 + rr, col = kcol0 + cg * 4;
                    if (row >= g.M || col >= g.N) continue;
                    const float4 gv = *reinterpret_cast<const float4*>(&st[(r0 + rr) * LD + cg * 4]);
                    if (slab != nullptr) {
                        float* o = slab + (int64_t)row * g.N + col;
                        if ((g.N & 3) == 0 && col + 4 <= g.N) {
                            *reinterpret_cast<float4*>(o) = gv;
                        } else {
                            const float gq[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                if (col + q < g.N) o[q] = gq[q];
                        }
                        continue;
                    }
                    long long* o = out + (int64_t)row * ldo + col;
                    if (vec && col + 4 <= g.N) {
                        typedef long long ll2 __attribute__((ext_vector_type(2)));
                        *reinterpret_cast<ll2*>(o) = ll2{fx_q(gv.x), fx_q(gv.y)};
                        *reinterpret_cast<ll2*>(o + 2) = ll2{fx_q(gv.z), fx_q(gv.w)};
                    } else {
                        const float gq[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
                        for (int q = 0; q < 4; ++q)
                            if (col + q < g.N) o[q] = fx_q(gq[q]);
                    }
                }
            }
        }
        return;
    }
#pragma unroll
    for (int i = 0; i < TF; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) {
            const int col = kcol0 + j * 16 + c16;
            if (col >= g.N) continue;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = frow0 + i * 16 + rq + r;
                if (row < g.M) {
                    // GF_WSLAB: m-split -> this split's fp32 slab (plain stores; wgrad_finalize sums the splits in
                    // order); GF_WSTORE: this block is the problem's only m-split -> the sole writer
                    if (slab != nullptr) slab[(int64_t)row * g.N + col] = acc[i][j][r];
                    else if (g.flags & GF_WSTORE) out[(int64_t)row * ldo + col] = fx_q(acc[i][j][r]);
                    else fx_add(out + (int64_t)row * ldo + col, acc[i][j][r]);
                }
            }
        }
}

// ==================================================================================================
// WGRAD: dWm[f][k] += sum_m dZ[m][f] * im2col(X)[m][k].  Tile BMF (f) x BNK (k), 64 rows of m per
// step (two MFMA k-substeps per barrier pair).  Both operands are m-major in memory and are staged
// in LDS in that layout with 16-B writes; MFMA fragments come from ds_read_b64_tr_b16.
template <int BMF, int BNK, bool GEN, int NWV = 4, int RG = 1>
__global__ __launch_bounds__(64 * NWV * RG) WG_OCC void g3_wgrad_kernel(const GemmDesc* __restrict__ descs,
                                                            const int4* __restrict__ tiles) {
    constexpr int BKM = 64;
    constexpr int NTH = 64 * NWV;                    // threads per row group (RG row groups per block)
    constexpr int LDA = BMF, LDB = BNK;              // unpadded rows, XOR-swizzled blocks (tr_swz)
    constexpr int NBA = BMF / 16, NBB = BNK / 16;
    constexpr int SMEM = RG * BKM * (LDA + LDB);     // bf16 elements: one As / Bs pair per row group
    __shared__ __attribute__((aligned(16))) bf16_t smem[SMEM];
    const int rg = threadIdx.x / NTH;
    bf16_t* __restrict__ As = smem + rg * BKM * (LDA + LDB);
    bf16_t* __restrict__ Bs = As + BKM * LDA;
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G3 g = geo3(d);                 // WGRAD dims: M = F (rows), N = KH*KW*C (cols), K = B*OH*OW
    const int f0 = td.y * BMF, k0c = td.z * BNK;
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;   // in units of 32 rows of m
    // Row groups (RG = 2, m-split problems): the block's k range is split into contiguous halves of whole
    // 64-row steps, one per group of NWV waves with its own LDS tiles; the groups' tiles are summed in LDS
    // (group order) before the one flush per block -- half the fixed-point atomics of two separate blocks
    // at the same parallelism.  Every group runs group 0's step count (same barrier sequence); loads past
    // its own range are masked to zeros.  Single-split problems (plain store / fused Adam) keep RG = 1:
    // their 750-row reductions ran 11 % slower per step as two half-length groups (ancestor population).
    const int kh = RG > 1 ? ((kt1 - kt0 + 2 * RG - 1) / (2 * RG)) * 2 : kt1 - kt0;
    const int gk0 = min(kt1, kt0 + rg * kh), gk1 = min(kt1, gk0 + kh);
    const int mlim = min(g.K, gk1 * 32);
    long long* __restrict__ dbias = reinterpret_cast<long long*>(d.bias);   // Q40 gradient arena
    const int t = threadIdx.x - rg * NTH, lane = t & 63, wave = t >> 6;
    const int ohw = g.OH * g.OW;
    const int64_t nb = g.K / ohw;                              // batch
    const rsrc_t rZ = mkrsrc(d.a, (int64_t)g.K * g.F * 2);
    const rsrc_t rY = mkrsrc(d.aux, d.aux ? (int64_t)g.K * g.F * 2 : 0);
    const rsrc_t rX = mkrsrc(d.b, nb * g.H * g.W * g.C * 2);

    // BNK = 16 (layers with <= 16 reduction columns, e.g. Dense on the raw image): the 4 waves split f
    // waves along f (a 128/256-row f tile covering a whole merged-Dense layer was measured 20 % slower
    // per step than 64-row tiles despite reading X once: fewer, heavier blocks)
    constexpr int WR = (BNK == 16) ? 4 : ((BMF >= 64) ? 2 : 1);
    constexpr int WC = NWV / WR;                     // waves along k
    constexpr int TF = BMF / WR / 16;
    constexpr int TK = BNK / WC / 16;
    const int wf = wave / WC, wk = wave % WC;

    // A loader: rows m (64) x f (BMF) in chunks of 8 f (BMF = 160 / 192: 20 / 24 chunks per row, the
    // threads past ACH * AROWS idle)
    constexpr int ACH = BMF / 8;
    constexpr int AROWS = NTH / ACH;                 // rows per pass
    constexpr int APASS = (BKM + AROWS - 1) / AROWS;
    const int a_f = (t % ACH) * 8, a_r = t / ACH;
    const bool a_act = a_r < BKM && t < ACH * AROWS;
    const int a_nv = min(8, g.F - (f0 + a_f));       // valid f of this chunk (may be <= 0)
    // B loader: rows m (64) x k (BNK) in chunks of 8 k; the k chunk is fixed per thread
    constexpr int BCH = BNK / 8;
    constexpr int BROWS = NTH / BCH;
    constexpr int BPASS = (BKM + BROWS - 1) / BROWS;
    const int b_k = (t % BCH) * 8, b_r = t / BCH;
    const int kk = k0c + b_k;
    G3 gx = g;                                       // im2col width is N (= KH*KW*C)
    gx.K = g.N;
    const KChunk kc = im2col_chunk(gx, kk);
    const bool pix1 = g.KH == 1 && g.KW == 1 && g.SH == 1 && g.SW == 1;

    // two register sets: the loads of 64-row step i+1 are issued one full step before step i+1 is
    // staged, so every global load has two MFMA steps (not one) to land -- the loop is load-latency
    // bound for the streaming (many rows, small F x N) problems
    // dY and Y are loaded raw and dZ = dY * act'(Y) is formed when the step is staged: forming it
    // at load time made the wave wait for the loads it had just issued (s_waitcnt vmcnt(0) before the
    // MFMAs of the current step), which defeated the register double buffer
    // Row-affine operands: a load's byte offset is a per-thread constant plus the step's row base
    // m0 * row bytes (one scalar), and rows >= mlim (the next m split) are masked by one compare against
    // a per-thread row key (2^30 for threads without a chunk).  dZ / Y are [K][F] row-major always; X is
    // when the layer is 1x1 stride 1 (row m of the im2col is input row m).  For those, lanes past a
    // row's last column (the next row's data) only feed accumulator columns that are never stored.
    int aoff[APASS], akey[APASS], boff[BPASS], bkey[BPASS];
#pragma unroll
    for (int p = 0; p < APASS; ++p) {
        const int r = a_r + p * AROWS;
        const bool v = a_act && r < BKM && a_nv > 0;
        aoff[p] = (r * g.F + f0 + a_f) * 2;
        akey[p] = v ? r : (1 << 30);
    }
#pragma unroll
    for (int p = 0; p < BPASS; ++p) {
        const int r = b_r + p * BROWS;
        boff[p] = (r * g.C + kk) * 2;
        bkey[p] = (r < BKM && kk < g.N) ? r : (1 << 30);
    }
    Frag ra0[APASS], rb0[BPASS], ra1[APASS], rb1[BPASS], ry0[APASS], ry1[APASS];
    auto load = [&](int kt, Frag (&ra)[APASS], Frag (&ry)[APASS], Frag (&rbv)[BPASS]) {
        const int m0 = kt * 32;
        const int lim = mlim - m0;                   // rows of this step inside the split
        const int sa = m0 * g.F * 2;
#pragma unroll
        for (int p = 0; p < APASS; ++p) {
            const int off = akey[p] < lim ? aoff[p] + sa : OOB;
            ra[p].u = bl16b(rZ, off);
            if (g.act != ACT_LINEAR) ry[p].u = bl16b(rY, off);
        }
        if (pix1) {
            const int sb = m0 * g.C * 2;
#pragma unroll
            for (int p = 0; p < BPASS; ++p) rbv[p].u = bl16b(rX, bkey[p] < lim ? boff[p] + sb : OOB);
            return;
        }
#pragma unroll
        for (int p = 0; p < BPASS; ++p) {
            const int m = m0 + b_r + p * BROWS;
            if (m < mlim && b_r + p * BROWS < BKM) {
                int base;
                if (pix1) {                                // 1x1 stride 1: input row m is output row m
                    base = m * g.C;
                } else {
                    const int b = fdiv(m, g.dOHW);
                    const int r = m - b * ohw;
                    const int oh = fdiv(r, g.dOW);
                    const int ow = r - oh * g.OW;
                    base = ((b * g.H + oh * g.SH) * g.W + ow * g.SW) * g.C;
                }
                rbv[p].u = im2col_load<GEN>(rX, gx, base, kc, kk);
            } else {
                rbv[p].u = make_uint4(0, 0, 0, 0);
            }
        }
    };
    auto stash = [&](Frag (&ra)[APASS], const Frag (&ry)[APASS], const Frag (&rbv)[BPASS]) {
#pragma unroll
        for (int p = 0; p < APASS; ++p) {
            uint4 v = ra[p].u;
            if (g.act != ACT_LINEAR) v = mul_act_grad(v, ry[p].u, g.act);
            if (a_nv < 8) v = splice(v, make_uint4(0, 0, 0, 0), a_nv);
            ra[p].u = v;                                 // (bias_acc reads dZ)
            const int r = a_r + p * AROWS;
            if (a_act && r < BKM) *reinterpret_cast<uint4*>(&As[tr_swz<NBA>(r, a_f)]) = v;
        }
#pragma unroll
        for (int p = 0; p < BPASS; ++p)
            if (b_r + p * BROWS < BKM) *reinterpret_cast<uint4*>(&Bs[tr_swz<NBB>(b_r + p * BROWS, b_k)]) = rbv[p].u;
    };

    f32x4_t acc[TF][TK];
#pragma unroll
    for (int i = 0; i < TF; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const bool do_bias = dbias != nullptr && td.z == 0;
    float bsum[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bsum[j] = 0.f;

    auto compute = [&]() {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            const int mr = sub * 32 + grp * 8 + q;
            bf16x8_t fa[TF], fbk[TK];
#pragma unroll
            for (int i = 0; i < TF; ++i) {
                const int col = wf * (BMF / WR) + i * 16 + 4 * pp;
                fa[i] = tr_frag(&As[tr_swz<NBA>(mr, col)], &As[tr_swz<NBA>(mr + 4, col)]);
            }
#pragma unroll
            for (int j = 0; j < TK; ++j) {
                const int col = wk * (BNK / WC) + j * 16 + 4 * pp;
                fbk[j] = tr_frag(&Bs[tr_swz<NBB>(mr, col)], &Bs[tr_swz<NBB>(mr + 4, col)]);
            }
#pragma unroll
            for (int i = 0; i < TF; ++i)
#pragma unroll
                for (int j = 0; j < TK; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fbk[j], acc[i][j], 0, 0, 0);
        }
    };
    auto bias_acc = [&](const Frag (&ra)[APASS]) {
        if (do_bias) {
#pragma unroll
            for (int p = 0; p < APASS; ++p)
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum[j] += bf2f(ra[p].h[j]);
        }
    };

    // kt counts 32-row units; one step consumes two of them (64 rows); steps rotate over WG_NSETS
    // register sets, so the loads of a step are issued WG_NSETS steps before it is staged
    const int ks = kt0 + rg * kh, ke = ks + kh;      // this group's steps (past gk1: masked loads)
#if WG_NSETS == 2
    if (ks < ke) load(ks, ra0, ry0, rb0);
    if (ks + 2 < ke) load(ks + 2, ra1, ry1, rb1);
    for (int kt = ks; kt < ke; kt += 4) {
        __syncthreads();
        stash(ra0, ry0, rb0);
        bias_acc(ra0);
        __syncthreads();
        if (kt + 4 < ke) load(kt + 4, ra0, ry0, rb0);
        compute();
        if (kt + 2 >= ke) break;
        __syncthreads();
        stash(ra1, ry1, rb1);
        bias_acc(ra1);
        __syncthreads();
        if (kt + 6 < ke) load(kt + 6, ra1, ry1, rb1);
        compute();
    }
#else
    Frag rax[WG_NSETS][APASS], ryx[WG_NSETS][APASS], rbx[WG_NSETS][BPASS];
#pragma unroll
    for (int q_ = 0; q_ < WG_NSETS; ++q_)
        if (ks + 2 * q_ < ke) load(ks + 2 * q_, rax[q_], ryx[q_], rbx[q_]);
    for (int kt = ks; kt < ke; kt += 2 * WG_NSETS) {
#pragma unroll
        for (int q_ = 0; q_ < WG_NSETS; ++q_) {
            const int kc = kt + 2 * q_;
            if (kc >= ke) break;
            __syncthreads();
            stash(rax[q_], ryx[q_], rbx[q_]);
            bias_acc(rax[q_]);
            __syncthreads();
            if (kc + 2 * WG_NSETS < ke) load(kc + 2 * WG_NSETS, rax[q_], ryx[q_], rbx[q_]);
            compute();
        }
    }
#endif
    if constexpr (RG > 1) {
        // group 1 hands its accumulators and bias sums to group 0 through LDS (the tiles are free now)
        constexpr int PER = TF * TK * 4 + 8;
        static_assert(NTH * PER * 4 <= SMEM * 2, "row-group reduction must fit in the LDS tiles");
        static_assert(RG == 2, "two row groups");
        float* red = reinterpret_cast<float*>(smem);
        __syncthreads();
        if (rg == 1) {
#pragma unroll
            for (int i = 0; i < TF; ++i)
#pragma unroll
                for (int j = 0; j < TK; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) red[((i * TK + j) * 4 + r) * NTH + t] = acc[i][j][r];
#pragma unroll
            for (int j = 0; j < 8; ++j) red[(TF * TK * 4 + j) * NTH + t] = bsum[j];
        }
        __syncthreads();
        if (rg == 1) return;
#pragma unroll
        for (int i = 0; i < TF; ++i)
#pragma unroll
            for (int j = 0; j < TK; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) acc[i][j][r] += red[((i * TK + j) * 4 + r) * NTH + t];
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += red[(TF * TK * 4 + j) * NTH + t];
    }

    if (do_bias) {
        if ((ACH & (ACH - 1)) == 0) {
            // lanes of one wave holding the same f chunk differ in the bits >= log2(ACH)
#pragma unroll
            for (int xo = ACH; xo < 64; xo <<= 1)
#pragma unroll
                for (int j = 0; j < 8; ++j) bsum[j] += __shfl_xor(bsum[j], xo, 64);
            if (a_act && lane < ACH) {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (j < a_nv) fx_add(dbias + f0 + a_f + j, bsum[j]);
            }
        } else if (a_act) {
            // non-power-of-two chunk count (BMF = 160 / 192): one atomic per thread and f
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (j < a_nv) fx_add(dbias + f0 + a_f + j, bsum[j]);
        }
    }
    // (the fused-Adam epilogue stages through the LDS tiles when two wave tiles of fp32 fit in them)
    constexpr bool ADAM_STAGE = RG == 1 && NWV == 4 && 2 * (TF * 16) * (TK * 16 + 4) * 4 <= SMEM * 2;
    // GF_WSLAB (m-split): split kt0 / kper's fp32 slab [M][N] at ext (serann_hip.h GF_WSLAB)
    float* slab = (d.flags & GF_WSLAB) ? reinterpret_cast<float*>(d.ext) + (int64_t)(kt0 / (int)d.kper) * g.M * g.N
                                       : nullptr;
    wgrad_flush<TF, TK>(d, g, acc, f0 + wf * (BMF / WR), k0c + wk * (BNK / WC), lane,
                        ADAM_STAGE ? reinterpret_cast<float*>(smem) : nullptr, wave, slab);
}

// ==================================================================================================
// WGRAD of a small filter bank over a long reduction (round 6): F <= 16 filters, N <= 16 NK columns, 1x1 stride-1
// geometry -- the first layers over the shared im2col matrix (F = 8 / 16, N = 9 / 25 / 49 taps, 100k-500k rows) and
// small Dense layers.  The whole [F x N] output is one 16-row MFMA tile, so g3_wgrad_kernel's 64-row f tile left 3 of
// its 4 waves on zero rows, every 64-row step behind two block barriers.  Here each wave walks its own 64-row steps
// (wave w: steps w, w + 4, ... of the block's range) through a wave-private LDS stage (no block barrier in the loop,
// two register sets: a step's loads are issued two of its steps ahead), and the 4 partial tiles and bias sums meet
// in LDS in wave order at the end (deterministic); wave 0 flushes them with g3_wgrad_kernel's epilogue (Q40 store,
// fused Adam, or the split's fp32 slab).
template <int NK>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NK == 1 ? 4 : (NK == 2 ? 3 : 2)))) void g3_wgrad_tiny_kernel(const GemmDesc* __restrict__ descs,
                                                            const int4* __restrict__ tiles) {
    constexpr int BKM = 64, BNK = 16 * NK, AS = BKM * 16, BS = BKM * BNK, BCH = 2 * NK;
    __shared__ __attribute__((aligned(16))) bf16_t smem[4 * (AS + BS)];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G3 g = geo3(d);                 // M = F (<= 16), N (<= BNK) columns, K rows; X row m = im2col row m
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;   // 32-row units
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    bf16_t* __restrict__ As = smem + wave * (AS + BS);
    bf16_t* __restrict__ Bs = As + AS;
    const int mlim = min(g.K, kt1 * 32);
    const rsrc_t rZ = mkrsrc(d.a, (int64_t)g.K * g.F * 2);
    const rsrc_t rY = mkrsrc(d.aux, d.aux ? (int64_t)g.K * g.F * 2 : 0);
    const rsrc_t rX = mkrsrc(d.b, (int64_t)g.K * g.C * 2);
    long long* __restrict__ dbias = reinterpret_cast<long long*>(d.bias);
    // A (dZ, Y): chunk c = lane + 64 p -> row c / 2, filters (c % 2) * 8 .. + 7 (a lane keeps one filter group)
    const int a_f = (lane & 1) * 8, a_nv = min(8, g.F - a_f);
    // B (X): chunk c = lane + 64 p -> row c / BCH, columns (c % BCH) * 8 .. + 7
    // (chunk p of a lane is its chunk 0 moved down 32 / (64 / BCH) rows: one offset and one row key per operand)
    const int arow = a_nv > 0 ? (lane >> 1) : (1 << 30), aoff = ((lane >> 1) * g.F + a_f) * 2;
    const int bcol = (lane % BCH) * 8;
    const int brow = bcol < g.N ? lane / BCH : (1 << 30), boff = ((lane / BCH) * g.C + bcol) * 2;
    constexpr int BRP = 64 / BCH;                     // rows between a lane's B chunks
    const int nst = (kt1 - kt0 + 1) >> 1;             // 64-row steps of the block
    Frag ra0[2], ry0[2], rb0[BCH], ra1[2], ry1[2], rb1[BCH];
    auto load = [&](int s, Frag (&ra)[2], Frag (&ry)[2], Frag (&rb)[BCH]) {
        const int m0 = (kt0 + 2 * s) * 32, lim = mlim - m0;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            const int off = arow + 32 * p < lim ? aoff + (m0 + 32 * p) * g.F * 2 : OOB;
            ra[p].u = bl16b(rZ, off);
            if (g.act != ACT_LINEAR) ry[p].u = bl16b(rY, off);
        }
#pragma unroll
        for (int p = 0; p < BCH; ++p)
            rb[p].u = bl16b(rX, brow + BRP * p < lim ? boff + (m0 + BRP * p) * g.C * 2 : OOB);
    };
    float bsum[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) bsum[j] = 0.f;
    auto stash = [&](Frag (&ra)[2], const Frag (&ry)[2], const Frag (&rb)[BCH]) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
            uint4 v = ra[p].u;
            if (g.act != ACT_LINEAR) v = mul_act_grad(v, ry[p].u, g.act);
            if (a_nv < 8) v = splice(v, make_uint4(0, 0, 0, 0), a_nv);
            Frag f;
            f.u = v;
#pragma unroll
            for (int j = 0; j < 8; ++j) bsum[j] += bf2f(f.h[j]);
            *reinterpret_cast<uint4*>(&As[tr_swz<1>((lane + 64 * p) >> 1, a_f)]) = v;
        }
#pragma unroll
        for (int p = 0; p < BCH; ++p) {
            const int c = lane + 64 * p;
            *reinterpret_cast<uint4*>(&Bs[tr_swz<NK>(c / BCH, (c % BCH) * 8)]) = rb[p].u;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    f32x4_t acc[1][NK];
#pragma unroll
    for (int j = 0; j < NK; ++j) acc[0][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    auto compute = [&]() {
#pragma unroll
        for (int sub = 0; sub < 2; ++sub) {
            const int mr = sub * 32 + grp * 8 + q;
            const bf16x8_t fa = tr_frag(&As[tr_swz<1>(mr, 4 * pp)], &As[tr_swz<1>(mr + 4, 4 * pp)]);
#pragma unroll
            for (int j = 0; j < NK; ++j) {
                const int col = j * 16 + 4 * pp;
                const bf16x8_t fb = tr_frag(&Bs[tr_swz<NK>(mr, col)], &Bs[tr_swz<NK>(mr + 4, col)]);
                acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[0][j], 0, 0, 0);
            }
        }
    };
    if (wave < nst) load(wave, ra0, ry0, rb0);
    if (wave + 4 < nst) load(wave + 4, ra1, ry1, rb1);
    for (int s = wave; s < nst; s += 8) {
        stash(ra0, ry0, rb0);
        if (s + 8 < nst) load(s + 8, ra0, ry0, rb0);
        compute();
        if (s + 4 >= nst) break;
        stash(ra1, ry1, rb1);
        if (s + 12 < nst) load(s + 12, ra1, ry1, rb1);
        compute();
    }
    // bias partials: lanes of one filter group differ in bits 1..5
#pragma unroll
    for (int xo = 2; xo < 64; xo <<= 1)
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += __shfl_xor(bsum[j], xo, 64);
    // the waves' tiles and bias sums meet in LDS (the stages are dead), summed by wave 0 in wave order
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    constexpr int PER = NK * 4 + 8;
    static_assert(3 * PER * 64 * 4 <= 4 * (AS + BS) * 2, "wave reduction must fit in the stages");
    if (wave > 0) {
#pragma unroll
        for (int j = 0; j < NK; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) red[((wave - 1) * PER + j * 4 + r) * 64 + lane] = acc[0][j][r];
#pragma unroll
        for (int j = 0; j < 8; ++j) red[((wave - 1) * PER + NK * 4 + j) * 64 + lane] = bsum[j];
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int w = 0; w < 3; ++w) {
#pragma unroll
        for (int j = 0; j < NK; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[0][j][r] += red[(w * PER + j * 4 + r) * 64 + lane];
#pragma unroll
        for (int j = 0; j < 8; ++j) bsum[j] += red[(w * PER + NK * 4 + j) * 64 + lane];
    }
    if (dbias != nullptr && lane < 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (j < a_nv) fx_add(dbias + a_f + j, bsum[j]);
    }
    float* slab = (d.flags & GF_WSLAB) ? reinterpret_cast<float*>(d.ext) + (int64_t)(kt0 / (int)d.kper) * g.M * g.N
                                       : nullptr;
    wgrad_flush<1, NK>(d, g, acc, 0, 0, lane, nullptr, 0, slab);
}

// ==================================================================================================
// Dense / 1x1 stride-1 WGRAD with an LDS-DMA staging ring (round 5).  Same tiles, splits and flush as
// g3_wgrad_kernel, but the dY (and Y) and X row panels of a 64-row step go global -> LDS by buffer_load ... lds
// (no VGPR staging, no ds_write): each lane of a wave instruction fetches the 16-B piece the XOR-swizzled
// transposing reads expect at its lane-linear LDS slot (tr_swz_piece).  NST - 1 steps of loads stay in flight
// behind the MFMAs; the ring is retired with counted vmcnt waits and raw s_barriers.  act' is applied to the A
// fragments in registers (HASY: the Y tile is staged beside dY).  Requires F % 8 == 0 and C % 8 == 0 (16-B
// pieces never straddle a row; hip_ops.dwgrad_ok).
__host__ __device__ constexpr int dwgrad_stages(int stage_bytes) {
    return 3 * stage_bytes <= 80 * 1024 ? 3 : (4 * stage_bytes <= 160 * 1024 ? 4 : (3 * stage_bytes <= 160 * 1024 ? 3 : 2));
}
template <int BMF, int BNK, bool HASY>
__global__ __launch_bounds__(256) void g3_dwgrad_kernel(const GemmDesc* __restrict__ descs,
                                                        const int4* __restrict__ tiles) {
    constexpr int TM = 64, NBA = BMF / 16, NBB = BNK / 16;
    constexpr int AT = TM * BMF, BT = TM * BNK;                 // bf16 elements of the dY (Y) and X tiles
    constexpr int STG = AT * (HASY ? 2 : 1) + BT;
    constexpr int NST = dwgrad_stages(STG * 2);
    static_assert(NST * STG * 2 <= 160 * 1024, "dense WGRAD stages exceed the LDS");
    constexpr int APC = AT / 8, BPC = BT / 8;                   // 16-B pieces per tile
    static_assert(APC % 64 == 0 && BPC % 256 == 0, "whole wave instructions per tile");
    constexpr int AD = (APC + 255) / 256, BD = BPC / 256;       // DMA instructions per thread and step
    constexpr int PER = AD * (HASY ? 2 : 1) + BD;               // vector-memory ops per thread and step (fixed)
    constexpr int WR = (BMF >= 64) ? 2 : 1, WC = 4 / WR;
    constexpr int TF = BMF / WR / 16, TK = BNK / WC / 16;
    // one __shared__ object per stage, compile-time stage selection (see g3_conv_wgrad_kernel)
    __shared__ __attribute__((aligned(16))) bf16_t sm0[STG];
    __shared__ __attribute__((aligned(16))) bf16_t sm1[STG];
    __shared__ __attribute__((aligned(16))) bf16_t sm2[NST > 2 ? STG : 8];
    __shared__ __attribute__((aligned(16))) bf16_t sm3[NST > 3 ? STG : 8];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G3 g = geo3(d);                 // WGRAD dims: M = F (rows), N = C (cols), K = rows of the batch
    const int f0 = td.y * BMF, k0c = td.z * BNK;
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;   // in units of 32 rows
    const int mb = kt0 * 32, me = min(g.K, kt1 * 32);
    const int nstep = (me - mb + TM - 1) / TM;
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int wf = wave / WC, wk = wave % WC;
    const rsrc_t rZ = mkrsrc(d.a, (int64_t)g.K * g.F * 2);
    const rsrc_t rY = mkrsrc(d.aux, d.aux ? (int64_t)g.K * g.F * 2 : 0);
    const rsrc_t rX = mkrsrc(d.b, (int64_t)g.K * g.C * 2);
    long long* __restrict__ dbias = reinterpret_cast<long long*>(d.bias);   // Q40 gradient arena
    const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;

    // per-thread piece geometry (fixed over the steps; a step adds m0 rows): A / Y pieces, then X pieces
    int aoff[AD], arow[AD], boff[BD], brow[BD];
#pragma unroll
    for (int k = 0; k < AD; ++k) {
        const int q0 = ((k * 4 + wave) * 64) % APC;             // (APC < 256: waves repeat pieces -- same data)
        int r, fc;
        tr_swz_piece<NBA>(q0 + lane, r, fc);
        const bool ok = f0 + fc < g.F;
        aoff[k] = (r * g.F + f0 + fc) * 2;
        arow[k] = ok ? r : (1 << 30);
    }
#pragma unroll
    for (int k = 0; k < BD; ++k) {
        int r, kc;
        tr_swz_piece<NBB>((k * 4 + wave) * 64 + lane, r, kc);
        const bool ok = k0c + kc < g.N;
        boff[k] = (r * g.C + k0c + kc) * 2;
        brow[k] = ok ? r : (1 << 30);
    }
    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    auto issue = [&](int step, bf16_t* const stage) __attribute__((always_inline)) {
        const int m0 = mb + step * TM, lim = me - m0;
#pragma unroll
        for (int k = 0; k < AD; ++k) {
            const int q0 = ((k * 4 + wave) * 64) % APC;
            const int off = arow[k] < lim ? aoff[k] + m0 * g.F * 2 : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rZ, (lds_ptr_t)(stage + q0 * 8), 16, off, 0, 0, 0);
            if constexpr (HASY)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(rY, (lds_ptr_t)(stage + AT + q0 * 8), 16, off, 0, 0, 0);
        }
        bf16_t* const xt = stage + AT * (HASY ? 2 : 1);
#pragma unroll
        for (int k = 0; k < BD; ++k) {
            const int q0 = (k * 4 + wave) * 64;
            const int off = brow[k] < lim ? boff[k] + m0 * g.C * 2 : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_ptr_t)(xt + q0 * 8), 16, off, 0, 0, 0);
        }
    };

    f32x4_t acc[TF][TK];
#pragma unroll
    for (int i = 0; i < TF; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const bool do_bias = dbias != nullptr && td.z == 0 && wk == 0;
    float bsum[TF];
#pragma unroll
    for (int i = 0; i < TF; ++i) bsum[i] = 0.f;

    if (nstep > 0) issue(0, sm0);
    if (NST >= 3 && nstep > 1) issue(1, sm1);
    if (NST >= 4 && nstep > 2) issue(2, sm2);
    auto run_step = [&](int step, const bf16_t* const As, bf16_t* const rdst) __attribute__((always_inline)) {
        const int ahead = min(NST - 2, nstep - 1 - step);       // steps issued after this one (still in flight)
        if (NST >= 4 && ahead >= 2) wait_vmcnt<(NST >= 4 ? 2 * PER : 0)>();
        else if (NST >= 3 && ahead >= 1) wait_vmcnt<(NST >= 3 ? PER : 0)>();
        else wait_vmcnt<0>();
        __builtin_amdgcn_s_barrier();
        // the stage of step - 1 is free (every wave is past its reads): refill it with step + NST - 1
        if (step + NST - 1 < nstep) issue(step + NST - 1, rdst);
        const bf16_t* const Ys = As + AT;
        const bf16_t* const Bs = As + AT * (HASY ? 2 : 1);
#pragma unroll
        for (int sub = 0; sub < TM / 32; ++sub) {
            const int mr = sub * 32 + grp * 8 + q;
            bf16x8_t fa[TF], fb[TK];
#pragma unroll
            for (int i = 0; i < TF; ++i) {
                const int col = wf * (BMF / WR) + i * 16 + 4 * pp;
                bf16x8_t v = tr_frag(&As[tr_swz<NBA>(mr, col)], &As[tr_swz<NBA>(mr + 4, col)]);
                if constexpr (HASY) {
                    const bf16x8_t y = tr_frag(&Ys[tr_swz<NBA>(mr, col)], &Ys[tr_swz<NBA>(mr + 4, col)]);
                    v = __builtin_bit_cast(bf16x8_t, mul_act_grad(__builtin_bit_cast(uint4, v),
                                                                  __builtin_bit_cast(uint4, y), g.act));
                }
                fa[i] = v;
                if (do_bias) {
                    Frag fv;
                    fv.v = v;
#pragma unroll
                    for (int e = 0; e < 8; ++e) bsum[i] += bf2f(fv.h[e]);
                }
            }
#pragma unroll
            for (int j = 0; j < TK; ++j) {
                const int col = wk * (BNK / WC) + j * 16 + 4 * pp;
                fb[j] = tr_frag(&Bs[tr_swz<NBB>(mr, col)], &Bs[tr_swz<NBB>(mr + 4, col)]);
            }
#pragma unroll
            for (int i = 0; i < TF; ++i)
#pragma unroll
                for (int j = 0; j < TK; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
    };
    for (int step = 0; step < nstep; step += NST) {
        run_step(step, sm0, NST == 2 ? sm1 : (NST == 3 ? sm2 : sm3));
        if (step + 1 >= nstep) break;
        run_step(step + 1, sm1, sm0);
        if (NST >= 3) {
            if (step + 2 >= nstep) break;
            run_step(step + 2, sm2, sm1);
        }
        if (NST >= 4) {
            if (step + 3 >= nstep) break;
            run_step(step + 3, sm3, sm2);
        }
    }
    if (do_bias) {
        // lane l holds the 8-row sums of filter l % 16 of each f tile: add the 4 row groups
#pragma unroll
        for (int i = 0; i < TF; ++i) {
            bsum[i] += __shfl_xor(bsum[i], 16, 64);
            bsum[i] += __shfl_xor(bsum[i], 32, 64);
            const int f = f0 + wf * (BMF / WR) + i * 16 + lane;
            if (lane < 16 && f < g.F) fx_add(dbias + f, bsum[i]);
        }
    }
    float* slab = (d.flags & GF_WSLAB) ? reinterpret_cast<float*>(d.ext) + (int64_t)(kt0 / (int)d.kper) * g.M * g.N
                                       : nullptr;
    wgrad_flush<TF, TK>(d, g, acc, f0 + wf * (BMF / WR), k0c + wk * (BNK / WC), lane, nullptr, 0, slab);
}

// ==================================================================================================
// FWD convolution with the input patch staged in LDS ("halo" tile).  A block covers TM = 64*RT
// consecutive output pixels of ONE image (x BN = 16*NT filters): the input rows they touch are one
// contiguous range of the NHWC tensor, copied once into LDS with the channel count padded to
// Cp = ceil8(C) (pad channels zero) and an odd number of 16-B slots per pixel (bank spread).  Every
// A fragment (output pixel x 8 channels of one tap) is then one aligned ds_read_b128 -- the kh*kw-fold
// re-reads of im2col are served by LDS instead of the vector-memory pipeline, and odd channel counts
// no longer produce misaligned global loads.  The reduction runs over (tap, padded channel) in
// 32-element MFMA k-steps; the weights are staged in LDS in chunks of KC k-steps ([BN][KC * 32],
// double-buffered, one barrier and one round of global loads per chunk) shared by the 4 waves.
// PATCH = LDS patch capacity in bf16 elements: 8192 / 16384 / 32768 (16 / 32 / 64 KB; with the weight
// tiles that allows about 8 / 4 / 2 resident blocks per CU).
template <int NT, int RT, int PATCH>
__global__ __launch_bounds__(256) void g3_conv_fwd_kernel(const GemmDesc* __restrict__ descs,
                                                          const int4* __restrict__ tiles) {
    constexpr int TM = 64 * RT, BN = NT * 16;
    // k-steps per weight chunk: the weight buffers stay near 4-5 KB with the 64 KB patch tier (two blocks
    // per CU: 16-KB weight buffers instead, one block per CU, measured slower -- profiles/r5/ab_conv_fwd_kc.txt)
    // and near 17 KB with the smaller tiers
    constexpr int KC = (PATCH >= 32768 ? 4 : 8) / NT;
    constexpr int LDBC = KC * 32 + 8;                   // weight row stride: an odd number of 16-B slots
    // the patch region doubles as the output staging tile after the k loop
    __shared__ __attribute__((aligned(16))) bf16_t patch[PATCH > TM * BN ? PATCH : TM * BN];
    __shared__ __attribute__((aligned(16))) bf16_t Bs[2][BN * LDBC];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G3 g = geo3(d);
    const Div dCp = mkdiv(d.dvCp);
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int r16 = lane & 15, kg = (lane >> 4) * 8;
    const int ohw = g.OH * g.OW;
    const int b = td.y, m0 = td.z, n0 = td.w * BN;
    const int Cp = (g.C + 7) & ~7, C8 = Cp >> 3;
    const int Cs = (C8 & 1) ? Cp : Cp + 8;             // LDS pixel stride (odd count of 16-B slots)
    const int oh_a = fdiv(m0, g.dOW);
    const int m_last = min(m0 + TM, ohw) - 1;
    const int oh_b = fdiv(m_last, g.dOW);
    const int rows_in = (oh_b - oh_a) * g.SH + g.KH;
    const int npix = rows_in * g.W;
    const uint4 zero = make_uint4(0, 0, 0, 0);

    // ---- stage the patch: input rows [oh_a*SH, oh_a*SH + rows_in) of image b ----------------------
    {
        const rsrc_t rA = mkrsrc(d.a, (int64_t)(g.M / ohw) * g.H * g.W * g.C * 2);
        const int gbase = (b * g.H + oh_a * g.SH) * g.W * g.C;
        for (int p = t; p < npix; p += 256) {
            for (int c = 0; c < Cp; c += 8) {
                uint4 v = bl16(rA, gbase + p * g.C + c);
                if (c + 8 > g.C) v = splice(v, zero, g.C - c);
                *reinterpret_cast<uint4*>(&patch[p * Cs + c]) = v;
            }
        }
    }

    // ---- per-lane row offsets into the patch ----------------------------------------------------
    int rowoff[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        int m = m0 + (wave * RT + i) * 16 + r16;
        if (m > m_last) m = m0;
        const int oh = fdiv(m, g.dOW);
        const int ow = m - oh * g.OW;
        rowoff[i] = ((oh - oh_a) * g.SH * g.W + ow * g.SW) * Cs;
    }

    // ---- weight chunks: KC k-steps of the [BN][32] weight tile per LDS buffer (double-buffered) ----
    // One barrier and one round of global loads per chunk instead of per k-step: with 1-4 MFMAs per
    // wave and k-step (BN = 16..64), a per-step barrier with the next step's weights loaded only one step
    // ahead left the loop waiting on load latency (round-3 roofline: 5-8 % MFMA busy, ~1 TB/s).
    const int taps = g.KH * g.KW;
    const int nsteps = (taps * Cp + 31) / 32;
    const int nchunks = (nsteps + KC - 1) / KC;
    const rsrc_t rB = mkrsrc(d.b, (int64_t)g.N * g.K * 2);
    constexpr int PPR = KC * 4;                         // 8-element pieces per weight row and chunk
    constexpr int NPC = BN * PPR / 256;                 // pieces per thread and chunk
    static_assert(NPC * 256 == BN * PPR, "weight chunk must split evenly over the block");
    int brow[NPC], bcol[NPC];
#pragma unroll
    for (int q = 0; q < NPC; ++q) {
        const int pc = t + q * 256;
        const int bn = pc / PPR;
        bcol[q] = (pc - bn * PPR) * 8;
        brow[q] = bn;
    }
    auto gload_chunk = [&](int ch, uint4 (&r)[NPC]) {
#pragma unroll
        for (int q = 0; q < NPC; ++q) {
            const int e = ch * KC * 32 + bcol[q];
            const int tap = fdiv(e, dCp);
            const int c = e - tap * Cp;
            const int n = n0 + brow[q];
            if (n >= g.N || tap >= taps || c >= g.C) {
                r[q] = zero;
            } else {
                uint4 v = bl16(rB, n * g.K + tap * g.C + c);
                if (c + 8 > g.C) v = splice(v, zero, g.C - c);
                r[q] = v;
            }
        }
    };
    auto stash_chunk = [&](int buf, const uint4 (&r)[NPC]) {
#pragma unroll
        for (int q = 0; q < NPC; ++q) *reinterpret_cast<uint4*>(&Bs[buf][brow[q] * LDBC + bcol[q]]) = r[q];
    };

    f32x4_t acc[RT][NT];
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    uint4 breg[NPC];
    gload_chunk(0, breg);
    stash_chunk(0, breg);
    __syncthreads();
    for (int ch = 0; ch < nchunks; ++ch) {
        const int cur = ch & 1;
        if (ch + 1 < nchunks) gload_chunk(ch + 1, breg);
        const int s_end = min(KC, nsteps - ch * KC);
        for (int sl = 0; sl < s_end; ++sl) {
            const int e = (ch * KC + sl) * 32 + kg;
            int tap = fdiv(e, dCp);
            const int c = e - tap * Cp;
            tap = min(tap, taps - 1);                   // past the end: finite A, zero B
            const int kh = fdiv(tap, g.dKW);
            const int kw = tap - kh * g.KW;
            const int tapoff = (kh * g.W + kw) * Cs + c;
            Frag fa[RT], fb[NT];
#pragma unroll
            for (int i = 0; i < RT; ++i) fa[i].u = *reinterpret_cast<const uint4*>(&patch[rowoff[i] + tapoff]);
#pragma unroll
            for (int j = 0; j < NT; ++j)
                fb[j].u = *reinterpret_cast<const uint4*>(&Bs[cur][(j * 16 + r16) * LDBC + sl * 32 + kg]);
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
        }
        if (ch + 1 < nchunks) stash_chunk(cur ^ 1, breg);
        __syncthreads();
    }

    // ---- epilogue ---------------------------------------------------------------------------------
    const float* bias = reinterpret_cast<const float*>(d.bias);
    bf16_t* o = reinterpret_cast<bf16_t*>(d.out);
    const int64_t rowbase = (int64_t)b * ohw;
    if (g.flags & GF_BNUSTAT) {
        __shared__ float bnred[4 * 2 * BN];
        bn_ustat_flush<RT, NT, 1>(d, acc, [&](int i, int rr) { return m0 + (wave * RT + i) * 16 + rr <= m_last; },
                                  n0, g.N, bias, g.act, bnred, wave, lane, g.N);
    }
    if (n0 == 0 && g.N <= BN && !(g.flags & GF_OUT_F32)) {
        // the block's rows are consecutive pixels of one image: contiguous output rows
        const int mw = m0 + wave * RT * 16;
        const int nrows = min(RT * 16, m_last + 1 - mw);
        if (nrows > 0)
            wave_store_rows<RT, NT>(&patch[wave * RT * 16 * BN], o, rowbase + mw, nrows, g.N,
                                    (g.flags & GF_ACCUM) != 0, acc, bias, g.act, lane);
        return;
    }
    const int rq = (lane >> 4) * 4;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        const int col = n0 + j * 16 + r16;
        if (col >= g.N) continue;
        const float bv = bias ? bias[col] : 0.f;
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int m = m0 + (wave * RT + i) * 16 + rq + r;
                if (m > m_last) continue;
                const int64_t off = (rowbase + m) * g.N + col;
                float v = apply_act(acc[i][j][r] + bv, g.act);
                if (g.flags & GF_OUT_F32) {
                    reinterpret_cast<float*>(d.out)[off] = v;
                    continue;
                }
                if (g.flags & GF_ACCUM) v += bf2f(o[off]);
                o[off] = f2bf(v);
            }
    }
}

// ==================================================================================================
// WGRAD of a KHxKW > 1 convolution with the input patch staged in LDS, as tap-shifted GEMMs.
//   dWm[f][tap][c] += sum_m dZ[m][f] * X[patch(m) + shift(tap)][c]
// A block owns BMF filters x BNK columns of the padded (tap, Cp) reduction space and sweeps a range of
// 128-pixel chunks [td.z, td.w) (chunk = (image, pixel tile)).  Every wave holds ALL TF = BMF / 16 filter
// tiles and NTW = BNK / 64 column tiles (columns j*64 + 16*wave of the block).  Per 32-row MFMA k step a
// wave reads its TF dZ fragments once; its column tiles are then pure LDS base shifts of one per-row patch
// address: tap (kh, kw) of output pixel m is input pixel patch(m) + kh * W + kw, so a B fragment is two
// ds_read_b64_tr_b16 at (row address + column offset) -- no per-lane im2col division, no restaging per
// column tile.  Stride 2 is the same loop (patch(m) carries the stride).
// Staging is an NST-deep ring of LDS stages filled by LDS-DMA (buffer_load ... lds: no VGPRs, no ds_write):
// the patch (padded channels: pixel p at p * Cs, an odd number of 16-B slots per pixel; pad slots and pixels
// past the patch load out of range = zeros), the raw dY tile and the Y tile (act' is applied to the A fragments
// in registers), and the per-row patch offsets.  Chunk ch + NST - 1 is issued while chunk ch is computed, so
// NST - 1 chunks of loads are in flight behind the MFMAs (a one-deep register prefetch left the loop waiting
// on load latency: ~3.5 us per chunk against ~0.5 us of MFMAs on a 16-filter problem).  Every DMA count is
// fixed per chunk, so the ring is retired with counted vmcnt waits and raw s_barriers (a __syncthreads would
// drain every DMA in flight).  Accumulators stay in registers across chunks; the flush writes fp32 split slabs
// (or the Q40 gradient of a single split); the bias gradient is reduced from the dZ fragments by wave 0 of
// the blocks of column range 0.
// Small outputs (OH*OW < 128, e.g. a 7x7 conv on an 11x11 map: 25 pixels) would leave most of a
// 128-row chunk empty, so a chunk then covers ipc = min(128 / (OH*OW), PATCH / (H*W*Cs)) whole
// consecutive images when ipc >= 2 (their input images are one contiguous NHWC range; hip_ops
// conv_wgrad_ipc mirrors the rule for the tile table).
// LDS-DMA stages of the conv WGRAD ring: 3 when two blocks of them fit a CU's 160 KB (latency hidden by two blocks
// and two chunks in flight each), else as many as one block can hold (at most 4, at least 2)
// Channel stride of a conv WGRAD patch pixel: Cp rounded up to an odd number of 16-B slots.  The 8 rows a
// ds_read_b64_tr_b16 lane group reads are 8 consecutive output pixels (conv_wgrad_row_pixel); at a stride of an
// odd number of 16-B slots their 32-B windows overlap at most once in the 256-B bank row.  (A stride with
// SW * Cs = 16 (mod 32), which tiles the bank row exactly, measured no faster and grows the patch up to 50 %:
// profiles/r5/cwg_isolated_*.log.)  hip_ops.conv_wgrad_cs mirrors it.
__host__ __device__ constexpr int conv_wgrad_cs(int Cp, int SW) {
    return ((Cp >> 3) & 1) ? Cp : Cp + 8;
}
// Pixel (relative to the chunk's first) of logical row r of a conv WGRAD chunk: inside each 32-row k step the rows
// a transposing read takes together -- {g * 8 + h * 4 + q : g in {0, 1} or {2, 3}, q < 4} for read h -- are 8
// consecutive pixels.  dY rows and patch row offsets use the same map, so the MFMA sums the same pairs.
__device__ __forceinline__ int conv_wgrad_row_pixel(int r) {
    const int g = (r >> 3) & 3, h = (r >> 2) & 1;
    return (r & ~31) | ((g >> 1) << 4) | (h << 3) | ((g & 1) << 2) | (r & 3);
}
constexpr int conv_wgrad_stages(int stage_bytes) {
    return 3 * stage_bytes <= 80 * 1024 ? 3
           : (4 * stage_bytes <= 160 * 1024 ? 4 : (3 * stage_bytes <= 160 * 1024 ? 3 : 2));
}
template <int BMF, int BNK, int PATCH>
__global__ __launch_bounds__(256) void g3_conv_wgrad_kernel(const GemmDesc* __restrict__ descs,
                                                            const int4* __restrict__ tiles) {
    constexpr int TM = 128, NBA = BMF / 16;
    constexpr int TF = BMF / 16, NTW = BNK / 64;
    static_assert(BNK % 256 == 0 || BNK == 128, "column tiles: NTW in {2, 4, 8, 16, 32}");
    constexpr int DYT = TM * BMF;                         // bf16 elements of the dY (and of the Y) tile
    constexpr int STG = PATCH + 2 * DYT;                  // stage: patch, dY, Y (+ the row offsets, TM ints, apart)
    constexpr int NST = conv_wgrad_stages(STG * 2 + TM * 4);
    static_assert(NST * (STG * 2 + TM * 4) <= 160 * 1024, "conv WGRAD stages exceed the LDS");
    constexpr int PD = PATCH / 2048;                      // patch DMAs per thread and chunk (16-B pieces / 256)
    constexpr int AD = DYT / 2048;                        // dY DMAs per thread and chunk (as many Y DMAs)
    constexpr int PER = PD + 2 * AD;                      // vector-memory ops per thread and chunk (fixed)
    // One __shared__ object per ring stage, and the chunk loop unrolled by NST so every stage is a compile-time
    // object: the compiler's wait-count pass then sees that a chunk's LDS reads cannot alias the LDS-DMA refilling
    // another stage.  (With one array indexed by a runtime stage it put s_waitcnt vmcnt(0) in front of every k
    // step's reads -- each refill's loads were waited for as soon as they were issued.)
    __shared__ __attribute__((aligned(16))) bf16_t sm0[STG];
    __shared__ __attribute__((aligned(16))) bf16_t sm1[STG];
    __shared__ __attribute__((aligned(16))) bf16_t sm2[NST > 2 ? STG : 8];
    __shared__ __attribute__((aligned(16))) bf16_t sm3[NST > 3 ? STG : 8];
    // the per-stage row offsets are objects of their own too: written with ds_write, they would otherwise share an
    // object with the stage's LDS-DMA and wait for it
    __shared__ int rt0[TM], rt1[TM], rt2[NST > 2 ? TM : 1], rt3[NST > 3 ? TM : 1];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const G3 g = geo3(d);                 // WGRAD dims: M = F (rows), N = KH*KW*C (cols), K = B*OH*OW
    const Div dCp = mkdiv(d.dvCp);
    // (the wave index through readfirstlane: wave-uniform in an SGPR, so per-wave values are scalar)
    const int t = threadIdx.x, lane = t & 63, wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int f0 = (td.y >> 16) * BMF, kc0 = (td.y & 0xffff) * BNK;
    const int ohw = g.OH * g.OW;
    const int tpi = (ohw + TM - 1) / TM;
    const int Cp = (g.C + 7) & ~7, C8 = Cp >> 3;
    const int Cs = conv_wgrad_cs(Cp, g.SW), Cs8 = Cs >> 3;
    // q / Cs8 for slot indices q < 2^12 (PATCH / 8): (q * mCs) >> 17, mCs = ceil(2^17 / Cs8), exact for Cs8 <= 32;
    // wider channels use the generic magic (fdiv)
    const uint32_t mCs = (131072u + Cs8 - 1) / (uint32_t)Cs8;
    const bool small_cs = Cs8 <= 32;
    Div dCs8;
    {
        const uint32_t dv = (uint32_t)Cs8;
        uint32_t sh = 0;
        while ((1u << sh) < dv) ++sh;
        dCs8.mul = (uint32_t)(((1ull << 32) * ((1ull << sh) - dv)) / dv + 1);
        dCs8.sh = sh;
    }
    const int taps = g.KH * g.KW;
    const int nbatch = g.K / ohw;
    const int hwcs = g.H * g.W * Cs;
    const int ipc_full = ohw < TM ? min(TM / ohw, PATCH / hwcs) : 0;
    const bool multi = ipc_full >= 2;            // chunk = ipc whole images
    auto chunk_geom = [&](int ch, int& b, int& m0, int& m_last) {
        if (multi) {
            b = ch * ipc_full;
            m0 = 0;
            m_last = min(ipc_full, nbatch - b) * ohw - 1;
        } else {
            b = ch / tpi;
            m0 = (ch - b * tpi) * TM;
            m_last = min(m0 + TM, ohw) - 1;
        }
    };
    const rsrc_t rX = mkrsrc(d.b, (int64_t)nbatch * g.H * g.W * g.C * 2);
    const rsrc_t rZ = mkrsrc(d.a, (int64_t)g.K * g.F * 2);
    const rsrc_t rY = mkrsrc(d.aux, d.aux ? (int64_t)g.K * g.F * 2 : 0);
    long long* __restrict__ dbias = reinterpret_cast<long long*>(d.bias);   // Q40 gradient arena
    const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
    const bool has_act = g.act != ACT_LINEAR;

    // column tiles of this wave: block column kc0 + (j * 4 + wave) * 16; valid ones first, nvj of them
    const int ncolt = min(4 * NTW, (taps * Cp - kc0 + 15) >> 4);
    const int nvj = ncolt > wave ? (ncolt - wave + 3) >> 2 : 0;
    int coff[NTW];
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int kp = kc0 + (j * 4 + wave) * 16 + 4 * pp;
        int tap = fdiv(kp, dCp);
        const int c = kp - tap * Cp;
        tap = min(tap, taps - 1);
        const int kh = fdiv(tap, g.dKW);
        const int kw = tap - kh * g.KW;
        coff[j] = (kh * g.W + kw) * Cs + c;
    }
    const bool do_bias = dbias != nullptr && kc0 == 0 && wave == 0;
    float bsum[TF];
#pragma unroll
    for (int i = 0; i < TF; ++i) bsum[i] = 0.f;
    f32x4_t acc[TF][NTW];
#pragma unroll
    for (int i = 0; i < TF; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    typedef __attribute__((address_space(3))) void* lds_ptr_t;
    // Issue every load of chunk ch into stage st: exactly PER buffer_load ... lds per thread (pieces past the
    // patch / tile load out of range: zeros), and the stage's row offsets (ds_write, ordered by the barrier
    // that precedes the stage's use).
    // part: the loads are issued in 4 parts (part < 0: all at once), one per 32-row k step of the chunk being
    // computed, so their issue cost (~60 cycles per LDS-DMA) interleaves with MFMAs
    auto issue = [&](int ch, bf16_t* const stage, int* const rtab, int part) __attribute__((always_inline)) {
        int b, m0, m_last;
        chunk_geom(ch, b, m0, m_last);
        int npix, gbase, oh_a = 0;
        if (multi) {
            npix = (m_last / ohw + 1) * g.H * g.W;       // whole images
            gbase = b * g.H * g.W * g.C;
        } else {
            oh_a = fdiv(m0, g.dOW);
            const int oh_b = fdiv(m_last, g.dOW);
            npix = ((oh_b - oh_a) * g.SH + g.KH) * g.W;
            gbase = (b * g.H + oh_a * g.SH) * g.W * g.C;
        }
        constexpr int PQ = (PD + 3) / 4;
        const int k0 = part < 0 ? 0 : part * PQ, k1 = part < 0 ? PD : min(PD, (part + 1) * PQ);
#pragma unroll
        for (int k = 0; k < PD; ++k) {
            if (k < k0 || k >= k1) continue;
            const int q0 = (k * 4 + wave) * 64;          // wave-uniform first slot of this instruction
            const int qq = q0 + lane;
            const int p = small_cs ? (int)(((uint32_t)qq * mCs) >> 17) : fdiv(qq, dCs8);
            const int c8 = qq - p * Cs8;
            const int off = (p < npix && c8 < C8) ? (gbase + p * g.C + c8 * 8) * 2 : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rX, (lds_ptr_t)(stage + q0 * 8), 16, off, 0, 0, 0);
        }
        if (part > 0) return;
        bf16_t* const dyt = stage + PATCH;
#pragma unroll
        for (int k = 0; k < AD; ++k) {
            const int q0 = (k * 4 + wave) * 64;
            int r, fc;
            tr_swz_piece<NBA>(q0 + lane, r, fc);        // the logical piece the swizzled reads expect here
            const int m = m0 + conv_wgrad_row_pixel(r);
            const int off = (m <= m_last && f0 + fc < g.F) ? ((b * ohw + m) * g.F + f0 + fc) * 2 : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rZ, (lds_ptr_t)(dyt + q0 * 8), 16, off, 0, 0, 0);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rY, (lds_ptr_t)(dyt + DYT + q0 * 8), 16, has_act ? off : OOB,
                                                     0, 0, 0);
        }
        if (t < TM) {
            // row offsets (rows past the chunk end read a valid pixel: their dZ rows are zero)
            int m = m0 + conv_wgrad_row_pixel(t);
            if (m > m_last) m = m0;
            const int j = multi ? fdiv(m, g.dOHW) : 0;     // image inside the chunk
            const int pm = m - j * ohw;
            const int oh = fdiv(pm, g.dOW);
            const int ow = pm - oh * g.OW;
            rtab[t] = j * hwcs + ((oh - oh_a) * g.SH * g.W + ow * g.SW) * Cs;
        }
    };

    const int z = td.z, w = td.w;
    if (z < w) issue(z, sm0, rt0, -1);
    if (NST >= 3 && z + 1 < w) issue(z + 1, sm1, rt1, -1);
    if (NST >= 4 && z + 2 < w) issue(z + 2, sm2, rt2, -1);
    // one chunk: its loads retired, then 4 k steps on stage cur while stage rdst (chunk ch - 1's) is refilled
    auto chunk = [&](int ch, const bf16_t* const patch, const int* const rt, bf16_t* const rdst, int* const rtdst)
                     __attribute__((always_inline)) {
        // retire chunk ch's loads: the chunks issued after it (at most NST - 2) stay in flight
        const int ahead = min(NST - 2, w - 1 - ch);
        if (NST >= 4 && ahead >= 2) wait_vmcnt<(NST >= 4 ? 2 * PER : 0)>();
        else if (NST >= 3 && ahead >= 1) wait_vmcnt<(NST >= 3 ? PER : 0)>();
        else wait_vmcnt<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");              // row offsets written
        __builtin_amdgcn_s_barrier();
        // the stage of chunk ch - 1 is free now (every wave is past its reads): refill it, a quarter per k step
        const bool refill = ch + NST - 1 < w;
        const bf16_t* const dyt = patch + PATCH;
        const bf16_t* const yt = dyt + DYT;
#pragma unroll
        for (int sub = 0; sub < TM / 32; ++sub) {
            if (refill) issue(ch + NST - 1, rdst, rtdst, sub);
            const int mr = sub * 32 + grp * 8 + q;
            const bf16_t* p0 = patch + rt[mr];
            const bf16_t* p1 = patch + rt[mr + 4];
            bf16x8_t fa[TF];
#pragma unroll
            for (int i = 0; i < TF; ++i) {
                const int col = i * 16 + 4 * pp;
                bf16x8_t v = tr_frag(&dyt[tr_swz<NBA>(mr, col)], &dyt[tr_swz<NBA>(mr + 4, col)]);
                if (has_act) {
                    const bf16x8_t y = tr_frag(&yt[tr_swz<NBA>(mr, col)], &yt[tr_swz<NBA>(mr + 4, col)]);
                    v = __builtin_bit_cast(bf16x8_t, mul_act_grad(__builtin_bit_cast(uint4, v),
                                                                  __builtin_bit_cast(uint4, y), g.act));
                }
                fa[i] = v;
                if (do_bias) {
                    Frag fv;
                    fv.v = v;
#pragma unroll
                    for (int e = 0; e < 8; ++e) bsum[i] += bf2f(fv.h[e]);
                }
            }
            // every column tile of the block, branch-free (tiles past the reduction read a valid address; the
            // flush drops them): the B fragments of group g + 1 (4 tiles) are read while group g's MFMAs run
            constexpr int JG = NTW < 4 ? NTW : 4, NG = NTW / JG;
            bf16x8_t fb[2][JG];
#pragma unroll
            for (int jj = 0; jj < JG; ++jj) fb[0][jj] = tr_frag(p0 + coff[jj], p1 + coff[jj]);
#pragma unroll
            for (int gq = 0; gq < NG; ++gq) {
                if (gq + 1 < NG) {
#pragma unroll
                    for (int jj = 0; jj < JG; ++jj) {
                        const int j = (gq + 1) * JG + jj;
                        fb[(gq + 1) & 1][jj] = tr_frag(p0 + coff[j], p1 + coff[j]);
                    }
                }
#pragma unroll
                for (int jj = 0; jj < JG; ++jj)
#pragma unroll
                    for (int i = 0; i < TF; ++i)
                        acc[i][gq * JG + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[gq & 1][jj],
                                                                                     acc[i][gq * JG + jj], 0, 0, 0);
            }
        }
    };
    // stage of chunk z + k: k mod NST; the refilled stage is the previous chunk's
    for (int ch = z; ch < w; ch += NST) {
        chunk(ch, sm0, rt0, NST == 2 ? sm1 : (NST == 3 ? sm2 : sm3), NST == 2 ? rt1 : (NST == 3 ? rt2 : rt3));
        if (ch + 1 >= w) break;
        chunk(ch + 1, sm1, rt1, sm0, rt0);
        if (NST >= 3) {
            if (ch + 2 >= w) break;
            chunk(ch + 2, sm2, rt2, sm1, rt1);
        }
        if (NST >= 4) {
            if (ch + 3 >= w) break;
            chunk(ch + 3, sm3, rt3, sm2, rt2);
        }
    }

    if (do_bias) {
        // lane l holds the 8-row sums of filter l % 16 of each f tile: add the 4 row groups
#pragma unroll
        for (int i = 0; i < TF; ++i) {
            bsum[i] += __shfl_xor(bsum[i], 16, 64);
            bsum[i] += __shfl_xor(bsum[i], 32, 64);
            const int f = f0 + i * 16 + lane;
            if (lane < 16 && f < g.F) fx_add(dbias + f, bsum[i]);
        }
    }
    // Flush.  Split problems (d.ext = fp32 slab workspace [S][M][taps * Cp], split = td.z / d.kper): plain
    // stores of the block's partial tile in the padded column space; the grouped wgrad_finalize launch adds
    // the splits in order (no fixed-point atomics: at 16 x 1024 columns per block they were ~30x the MFMA
    // time).  A single split (GF_WSTORE) stores the Q40 gradient dWm[f][tap * C + c] itself.
    const int c16 = lane & 15, rq = (lane >> 4) * 4;
    if (d.ext) {
        const int ldp = taps * Cp;
        float* __restrict__ slab = reinterpret_cast<float*>(d.ext) + (int64_t)(td.z / (int)d.kper) * g.M * ldp;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int kp = kc0 + (j * 4 + wave) * 16 + c16;
            if (j >= nvj || kp >= ldp) continue;
#pragma unroll
            for (int i = 0; i < TF; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = f0 + i * 16 + rq + r;
                    if (row < g.M) slab[(int64_t)row * ldp + kp] = acc[i][j][r];
                }
        }
        return;
    }
    long long* out = reinterpret_cast<long long*>(d.out);
    const bool sole = g.flags & GF_WSTORE;
#pragma unroll
    for (int j = 0; j < NTW; ++j) {
        const int kp = kc0 + (j * 4 + wave) * 16 + c16;
        const int tap = fdiv(kp, dCp);
        const int c = kp - tap * Cp;
        if (j >= nvj || tap >= taps || c >= g.C) continue;
        const int col = tap * g.C + c;
#pragma unroll
        for (int i = 0; i < TF; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = f0 + i * 16 + rq + r;
                if (row < g.M) {
                    if (sole) out[(int64_t)row * g.N + col] = fx_q(acc[i][j][r]);
                    else fx_add(out + (int64_t)row * g.N + col, acc[i][j][r]);
                }
            }
    }
}

// ==================================================================================================
// Narrow layers: 1x1 / Dense problems with K <= 4 reduction channels (X_Dense on the raw image, or on a
// conv output with 1-4 filters).  There is nothing for MFMA to do -- K is 1..4 -- and the work is pure
// streaming of the wide [M][N] tensor, so these are VALU kernels with 16-B accesses: a thread keeps 8
// consecutive output channels (their K weights / gradient partial sums in registers) and walks rows.
constexpr int NARROW_ROWS = 256;        // FWD rows per block
constexpr int NARROW_WROWS = 1024;      // WGRAD rows per block

// ST (output channels N % 8 != 0, e.g. Dense(units=75) on the raw genotype): the rows are computed
// into an LDS tile and leave as one contiguous range with 16-B stores -- the row stride N is not a
// multiple of 8, so per-thread 16-B row chunks are not aligned and the plain path stores 2-B elements.
constexpr int NARROW_SROWS = 64;        // FWD staged pass: 64 x 256 bf16 = 32 KB of LDS, i.e.
                                        // (64 * 256 / N) & ~7 rows of N channels (<= NARROW_ROWS)
template <int K, bool ST>
__global__ __launch_bounds__(256) void g3_narrow_fwd_kernel(const GemmDesc* __restrict__ descs,
                                                            const int4* __restrict__ tiles) {
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const int M = (int)d.M, N = (int)d.N, act = (int)d.act;
    const int ldx = (int)d.C;                    // X row stride (= K, or K8 for the shared raw im2col)
    const int FC = (N + 7) >> 3;                 // 8-channel chunks per row (<= 32: N <= 256)
    const int RPI = 256 / FC;
    const int t = threadIdx.x;
    const bool active = t < RPI * FC;
    // GF_BNSTAT: this output feeds a BatchNormalization -- accumulate its phase-0 statistics here
    // (shifted sums against row 0's value, exactly what bn phase 0 would read) into aux[c], aux[N + c]
    const bool bnstat = (d.flags & GF_BNSTAT) != 0;
    const bool store = (d.flags & GF_NOSTORE) == 0;
    if (!ST && !bnstat && !active) return;
    const int chunk = t % FC, rl = t / FC;
    const int f0 = chunk * 8;
    const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ Wm = reinterpret_cast<const bf16_t*>(d.b);
    const float* bias = reinterpret_cast<const float*>(d.bias);
    bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(d.out);
    float w[8][K], bv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int f = min(f0 + j, N - 1);
        bv[j] = bias ? bias[f] : 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) w[j][k] = bf2f(Wm[f * K + k]);
    }
    float ks[8], s1[8], s2[8];                   // BN shift (row 0's output) and partial sums
#pragma unroll
    for (int j = 0; j < 8; ++j) { ks[j] = 0.f; s1[j] = 0.f; s2[j] = 0.f; }
    if (bnstat) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float v = bv[j];
#pragma unroll
            for (int k = 0; k < K; ++k) v += bf2f(X[k]) * w[j][k];
            ks[j] = store ? bf2f(f2bf(apply_act(v, act))) : apply_act(v, act);
        }
    }
    // statistics of what the BN will read: the stored bf16 output, or (GF_NOSTORE: nbn.hip recomputes it)
    // the fp32 value
    auto stat = [&](int j, bf16_t o, float yf) {
        if (bnstat) {
            const float dv = (store ? bf2f(o) : yf) - ks[j];
            s1[j] += dv;
            s2[j] += dv * dv;
        }
    };
    const bool vec = (N & 7) == 0;
    const int r0 = td.y * NARROW_ROWS, r1 = min(M, r0 + NARROW_ROWS);
    constexpr int U = 4;                         // rows in flight per thread
    if constexpr (ST) {
        __shared__ __attribute__((aligned(16))) bf16_t st[NARROW_SROWS * 256];
        // rows per pass: fill the buffer (N = 75: 216 rows, 2 passes per block instead of 4); a multiple
        // of 8 rows keeps every pass's first element 16-B aligned
        const int srows = min(NARROW_ROWS, ((NARROW_SROWS * 256) / N) & ~7);
        for (int p0 = r0; p0 < r1; p0 += srows) {
            const int p1 = min(r1, p0 + srows);
            if (active) {
                for (int rb = p0 + rl; rb < p1; rb += U * RPI) {
                    float xv[U][K];
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int r = min(rb + u * RPI, p1 - 1);
#pragma unroll
                        for (int k = 0; k < K; ++k) xv[u][k] = bf2f(X[(int64_t)r * ldx + k]);
                    }
#pragma unroll
                    for (int u = 0; u < U; ++u) {
                        const int r = rb + u * RPI;
                        if (r >= p1) break;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            if (f0 + j >= N) break;
                            float v = bv[j];
#pragma unroll
                            for (int k = 0; k < K; ++k) v += xv[u][k] * w[j][k];
                            const float yf = apply_act(v, act);
                            const bf16_t o = f2bf(yf);
                            stat(j, o, yf);
                            st[(r - p0) * N + f0 + j] = o;
                        }
                    }
                }
            }
            __syncthreads();
            // rows [p0, p1) are one contiguous range; p0 * N * 2 B is a multiple of 16 B
            const int total = (p1 - p0) * N, nvec = total >> 3;
            bf16_t* __restrict__ dst = Y + (int64_t)p0 * N;
            if (store) {
                for (int v = t; v < nvec; v += 256)
                    *reinterpret_cast<uint4*>(dst + 8 * v) = *reinterpret_cast<const uint4*>(&st[8 * v]);
                for (int e = nvec * 8 + t; e < total; e += 256) dst[e] = st[e];
            }
            __syncthreads();
        }
    } else if (active) {
        for (int rb = r0 + rl; rb < r1; rb += U * RPI) {
            float xv[U][K];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = min(rb + u * RPI, r1 - 1);
#pragma unroll
                for (int k = 0; k < K; ++k) xv[u][k] = bf2f(X[(int64_t)r * ldx + k]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = rb + u * RPI;
                if (r >= r1) break;
                union { uint4 u4; bf16_t h[8]; } o;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float v = bv[j];
#pragma unroll
                    for (int k = 0; k < K; ++k) v += xv[u][k] * w[j][k];
                    const float yf = apply_act(v, act);
                    o.h[j] = f2bf(yf);
                    if (f0 + j < N) stat(j, o.h[j], yf);
                }
                bf16_t* dst = Y + (int64_t)r * N + f0;
                if (!store) {
                } else if (vec) {
                    *reinterpret_cast<uint4*>(dst) = o.u4;
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (f0 + j < N) dst[j] = o.h[j];
                }
            }
        }
    }
    if (bnstat) {
        // combine the RPI row lanes of every (chunk, channel) through LDS; one atomic pair per channel
        __shared__ float red[2 * 8 * 256];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            red[j * 256 + t] = active ? s1[j] : 0.f;
            red[(8 + j) * 256 + t] = active ? s2[j] : 0.f;
        }
        __syncthreads();
        long long* ws = reinterpret_cast<long long*>(d.aux) + (blockIdx.x % BN_WS_STRIPES) * 4 * N;   // stripe
        for (int o = t; o < FC * 8; o += 256) {
            const int ch = o >> 3, j = o & 7, c = ch * 8 + j;
            if (c >= N) continue;
            float a = 0.f, b = 0.f;
            for (int q = 0; q < RPI; ++q) {
                a += red[j * 256 + q * FC + ch];
                b += red[(8 + j) * 256 + q * FC + ch];
            }
            fxw_add(ws + 2 * c, a);
            fxw_add(ws + 2 * (N + c), b);
        }
    }
}

// ST (F % 8 != 0): dY / Y rows are staged through LDS 16 rows at a time with contiguous 16-B loads (the
// plain path loads 2-B elements when the row stride F is not a multiple of 8); the staging buffers alias
// the reduction array, which is used only after the row loop.
constexpr int NARROW_WSROWS = 16;
template <int K, bool ST>
__global__ __launch_bounds__(256) void g3_narrow_wgrad_kernel(const GemmDesc* __restrict__ descs,
                                                              const int4* __restrict__ tiles) {
    // WGRAD dims: M = F (rows of dW), N = K (columns), K = reduction rows; dZ = dY * act'(Y)
    constexpr int NA = 8 * (K + 1);               // per-thread partials: 8 x K weights + 8 biases
    __shared__ float red[256 * NA];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const int F = (int)d.M, R = (int)d.K, act = (int)d.act;
    const int ldx = (int)d.C;                    // X row stride (= K, or K8 for the shared raw im2col)
    const int FC = (F + 7) >> 3;
    const int RPI = 256 / FC;
    const int t = threadIdx.x;
    const bool active = t < RPI * FC;
    const int chunk = t % FC, rl = t / FC;
    const int f0 = chunk * 8;
    const bf16_t* __restrict__ dY = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(d.b);
    const bf16_t* __restrict__ Yv = reinterpret_cast<const bf16_t*>(d.aux);
    long long* dbias = reinterpret_cast<long long*>(d.bias);   // Q40 gradient arena
    float acc[NA];
#pragma unroll
    for (int j = 0; j < NA; ++j) acc[j] = 0.f;
    const bool vec = (F & 7) == 0;
    const int r0 = td.y * NARROW_WROWS, r1 = min(R, r0 + NARROW_WROWS);
    if constexpr (ST) {
        static_assert(2 * NARROW_WSROWS * 256 * 2 <= 256 * NA * 4, "staging must fit in the reduction array");
        bf16_t* sg = reinterpret_cast<bf16_t*>(red);
        bf16_t* sy = sg + NARROW_WSROWS * 256;
        // rows per pass: fill the 16 x 256 staging buffers (F = 75: 48 rows per pass instead of 16 -- each
        // pass is one 16-B load per thread between two barriers, so short passes are latency-bound)
        const int srows = max(8, ((NARROW_WSROWS * 256) / F) & ~7);
        for (int p0 = r0; p0 < r1; p0 += srows) {
            const int p1 = min(r1, p0 + srows);
            const int total = (p1 - p0) * F, nvec = total >> 3;
            // p0 * F * 2 B is a multiple of 16 B: aligned 16-B loads of the contiguous row range
            const bf16_t* gsrc = dY + (int64_t)p0 * F;
            const bf16_t* ysrc = Yv + (int64_t)p0 * F;
            for (int v = t; v < nvec; v += 256) {
                *reinterpret_cast<uint4*>(&sg[8 * v]) = *reinterpret_cast<const uint4*>(gsrc + 8 * v);
                if (act != ACT_LINEAR)
                    *reinterpret_cast<uint4*>(&sy[8 * v]) = *reinterpret_cast<const uint4*>(ysrc + 8 * v);
            }
            for (int e = nvec * 8 + t; e < total; e += 256) {
                sg[e] = gsrc[e];
                if (act != ACT_LINEAR) sy[e] = ysrc[e];
            }
            __syncthreads();
            if (active) {
                for (int r = p0 + rl; r < p1; r += RPI) {
                    float xv[K];
#pragma unroll
                    for (int k = 0; k < K; ++k) xv[k] = bf2f(X[(int64_t)r * ldx + k]);
                    const int base = (r - p0) * F + f0;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        if (f0 + j >= F) break;
                        float gz = bf2f(sg[base + j]);
                        if (act != ACT_LINEAR) gz = bf2f(f2bf(gz * act_grad_from_y(bf2f(sy[base + j]), act)));
#pragma unroll
                        for (int k = 0; k < K; ++k) acc[j * K + k] += gz * xv[k];
                        acc[8 * K + j] += gz;
                    }
                }
            }
            __syncthreads();
        }
    } else if (active) {
        constexpr int U = 4;                     // rows in flight per thread
        for (int rb = r0 + rl; rb < r1; rb += U * RPI) {
            union V8 { uint4 u; bf16_t h[8]; };
            V8 g[U], y[U];
            float xv[U][K];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int r = rb + u * RPI;
                const bool ok = r < r1;
                const int rr = ok ? r : r0;
                const bf16_t* src = dY + (int64_t)rr * F + f0;
                const bf16_t* ysrc = Yv + (int64_t)rr * F + f0;
                if (vec) {
                    g[u].u = *reinterpret_cast<const uint4*>(src);
                    if (act != ACT_LINEAR) y[u].u = *reinterpret_cast<const uint4*>(ysrc);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        g[u].h[j] = f0 + j < F ? src[j] : (bf16_t)0;
                        if (act != ACT_LINEAR) y[u].h[j] = f0 + j < F ? ysrc[j] : (bf16_t)0;
                    }
                }
                if (!ok) g[u].u = make_uint4(0, 0, 0, 0);
#pragma unroll
                for (int k = 0; k < K; ++k) xv[u][k] = bf2f(X[(int64_t)rr * ldx + k]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float gz = bf2f(g[u].h[j]);
                    if (act != ACT_LINEAR) gz = bf2f(f2bf(gz * act_grad_from_y(bf2f(y[u].h[j]), act)));
#pragma unroll
                    for (int k = 0; k < K; ++k) acc[j * K + k] += gz * xv[u][k];
                    acc[8 * K + j] += gz;
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < NA; ++j) red[j * 256 + t] = active ? acc[j] : 0.f;
    __syncthreads();
    // combine the RPI row lanes of every (chunk, partial) and flush
    for (int o = t; o < FC * NA; o += 256) {
        const int ch = o / NA, j = o - ch * NA;
        float v = 0.f;
        for (int q = 0; q < RPI; ++q) v += red[j * 256 + q * FC + ch];
        if (j < 8 * K) {
            const int f = ch * 8 + j / K, k = j % K;
            if (f < F) fx_add(reinterpret_cast<long long*>(d.out) + (int64_t)f * K + k, v);
        } else {
            const int f = ch * 8 + (j - 8 * K);
            if (dbias && f < F) fx_add(dbias + f, v);
        }
    }
}

// "Super-row" (SR) forms of the narrow kernels for a row width W = N (FWD) or F (WGRAD) that is not a
// multiple of 8 (W > 8).  The [rows][W] tensor is walked in super-rows of 8 rows = W chunks of 8
// elements; thread i of a super-row always takes chunk i, so its 8 elements always belong to the same
// channels (8i + j) mod W and lie in rows ro[j] = (8i + j) / W of the super-row (at most two distinct
// rows, W > 8).  Every global access is an aligned 16-B vector, there is no LDS staging and no barrier
// in the row loop, the per-channel weights and partial sums stay in registers, and channels are
// combined once per block through LDS (slot g * 8W + 8i + j holds channel (8i + j) mod W of super-row
// group g -- the BatchNorm bn_vec layout).
constexpr int NARROW_SR_U = 4;          // super-rows in flight per thread

template <int K>
__global__ __launch_bounds__(256) void g3_narrow_fwd_sr_kernel(const GemmDesc* __restrict__ descs,
                                                               const int4* __restrict__ tiles) {
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const int M = (int)d.M, N = (int)d.N, act = (int)d.act;
    const int ldx = (int)d.C;
    const int t = threadIdx.x, G = 256 / N, q = t / N, i = t - q * N;
    const bool active = q < G;
    const bool bnstat = (d.flags & GF_BNSTAT) != 0;
    const bool store = (d.flags & GF_NOSTORE) == 0;
    const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ Wm = reinterpret_cast<const bf16_t*>(d.b);
    const float* bias = reinterpret_cast<const float*>(d.bias);
    bf16_t* __restrict__ Y = reinterpret_cast<bf16_t*>(d.out);
    int ch[8], ro[8];
    float w[8][K], bv[8], ks[8], s1[8], s2[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        const int e = 8 * i + j;
        ch[j] = e % N;
        ro[j] = e / N;
        bv[j] = bias ? bias[ch[j]] : 0.f;
#pragma unroll
        for (int k = 0; k < K; ++k) w[j][k] = bf2f(Wm[ch[j] * K + k]);
        s1[j] = 0.f;
        s2[j] = 0.f;
        ks[j] = 0.f;
        if (bnstat) {              // BN phase-0 shift: row 0's output (what bn phase 0 would read)
            float v = bv[j];
#pragma unroll
            for (int k = 0; k < K; ++k) v += bf2f(X[k]) * w[j][k];
            ks[j] = store ? bf2f(f2bf(apply_act(v, act))) : apply_act(v, act);
        }
    }
    const int64_t total = (int64_t)M * N;
    // rows per block: NARROW_ROWS, or d.kper (a multiple of 8) for a statistics-only pass (GF_NOSTORE: ~nothing to
    // do per row, so the per-block weight setup and statistics flush would dominate 256-row blocks)
    const int rpb = d.kper ? (int)d.kper : NARROW_ROWS;
    const int r0 = td.y * rpb, r1 = min(M, r0 + rpb);
    const int sr0 = r0 / 8, sr1 = (r1 + 7) / 8;
    if (active) {
        constexpr int U = NARROW_SR_U;
        for (int sb = sr0 + q; sb < sr1; sb += U * G) {
            float xa[U][K], xb[U][K];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int sr = min(sb + u * G, sr1 - 1);
                const int ra = min(M - 1, sr * 8 + ro[0]), rb = min(M - 1, ra + 1);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    xa[u][k] = bf2f(X[(int64_t)ra * ldx + k]);
                    xb[u][k] = bf2f(X[(int64_t)rb * ldx + k]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int sr = sb + u * G;
                const int64_t e = (int64_t)sr * 8 * N + 8 * i;
                const int nv = sr < sr1 ? (int)max((int64_t)0, min((int64_t)8, total - e)) : 0;
                if (nv <= 0) continue;
                union { uint4 u4; bf16_t h[8]; } o;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool hi = ro[j] != ro[0];
                    float v = bv[j];
#pragma unroll
                    for (int k = 0; k < K; ++k) v += (hi ? xb[u][k] : xa[u][k]) * w[j][k];
                    const float yf = apply_act(v, act);
                    o.h[j] = f2bf(yf);
                    if (bnstat && j < nv) {
                        const float dv = (store ? bf2f(o.h[j]) : yf) - ks[j];
                        s1[j] += dv;
                        s2[j] += dv * dv;
                    }
                }
                if (!store) {
                } else if (nv == 8) {
                    *reinterpret_cast<uint4*>(Y + e) = o.u4;
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < nv) Y[e + j] = o.h[j];
                }
            }
        }
    }
    if (bnstat) {
        __shared__ float red[2 * 2048];
        if (active) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                red[q * 8 * N + 8 * i + j] = s1[j];
                red[2048 + q * 8 * N + 8 * i + j] = s2[j];
            }
        }
        __syncthreads();
        long long* ws = reinterpret_cast<long long*>(d.aux) + (blockIdx.x % BN_WS_STRIPES) * 4 * N;   // stripe
        for (int c = t; c < N; c += 256) {
            float a = 0.f, b = 0.f;
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int m = 0; m < 8; ++m) {
                    a += red[g * 8 * N + c + m * N];
                    b += red[2048 + g * 8 * N + c + m * N];
                }
            fxw_add(ws + 2 * c, a);
            fxw_add(ws + 2 * (N + c), b);
        }
    }
}

template <int K>
__global__ __launch_bounds__(256) void g3_narrow_wgrad_sr_kernel(const GemmDesc* __restrict__ descs,
                                                                 const int4* __restrict__ tiles) {
    // WGRAD dims: M = F (rows of dW), N = K (columns), K = reduction rows; dZ = dY * act'(Y)
    __shared__ float red[(K + 1) * 2048];
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const int F = (int)d.M, R = (int)d.K, act = (int)d.act;
    const int ldx = (int)d.C;
    const int t = threadIdx.x, G = 256 / F, q = t / F, i = t - q * F;
    const bool active = q < G;
    const bf16_t* __restrict__ dY = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ X = reinterpret_cast<const bf16_t*>(d.b);
    const bf16_t* __restrict__ Yv = reinterpret_cast<const bf16_t*>(d.aux);
    long long* dbias = reinterpret_cast<long long*>(d.bias);   // Q40 gradient arena
    int ro[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) ro[j] = (8 * i + j) / F;
    float acc[8 * (K + 1)];
#pragma unroll
    for (int j = 0; j < 8 * (K + 1); ++j) acc[j] = 0.f;
    const int64_t total = (int64_t)R * F;
    const int r0 = td.y * NARROW_WROWS, r1 = min(R, r0 + NARROW_WROWS);
    const int sr0 = r0 / 8, sr1 = (r1 + 7) / 8;
    if (active) {
        constexpr int U = NARROW_SR_U;
        union V8 { uint4 u; bf16_t h[8]; };
        for (int sb = sr0 + q; sb < sr1; sb += U * G) {
            V8 g[U], y[U];
            float xa[U][K], xb[U][K];
            int nv[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int sr = sb + u * G;
                const int64_t e = (int64_t)sr * 8 * F + 8 * i;
                nv[u] = sr < sr1 ? (int)max((int64_t)0, min((int64_t)8, total - e)) : 0;
                g[u].u = make_uint4(0, 0, 0, 0);
                y[u].u = make_uint4(0, 0, 0, 0);
                if (nv[u] == 8) {
                    g[u].u = *reinterpret_cast<const uint4*>(dY + e);
                    if (act != ACT_LINEAR) y[u].u = *reinterpret_cast<const uint4*>(Yv + e);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        if (j < nv[u]) {
                            g[u].h[j] = dY[e + j];
                            if (act != ACT_LINEAR) y[u].h[j] = Yv[e + j];
                        }
                }
                const int ra = min(R - 1, min(sr, sr1 - 1) * 8 + ro[0]), rb = min(R - 1, ra + 1);
#pragma unroll
                for (int k = 0; k < K; ++k) {
                    xa[u][k] = bf2f(X[(int64_t)ra * ldx + k]);
                    xb[u][k] = bf2f(X[(int64_t)rb * ldx + k]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float gz = bf2f(g[u].h[j]);          // 0 past the end
                    if (act != ACT_LINEAR) gz = bf2f(f2bf(gz * act_grad_from_y(bf2f(y[u].h[j]), act)));
                    const bool hi = ro[j] != ro[0];
#pragma unroll
                    for (int k = 0; k < K; ++k) acc[j * K + k] += gz * (hi ? xb[u][k] : xa[u][k]);
                    acc[8 * K + j] += gz;
                }
            }
        }
        // quantity p (k < K: weight column k, K: bias) of slot q * 8F + 8i + j
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
            for (int k = 0; k < K; ++k) red[k * 2048 + q * 8 * F + 8 * i + j] = acc[j * K + k];
            red[K * 2048 + q * 8 * F + 8 * i + j] = acc[8 * K + j];
        }
    }
    __syncthreads();
    for (int o = t; o < F * (K + 1); o += 256) {
        const int c = o / (K + 1), p = o - c * (K + 1);
        float v = 0.f;
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int m = 0; m < 8; ++m) v += red[p * 2048 + g * 8 * F + c + m * F];
        if (p < K) fx_add(reinterpret_cast<long long*>(d.out) + (int64_t)c * K + p, v);
        else if (dbias) fx_add(dbias + c, v);
    }
}

// ==================================================================================================
// LDS-tiled GEMM for 1x1 / Dense problems (row-major A[M][K] with row stride C, B[N][K]):
//   FWD   : Y = act(A . B^T + bias)          A = layer input,  B = Wm
//   DGRAD : dX (+)= (dY * act'(Y)) . B^T     A = dY (+ Y),     B = Wt
// Block tile 128 x BN (BN = 64, 128, 160 or 192: one n tile covers a merged Dense of up to 192 units, so
// its input panel is read once and no half-empty second tile is computed) x 32, 4 waves in a 2 x 2
// layout (64 x BN/2 each).  Both
// operand tiles go through LDS, so the weight tile is fetched once per block instead of once per
// wave (the direct-fragment kernel re-reads B in every wave), and the next k-step's global loads are in
// flight while the current step multiplies (register-staged double buffer, one barrier per step).
// LDS rows are 32 elements (64 B) with the four 16-B k chunks of a row XOR-swizzled by its row quad
// (row >> 2) & 3 -> {0, 2, 3, 1}: every 16-lane group of a ds_read_b128 fragment read ({0-3, 12-15,
// 20-27}, ...: rows 0-3 and 12-15 at one k chunk, rows 4-11 at the next) then hits 16 distinct 16-B slots of
// the 256-B bank row, and the 8-lane groups of the ds_write_b128 staging stores stay inside one 128-B
// window.  (The former 80-B padded rows put rows 1 and 4 + chunk 1 on one slot: 5.3 conflict cycles per LDS
// instruction measured, profiles/r4/pmc_heavy_launches.txt.)  The epilogue stages the block's tile in LDS and streams it out with 16-B stores
// when the block spans all N columns (the usual case: N <= 128).
// BT (DGRAD only): B is the layer's weight matrix in its natural [K = F][N = C] layout (row stride ldb,
// default N) instead of the transposed copy Wt[C][F]: a k-step's B tile is loaded as 32 k rows x BN
// columns (16-B chunks along n), staged k-major in LDS ([32][BN + 8]) and its MFMA fragments are read
// with ds_read_b64_tr_b16 (lane i of a 16-lane group receives column i of 4 consecutive k rows, k row q
// in element q -- the k order of the ds_read_b128 A fragments).  No per-step weight transpose launch.
// (Occupancy: requesting 3 waves per SIMD for BN <= 160 -- accumulators in VGPRs, no spills -- measured 2-3 %
// slower on the ancestor population and neutral on the generation-3 mix: profiles/r4/ab_tiled_occupancy.txt)
template <int MODE, int BN, bool BT = false, bool NS = false>
__global__ __launch_bounds__(256) void g3_tiled_kernel(const GemmDesc* __restrict__ descs,
                                                       const int4* __restrict__ tiles) {
    constexpr int BM = 128, BK = 32, LDS_ROW = BK;
    constexpr int NTW = BN / 32;                     // 16-col tiles per wave (2 waves along n)
    constexpr int LDBT = BN + 8;                     // BT: k-major B row (multiple of 8 elements)
    constexpr int ABYTES = 2 * BM * LDS_ROW, BBYTES = BT ? 2 * BK * LDBT : 2 * BN * LDS_ROW;
    constexpr int STAGE = BM * (BN + 8);             // epilogue staging (bf16 elements, padded rows)
    constexpr int LDSN0 = (ABYTES + BBYTES) > STAGE ? (ABYTES + BBYTES) : STAGE;
    // NS epilogue staging (floats): x tile [BN / 8 + 2][BM + 4], dY slice [32][BM + 4], sums [2][8][32][8]
    constexpr int NSLDS = NS ? 2 * ((BN / 8 + 2) * (BM + 4) + 32 * (BM + 4) + 2 * 8 * 32 * 8) : 0;
    constexpr int LDSN = LDSN0 > NSLDS ? LDSN0 : NSLDS;
    __shared__ __attribute__((aligned(16))) bf16_t lds[LDSN];
    bf16_t* As = lds;                                // [2][BM][LDS_ROW]
    bf16_t* Bs = lds + ABYTES;                       // [2][BN][LDS_ROW]
    const int4 td = tiles[blockIdx.x];
    const GemmDesc& d = descs[td.x];
    const int M = (int)d.M, N = (int)d.N, K = (int)d.K, act = (int)d.act, flags = (int)d.flags;
    // A row stride: FWD reads the layer input [M][C] (C == K, or K8 for the shared raw im2col);
    // DGRAD reads dY [M][F] with F == K for a 1x1 layer
    const int lda = (MODE == MODE_FWD) ? (int)d.C : K;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int r16 = lane & 15;
    // swizzled k-chunk offsets (elements) of this lane's fragment reads and of its staging stores
    auto kswz = [](int row, int chunk) { return (chunk ^ ((0x1320 >> (((row >> 2) & 3) * 4)) & 3)) << 3; };
    const int kfa = kswz(r16, lane >> 4);
    // td.z: first n tile | (n tiles of this block << 16): a block walks ntc consecutive column tiles of its row tile
    // (the tiles are independent -- each output tile is one block's -- so the grouping is a schedule choice only)
    const int m0 = td.y * BM;
    int n0 = (td.z & 0xffff) * BN;
    const int ntc = max(1, td.z >> 16);
    const int kt0 = td.w & 0xffff, kt1 = (td.w >> 16) & 0xffff;
    const int64_t a_elems = (int64_t)M * lda;
    const rsrc_t rA = mkrsrc(d.a, a_elems * 2);
    const rsrc_t rY = mkrsrc(d.aux, d.aux ? a_elems * 2 : 0);
    // B row stride: a K slice of a wider weight matrix (FWD), or the natural [K][N] weights (BT)
    const int ldb = d.ldb ? (int)d.ldb : (BT ? N : K);
    const rsrc_t rB = mkrsrc(d.b, (int64_t)(BT ? K : N) * ldb * 2);
    const uint4 zero = make_uint4(0, 0, 0, 0);
    const int gact = (MODE == MODE_DGRAD) ? act : ACT_LINEAR;

    // loaders: thread t -> (row t/4 + 64 i, k chunk (t % 4) * 8)
    const int lr = t >> 2, lk = (t & 3) * 8;
    const int lks = kswz(lr, t & 3);                 // (rows lr + 64 i share lr's row quad)
    constexpr int BPT = (BN + 63) / 64;              // B chunks per thread (BN = 160 / 192: the last partial)
    // BT loader: thread t -> (k row t / NCH + BKP i, n chunk (t % NCH) * 8)
    constexpr int NCH = BN / 8, BKP = 256 / NCH, BTP = (BK + BKP - 1) / BKP;
    const int bkr = t / NCH, bnc = (t % NCH) * 8;
    const bool bt_act = t < NCH * BKP;
    // DGRAD: dY and Y load raw and dZ = dY * act'(Y) is formed in sstore(), after the MFMAs of the
    // current step (forming it here made the step wait for the loads of the next one).  Measured
    // slower in g3_direct_kernel, whose fragments stay in registers: there the extra Y registers of
    // both pipeline sets cost a wave per SIMD (profiles/r2e/kb_dgrad_compare.txt)
    uint4 ra[2], ry[2], rb[BT ? BTP : BPT];
    int arun = 8;
    auto gload = [&](int kt) {
        const int k = kt * BK + lk;
        const int run = min(8, K - k);
        arun = run;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int m = m0 + lr + 64 * i;
            const int off = (m < M && run > 0) ? m * lda + k : -1;
            ra[i] = bl16(rA, off);
            if (gact != ACT_LINEAR) ry[i] = bl16(rY, off);
        }
        if (BT) {
#pragma unroll
            for (int i = 0; i < BTP; ++i) {
                const int kk = kt * BK + bkr + BKP * i;
                const int n = n0 + bnc;
                const int off = (bt_act && bkr + BKP * i < BK && kk < K && n < N) ? kk * ldb + n : -1;
                uint4 v = bl16(rB, off);
                if (N - n < 8) v = splice(v, zero, N - n);
                rb[i] = v;
            }
        } else {
#pragma unroll
            for (int i = 0; i < BPT; ++i) {
                const int n = n0 + lr + 64 * i;
                const int off = (lr + 64 * i < BN && n < N && run > 0) ? n * ldb + k : -1;
                uint4 v = bl16(rB, off);
                if (run < 8) v = splice(v, zero, run);
                rb[i] = v;
            }
        }
    };
    auto sstore = [&](int buf) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            uint4 v = ra[i];
            if (gact != ACT_LINEAR) v = mul_act_grad(v, ry[i], gact);
            if (arun < 8) v = splice(v, zero, arun);
            *reinterpret_cast<uint4*>(&As[(buf * BM + lr + 64 * i) * LDS_ROW + lks]) = v;
        }
        if (BT) {
#pragma unroll
            for (int i = 0; i < BTP; ++i)
                if (bt_act && bkr + BKP * i < BK)
                    *reinterpret_cast<uint4*>(&Bs[(buf * BK + bkr + BKP * i) * LDBT + bnc]) = rb[i];
        } else {
#pragma unroll
            for (int i = 0; i < BPT; ++i)
                if (lr + 64 * i < BN) *reinterpret_cast<uint4*>(&Bs[(buf * BN + lr + 64 * i) * LDS_ROW + lks]) = rb[i];
        }
    };

    bool pre = false;
    for (int nti = 0; nti < ntc; ++nti, n0 += BN) {
    if (nti > 0) __syncthreads();                    // the previous tile's epilogue is done with the LDS
    f32x4_t acc[4][NTW];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NTW; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    if (kt0 < kt1) {
        if (!pre) gload(kt0);                        // (pre: this tile's first k step was loaded during the
        sstore(0);                                   //  previous tile's epilogue)
    }
    pre = false;
    __syncthreads();
    for (int kt = kt0; kt < kt1; ++kt) {
        const int buf = (kt - kt0) & 1;
        if (kt + 1 < kt1) {
            gload(kt + 1);
        } else if (nti + 1 < ntc) {
            // last k step: the next n tile's first k step goes in flight now, across this tile's epilogue
            n0 += BN;
            gload(kt0);
            n0 -= BN;
            pre = true;
        }
        Frag fa[4], fb[NTW];
#pragma unroll
        for (int i = 0; i < 4; ++i)
            fa[i].u = *reinterpret_cast<const uint4*>(&As[(buf * BM + wr * 64 + i * 16 + r16) * LDS_ROW + kfa]);
        if (BT) {
            const int grp = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
#pragma unroll
            for (int j = 0; j < NTW; ++j) {
                const int colb = wc * (BN / 2) + j * 16 + 4 * pp;
                fb[j].v = tr_frag(&Bs[(buf * BK + grp * 8 + q) * LDBT + colb], &Bs[(buf * BK + grp * 8 + 4 + q) * LDBT + colb]);
            }
        } else {
#pragma unroll
            for (int j = 0; j < NTW; ++j)
                fb[j].u = *reinterpret_cast<const uint4*>(&Bs[(buf * BN + wc * (BN / 2) + j * 16 + r16) * LDS_ROW + kfa]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < NTW; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i].v, fb[j].v, acc[i][j], 0, 0, 0);
        if (kt + 1 < kt1) sstore(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue ---------------------------------------------------------------------------------
    const float* bias = (MODE == MODE_FWD) ? reinterpret_cast<const float*>(d.bias) : nullptr;
    const int oact = (MODE == MODE_FWD) ? act : ACT_LINEAR;
    const int rq = (lane >> 4) * 4;
    if constexpr (MODE == MODE_FWD) {
        if (flags & GF_BNUSTAT) {                    // (never with GF_SPLITWS: the planner's condition)
            float* bnred = reinterpret_cast<float*>(lds);        // the k loop ended on a barrier
            bn_ustat_flush<4, NTW, 2>(d, acc, [&](int i, int rr) { return m0 + wr * 64 + i * 16 + rr < M; }, n0, N,
                                      bias, act, bnred, wave, lane, N);
            __syncthreads();                         // (the staging epilogue below reuses the LDS)
        }
    }
    if constexpr (MODE == MODE_DGRAD && NS) {
        // NS (GF_NBNSUM; its own instantiation, so the other DGRADs keep their registers / occupancy).
        // This DGRAD produces dY of a fused raw-input Dense -> BatchNormalization pair with ONE input channel
        // (nbn.hip; the planner's condition) and is its only producer: dY is never stored.  Per column n
        // (BN row r = m * np + n / F, channel f = n % F) the block reduces, over its rows and from the fp32
        // accumulators, what the BN backward and the Dense WGRAD need (y recomputed from the raw input x
        // exactly as nbn.hip does, xhat = (y - mean) invstd, a = act'(y)):
        //   [0] dy  [1] dy xhat  [2] a dy  [3] a xhat  [4] a  [5] a x dy  [6] a x xhat  [7] a x
        // and stores them to NbnDesc::part, slot m tile -- plain stores, one writer per (slot, column).  nbn
        // phase 6 adds the slots in a fixed order and forms dgamma, dbeta, dW, db.
        constexpr int NSUM = 8;
        const NbnDesc& nd = *reinterpret_cast<const NbnDesc*>(d.ext);
        const int Fb = (int)nd.F, ldxr = (int)nd.ldx, NPc = (int)nd.np, nact = (int)nd.act;
        const bf16_t* __restrict__ Xr = reinterpret_cast<const bf16_t*>(nd.x);
        const bf16_t* __restrict__ Wn = reinterpret_cast<const bf16_t*>(nd.w);
        const float* __restrict__ nb = reinterpret_cast<const float*>(nd.bias);
        const float* __restrict__ nmean = reinterpret_cast<const float*>(nd.mean);
        const float* __restrict__ nis = reinterpret_cast<const float*>(nd.invstd);
        // the block's raw inputs x[m][p] (rows m0.., positions p0..p1 of its columns) staged once in LDS, and
        // per column tile j the fp32 dY slice [BM][32] (both waves along n): the sums are then formed from LDS
        // by (column, 16-row group) threads -- reading the accumulators in place would keep the whole tile
        // in VGPRs through the epilogue, and that peak (not the k loop) would set the occupancy
        // Layouts are column-major so that every LDS access is a 16-B vector: the accumulators' 4 consecutive
        // rows go out as one ds_write_b128 and a (column, 16-row group) thread reads its rows as 4 of them;
        // strides of BM + 4 floats put the 16 lanes of a b128 group on distinct banks
        constexpr int SLT = BM + 4;
        const int p0 = n0 / Fb, npos = min(N - 1, n0 + BN - 1) / Fb - p0 + 1;
        float* xs = reinterpret_cast<float*>(lds);       // [npos][SLT]; the k loop ended on a barrier
        float* sl = xs + (BN / 8 + 2) * SLT;             // [32 columns][SLT]
        float* red = sl + 32 * SLT;                      // [2 buffers][8 row groups][32 columns][NSUM]
        static_assert(((BN / 8 + 2) * SLT + 32 * SLT + 2 * 8 * 32 * NSUM) * 4 <= LDSN * 2,
                      "NBNSUM staging must fit in the LDS tiles");
        for (int u = t; u < BM * npos; u += 256) {
            const int pp = u / BM, rl = u - pp * BM;
            const int row = min(m0 + rl, M - 1);
            xs[pp * SLT + rl] = bf2f(Xr[((int64_t)row * NPc + p0 + pp) * ldxr]);
        }
        float* __restrict__ part = reinterpret_cast<float*>(nd.part) + (int64_t)td.y * N * NSUM;
        const int sc = t & 31, sg = t >> 5;              // column of the slice, 16-row group
        // rows past M: their dY is 0 (the A loads returned zeros) and their act' is masked below, so every
        // sum gets exact zeros from them.  Activation and the full-rows case are compile-time in the row
        // loop; the rows are taken in pairs so the sums issue as packed fp32 (v_pk_fma_f32)
        const int nrow = M - m0 - sg * 16;
        auto col_sums = [&](auto act_tag, auto full_tag, const float* xc, const float* gc, float w, float bv,
                            float mu, float is, float* sm) {
            constexpr int A = decltype(act_tag)::value;
            constexpr bool FULL = decltype(full_tag)::value;
            f32x2_t s[NSUM];
#pragma unroll
            for (int q = 0; q < NSUM; ++q) s[q] = f32x2_t{0.f, 0.f};
            const float nmis = -mu * is;
            // the 4 row quads stay a loop: unrolled, the hoisted LDS reads cost a wave per SIMD (112 VGPRs)
#pragma unroll 1
            for (int r4 = 0; r4 < 4; ++r4) {
                const float4 x4 = *reinterpret_cast<const float4*>(xc + 4 * r4);
                const float4 g4 = *reinterpret_cast<const float4*>(gc + 4 * r4);
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const f32x2_t xv = h ? f32x2_t{x4.z, x4.w} : f32x2_t{x4.x, x4.y};
                    const f32x2_t gy = h ? f32x2_t{g4.z, g4.w} : f32x2_t{g4.x, g4.y};
                    const f32x2_t v = xv * w + bv;       // nbn.hip nbn_y: bias, then the product (one fma)
                    f32x2_t y, a;
                    if constexpr (A == ACT_RELU) {
                        y = f32x2_t{v.x > 0.f ? v.x : 0.f, v.y > 0.f ? v.y : 0.f};
                        a = f32x2_t{y.x > 0.f ? 1.f : 0.f, y.y > 0.f ? 1.f : 0.f};
                    } else if constexpr (A == ACT_SIGMOID) {
                        y = f32x2_t{apply_act(v.x, ACT_SIGMOID), apply_act(v.y, ACT_SIGMOID)};
                        a = y * (1.f - y);
                    } else {
                        y = v;
                        a = f32x2_t{1.f, 1.f};
                    }
                    if constexpr (!FULL) {
                        const int r = 4 * r4 + 2 * h;
                        a = f32x2_t{r < nrow ? a.x : 0.f, r + 1 < nrow ? a.y : 0.f};
                    }
                    const f32x2_t xh = y * is + nmis;
                    const f32x2_t ax = a * xv;
                    s[0] += gy;
                    s[1] += gy * xh;
                    s[2] += a * gy;
                    s[3] += a * xh;
                    s[4] += a;
                    s[5] += ax * gy;
                    s[6] += ax * xh;
                    s[7] += ax;
                }
            }
#pragma unroll
            for (int q = 0; q < NSUM; ++q) sm[q] = s[q].x + s[q].y;
        };
        const bool fullrows = m0 + BM <= M;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                *reinterpret_cast<float4*>(&sl[(wc * 16 + r16) * SLT + wr * 64 + i * 16 + rq]) =
                    make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
            __syncthreads();
            const int cl = (sc >> 4) * (BN / 2) + j * 16 + (sc & 15);   // block column of slice column sc
            const int n = n0 + cl;
            float sm[NSUM];
#pragma unroll
            for (int q = 0; q < NSUM; ++q) sm[q] = 0.f;
            if (n < N) {
                const int p = n / Fb, f = n - p * Fb;
                const float w = bf2f(Wn[f]), bv = nb ? nb[f] : 0.f, mu = nmean[f], is = nis[f];
                const float* xc = xs + (p - p0) * SLT + sg * 16;
                const float* gc = sl + sc * SLT + sg * 16;
                using TT = std::true_type;
                using FT = std::false_type;
                using RL = std::integral_constant<int, ACT_RELU>;
                using SG = std::integral_constant<int, ACT_SIGMOID>;
                using LN = std::integral_constant<int, ACT_LINEAR>;
                if (fullrows) {
                    if (nact == ACT_RELU) col_sums(RL{}, TT{}, xc, gc, w, bv, mu, is, sm);
                    else if (nact == ACT_SIGMOID) col_sums(SG{}, TT{}, xc, gc, w, bv, mu, is, sm);
                    else col_sums(LN{}, TT{}, xc, gc, w, bv, mu, is, sm);
                } else {
                    if (nact == ACT_RELU) col_sums(RL{}, FT{}, xc, gc, w, bv, mu, is, sm);
                    else if (nact == ACT_SIGMOID) col_sums(SG{}, FT{}, xc, gc, w, bv, mu, is, sm);
                    else col_sums(LN{}, FT{}, xc, gc, w, bv, mu, is, sm);
                }
            }
            // red is double-buffered: the next tile's writes cannot race this tile's reads (a barrier
            // lies between), so one barrier per tile is saved
            float* rb = red + (j & 1) * (8 * 32 * NSUM);
            *reinterpret_cast<float4*>(&rb[(sg * 32 + sc) * NSUM]) = make_float4(sm[0], sm[1], sm[2], sm[3]);
            *reinterpret_cast<float4*>(&rb[(sg * 32 + sc) * NSUM + 4]) = make_float4(sm[4], sm[5], sm[6], sm[7]);
            __syncthreads();
            {
                const int c2 = t / NSUM, q = t - c2 * NSUM;          // 32 columns x 8 sums = 256 threads
                const int n2 = n0 + (c2 >> 4) * (BN / 2) + j * 16 + (c2 & 15);
                float v = 0.f;
#pragma unroll
                for (int g = 0; g < 8; ++g) v += rb[(g * 32 + c2) * NSUM + q];
                if (n2 < N) part[(int64_t)n2 * NSUM + q] = v;
            }
        }
        continue;
    }
    if (MODE == MODE_FWD && (flags & GF_SPLITWS)) {
        // raw fp32 partial of this k split; splitk_finalize adds the splits, bias and activation
        float* w = reinterpret_cast<float*>(d.aux) + ((int64_t)d.sbase + kt0 / (int)d.kper) * M * N;
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int col = n0 + wc * (BN / 2) + j * 16 + r16;
            if (col >= N) continue;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wr * 64 + i * 16 + rq + r;
                    if (row < M) w[(int64_t)row * N + col] = acc[i][j][r];
                }
        }
        continue;
    }
    if (flags & GF_OUT_F32) {
        float* o = reinterpret_cast<float*>(d.out);
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int col = n0 + wc * (BN / 2) + j * 16 + r16;
            if (col >= N) continue;
            const float bv = bias ? bias[col] : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = m0 + wr * 64 + i * 16 + rq + r;
                    if (row >= M) continue;
                    o[(int64_t)row * N + col] = apply_act(acc[i][j][r] + bv, oact);
                }
        }
        continue;
    }
    bf16_t* o = reinterpret_cast<bf16_t*>(d.out);
    const bool accum = (flags & GF_ACCUM) != 0;
    if (n0 == 0 && N <= BN) {
        // the block's rows [m0, m0 + nrows) x all N columns are one contiguous range of the output
        bf16_t* st = lds;                            // k loop done (last barrier above)
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int col = wc * (BN / 2) + j * 16 + r16;
            if (col >= N) continue;
            const float bv = bias ? bias[col] : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st[(wr * 64 + i * 16 + rq + r) * N + col] = f2bf(apply_act(acc[i][j][r] + bv, oact));
        }
        __syncthreads();
        const int nrows = min(BM, M - m0);
        const int total = nrows * N, nvec = total >> 3;
        bf16_t* dst = o + (int64_t)m0 * N;           // m0 * N * 2 B is a multiple of 256 B
        for (int v = t; v < nvec; v += 256) {
            Frag f;
            f.u = *reinterpret_cast<const uint4*>(&st[v * 8]);
            if (accum) {
                Frag p;
                p.u = *reinterpret_cast<const uint4*>(&dst[v * 8]);
#pragma unroll
                for (int e = 0; e < 8; ++e) f.h[e] = f2bf(bf2f(f.h[e]) + bf2f(p.h[e]));
            }
            *reinterpret_cast<uint4*>(&dst[v * 8]) = f.u;
        }
        for (int e = nvec * 8 + t; e < total; e += 256) {
            float v = bf2f(st[e]);
            if (accum) v += bf2f(dst[e]);
            dst[e] = f2bf(v);
        }
        continue;
    }
    {
        // general tile (wide outputs: DGRAD of a merged Dense, FWD with N > BN): the tile is staged in LDS
        // and leaves as row segments of 8 columns -- 16-, 8- or 4-byte stores by the segment's alignment
        // (row stride N need not be a multiple of 8) -- instead of the MFMA layout's 2-byte column stores
        constexpr int SROW = BN + 8;
        bf16_t* st = lds;                            // k loop done (last barrier above)
#pragma unroll
        for (int j = 0; j < NTW; ++j) {
            const int cl = wc * (BN / 2) + j * 16 + r16;
            const float bv = (bias && n0 + cl < N) ? bias[n0 + cl] : 0.f;
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    st[(wr * 64 + i * 16 + rq + r) * SROW + cl] = f2bf(apply_act(acc[i][j][r] + bv, oact));
        }
        __syncthreads();
        const int nrows = min(BM, M - m0), ncols = min(BN, N - n0);
        constexpr int CH = BN / 8;
        for (int u = t; u < BM * CH; u += 256) {
            const int r = u / CH, c8 = (u % CH) * 8;
            if (r >= nrows || c8 >= ncols) continue;
            const int64_t g = (int64_t)(m0 + r) * N + n0 + c8;
            Frag f;
            f.u = *reinterpret_cast<const uint4*>(&st[r * SROW + c8]);
            const int nv = min(8, ncols - c8);
            if (accum) {
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (e < nv) f.h[e] = f2bf(bf2f(f.h[e]) + bf2f(o[g + e]));
            }
            if (nv == 8 && (g & 7) == 0) {
                *reinterpret_cast<uint4*>(o + g) = f.u;
            } else if (nv == 8 && (g & 3) == 0) {
                *reinterpret_cast<uint2*>(o + g) = make_uint2(f.w[0], f.w[1]);
                *reinterpret_cast<uint2*>(o + g + 4) = make_uint2(f.w[2], f.w[3]);
            } else if (nv == 8 && (g & 1) == 0) {
#pragma unroll
                for (int w = 0; w < 4; ++w) *reinterpret_cast<uint32_t*>(o + g + 2 * w) = f.w[w];
            } else {
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (e < nv) o[g + e] = f.h[e];
            }
        }
    }
    }   // n tiles
}

// variant encoding (FWD / DGRAD): NT (BN/16: 1, 2, 4, 8) + 10 * RT (2 or 4) + 100 * KW + 1000 * GEN,
//                 or 5000 + NT + 10 * RT for the single-k-step (K <= 32) form, 6000 + K for narrow (K <= 4; + 100 staged, + 200 super-row),
//                 7000 + BN for the LDS-tiled 1x1 kernel (BN = 64 / 128 / 160 / 192; tiles (prob, m tile, n tile,
//                 k range)), 8000 + BN the same for DGRAD with B = natural-layout weights [F][C] (BT)
//                 FWD LDS-halo convolution: 2000 + NT (1, 2, 4) + 10 * RT (1, 2, 4) + 100 * patch tier
//                 (0: 16 KB, 1: 32 KB, 2: 64 KB);
//                 tiles (prob, b, m0, ntile)
// variant encoding (WGRAD): BMF * 1000 + BNK (+ 1000000 * GEN); BMF in {16, 32, 64}, BNK in {16, 64, 128, 256}
//                 narrow (K <= 4): 4000000 + K (+ 100: LDS-staged rows, + 200: super-row form; F % 8 != 0);
//                 tiles (prob, row block, 0, 0)
//                 LDS-halo conv WGRAD: 3000000 + 100000 * patch tier + BMF * 1000 + BNK / 64 (column tiles per wave:
//                 2 .. 32);
//                 tiles (prob, ftile << 16 | ktile, chunk0, chunk1)
// The launcher is compiled in four parts (GEMM3_PART = 0..3, one object each, built in parallel: serann/build.py
// MULTI_PART); every part instantiates only the kernels its variants launch.  GEMM3_PART undefined: all parts here.
#ifndef GEMM3_PART
#define GEMM3_PART -1
#endif
#define G3_PART(k) (GEMM3_PART < 0 || GEMM3_PART == (k))
bool gemm3_launch_part0(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp, const int4* tp);
bool gemm3_launch_part1(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp, const int4* tp);
bool gemm3_launch_part2(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp, const int4* tp);
bool gemm3_launch_part3(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp, const int4* tp);

#if G3_PART(0)
// part 0: Dense / 1x1 and narrow WGRAD
bool gemm3_launch_part0(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp,
                          const int4* tp) {
    if (mode == MODE_WGRAD && variant > 8000000 && variant < 8000010) {
        // small-bank WGRAD (F <= 16, N <= 16 NK): 8000000 + NK
        switch (variant - 8000000) {
            case 1: hipLaunchKernelGGL((g3_wgrad_tiny_kernel<1>), grid, block, 0, s, dp, tp); break;
            case 2: hipLaunchKernelGGL((g3_wgrad_tiny_kernel<2>), grid, block, 0, s, dp, tp); break;
            case 4: hipLaunchKernelGGL((g3_wgrad_tiny_kernel<4>), grid, block, 0, s, dp, tp); break;
            default: throw std::runtime_error("gemm3: unknown small-bank WGRAD variant " + std::to_string(variant));
        }
        SERANN_CHECK(hipGetLastError());
        return true;
    }
    if (mode == MODE_WGRAD && variant >= 5000000) {
        // LDS-DMA Dense / 1x1 WGRAD: 5000000 + BMF * 1000 + BNK (+ 500: act' from a staged Y tile)
        const int v = variant - 5000000;
#define DW3(BMF_, BNK_)                                                                                  \
    if (v == BMF_ * 1000 + BNK_) { hipLaunchKernelGGL((g3_dwgrad_kernel<BMF_, BNK_, false>), grid, block, 0, s, dp, tp); \
                                   SERANN_CHECK(hipGetLastError()); return true; }                            \
    if (v == BMF_ * 1000 + BNK_ + 500) { hipLaunchKernelGGL((g3_dwgrad_kernel<BMF_, BNK_, true>), grid, block, 0, s, dp, tp); \
                                         SERANN_CHECK(hipGetLastError()); return true; }
        DW3(64, 128) DW3(64, 64) DW3(32, 128) DW3(32, 64) DW3(16, 256) DW3(16, 128) DW3(16, 64)
#undef DW3
        throw std::runtime_error("gemm3: unknown dense WGRAD variant " + std::to_string(variant));
    }
    if (mode == MODE_WGRAD && variant >= 4000000) {
        const int k = (variant - 4000000) % 100;
        const bool st = (variant - 4000000) >= 100, sr = (variant - 4000000) >= 200;
#define NW(K_) if (k == K_) { if (sr) hipLaunchKernelGGL((g3_narrow_wgrad_sr_kernel<K_>), grid, block, 0, s, dp, tp); \
                              else if (st) hipLaunchKernelGGL((g3_narrow_wgrad_kernel<K_, true>), grid, block, 0, s, dp, tp); \
                              else hipLaunchKernelGGL((g3_narrow_wgrad_kernel<K_, false>), grid, block, 0, s, dp, tp); }
        NW(1) else NW(2) else NW(3) else NW(4)
#undef NW
        else throw std::runtime_error("gemm3: unknown narrow WGRAD variant " + std::to_string(variant));
        SERANN_CHECK(hipGetLastError());
        return true;
    }
    if (mode == MODE_WGRAD && variant < 3000000) {     // (3000000 .. 3999999: conv WGRAD, part 1)
        const bool gen = variant >= 1000000;
        const int v = variant % 1000000;
        // v = BMF * 1000 + BNK (+ 500: two row groups per block, 512 threads)
#define W3(BMF_, BNK_) \
    if (v == BMF_ * 1000 + BNK_) { \
        if (gen) hipLaunchKernelGGL((g3_wgrad_kernel<BMF_, BNK_, true>), grid, block, 0, s, dp, tp); \
        else hipLaunchKernelGGL((g3_wgrad_kernel<BMF_, BNK_, false>), grid, block, 0, s, dp, tp); \
        SERANN_CHECK(hipGetLastError()); return true; } \
    if (v == BMF_ * 1000 + BNK_ + 500) { \
        const dim3 b2(512); \
        if (gen) hipLaunchKernelGGL((g3_wgrad_kernel<BMF_, BNK_, true, 4, 2>), grid, b2, 0, s, dp, tp); \
        else hipLaunchKernelGGL((g3_wgrad_kernel<BMF_, BNK_, false, 4, 2>), grid, b2, 0, s, dp, tp); \
        SERANN_CHECK(hipGetLastError()); return true; }
        W3(64, 128) W3(64, 64) W3(32, 128) W3(32, 64) W3(16, 256) W3(16, 128) W3(16, 64) W3(64, 16)
        // whole-F tiles of single-split Dense WGRADs (hip_ops.WGRAD_WIDE): X read once per column tile
        W3(96, 64) W3(128, 64) W3(160, 64) W3(192, 64)
#undef W3
        throw std::runtime_error("gemm3: unknown WGRAD variant " + std::to_string(variant));
    }
    return false;
}
#endif

#if G3_PART(1)
// part 1: LDS-halo conv WGRAD
bool gemm3_launch_part1(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp,
                          const int4* tp) {
    if (mode == MODE_WGRAD && variant >= 3000000) {
        const int tier = (variant / 100000) % 10;
        const int v = variant % 100000;
#define CW3T(BMF_, BNK_, TIER_, PATCH_)                                                               \
    if (v == BMF_ * 1000 + BNK_ / 64 && tier == TIER_) {                                                   \
        hipLaunchKernelGGL((g3_conv_wgrad_kernel<BMF_, BNK_, PATCH_>), grid, block, 0, s, dp, tp);     \
        SERANN_CHECK(hipGetLastError());                                                              \
        return true;                                                                                       \
    }
#define CW3(BMF_, BNK_) CW3T(BMF_, BNK_, 0, 8192) CW3T(BMF_, BNK_, 1, 16384) CW3T(BMF_, BNK_, 2, 32768)
        // (the 64 KB patch tier is instantiated for 16-filter blocks only: two stages of it fill the LDS)
#define CW3S(BMF_, BNK_) CW3T(BMF_, BNK_, 0, 8192) CW3T(BMF_, BNK_, 1, 16384)
        CW3(16, 2048) CW3(16, 1024) CW3(16, 512) CW3(16, 256) CW3(16, 128)
        CW3S(32, 1024) CW3S(32, 512) CW3S(32, 256) CW3S(32, 128) CW3S(64, 512) CW3S(64, 256) CW3S(64, 128)
#undef CW3S
#undef CW3T
#undef CW3
        throw std::runtime_error("gemm3: unknown conv WGRAD variant " + std::to_string(variant));
    }
    return false;
}
#endif

#if G3_PART(2)
// part 2: conv FWD and LDS-tiled FWD / DGRAD
bool gemm3_launch_part2(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp,
                          const int4* tp) {
    if (mode == MODE_FWD && variant >= 2000 && variant < 3000) {
        const int v = variant - 2000;
#define C3T(NT_, RT_, TIER_, PATCH_)                                                                  \
    if (v == 100 * TIER_ + NT_ + 10 * RT_) {                                                          \
        hipLaunchKernelGGL((g3_conv_fwd_kernel<NT_, RT_, PATCH_>), grid, block, 0, s, dp, tp);         \
        SERANN_CHECK(hipGetLastError());                                                              \
        return true;                                                                                       \
    }
#define C3(NT_, RT_) C3T(NT_, RT_, 0, 8192) C3T(NT_, RT_, 1, 16384) C3T(NT_, RT_, 2, 32768)
        C3(1, 1) C3(2, 1) C3(4, 1) C3(1, 2) C3(2, 2) C3(4, 2) C3(1, 4) C3(2, 4) C3(4, 4)
#undef C3T
#undef C3
        throw std::runtime_error("gemm3: unknown conv variant " + std::to_string(variant));
    }
    if (variant == 7064 || variant == 7128 || variant == 7160 || variant == 7192) {
#define TL(BN_)                                                                                     \
    if (variant == 7000 + BN_) {                                                                    \
        if (mode == MODE_FWD) hipLaunchKernelGGL((g3_tiled_kernel<MODE_FWD, BN_>), grid, block, 0, s, dp, tp); \
        else hipLaunchKernelGGL((g3_tiled_kernel<MODE_DGRAD, BN_>), grid, block, 0, s, dp, tp);      \
    }
        TL(64) TL(128) TL(160) TL(192)
#undef TL
        SERANN_CHECK(hipGetLastError());
        return true;
    }
    if (mode == MODE_DGRAD && variant > 17000 && variant < 19000) {
        // GF_NBNSUM: the BN-backward-sums epilogue (17000 + BN: transposed weights, 18000 + BN: natural)
#define TLS(BN_)                                                                                                \
    if (variant == 17000 + BN_) hipLaunchKernelGGL((g3_tiled_kernel<MODE_DGRAD, BN_, false, true>), grid, block, 0, s, dp, tp); \
    else if (variant == 18000 + BN_) hipLaunchKernelGGL((g3_tiled_kernel<MODE_DGRAD, BN_, true, true>), grid, block, 0, s, dp, tp); else
        TLS(64) TLS(128) TLS(160) TLS(192)
#undef TLS
        throw std::runtime_error("gemm3: unknown NBNSUM DGRAD variant " + std::to_string(variant));
        SERANN_CHECK(hipGetLastError());
        return true;
    }
    if (mode == MODE_DGRAD && (variant == 8064 || variant == 8128 || variant == 8160 || variant == 8192)) {
        // BT: natural-layout weights
        if (variant == 8064) hipLaunchKernelGGL((g3_tiled_kernel<MODE_DGRAD, 64, true>), grid, block, 0, s, dp, tp);
        else if (variant == 8128) hipLaunchKernelGGL((g3_tiled_kernel<MODE_DGRAD, 128, true>), grid, block, 0, s, dp, tp);
        else if (variant == 8160) hipLaunchKernelGGL((g3_tiled_kernel<MODE_DGRAD, 160, true>), grid, block, 0, s, dp, tp);
        else hipLaunchKernelGGL((g3_tiled_kernel<MODE_DGRAD, 192, true>), grid, block, 0, s, dp, tp);
        SERANN_CHECK(hipGetLastError());
        return true;
    }
    return false;
}
#endif

#if G3_PART(3)
// ==================================================================================================
// Shared-input FWD ("one input, many filter banks").  Every organism's first layer reads the same raw input batch
// (experiment_worker.py:226-227: one X / g batch for the whole population), so the planner materialises one im2col
// matrix per (input, kernel geometry) (hip_engine.py raw_conv_imcol) and its first-layer convolutions are [M x K8]
// x [K8 x F] problems over the SAME A.  Filter banks are small (layer_transitions.py:39: F = 2^clip(N(4.5, 1)),
// mostly 8 - 32), so one problem per block would re-read A for every organism and fill half-empty MFMA tiles with
// a few k steps of work per block.  Here a block holds its 256 rows of A in registers (KS k steps of 32; the
// matrix's row stride C = K8 <= 32 KS) and walks a run of problems that share it -- tile (first problem, m tile,
// problem count): per problem only its [N x K] filter bank (L2-resident) is loaded, multiplied, BN statistics
// accumulated (GF_BNUSTAT) and the tile stored through the per-wave LDS stage (16-B row-contiguous stores).
// Every problem of a run has N <= 16 NT (one column tile) and plain bf16 output (no GF_ACCUM / GF_OUT_F32).
template <int NT, int KS>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
void g3_shared_fwd_kernel(const GemmDesc* __restrict__ descs, const int4* __restrict__ tiles) {
    constexpr int RT = 4, WROWS = RT * 16, BNB = NT * 16;
    __shared__ __attribute__((aligned(16))) bf16_t ostage[4 * WROWS * BNB];
    __shared__ float bnred[4 * 2 * BNB];
    const int4 td = tiles[blockIdx.x];
    const int nprob = td.z;
    const GemmDesc& d0 = descs[td.x];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r16 = lane & 15, kg = (lane >> 4) * 8;
    const int M = (int)d0.M, C = (int)d0.C;
    const int m_w = td.y * 4 * WROWS + wave * WROWS;
    const rsrc_t rA = mkrsrc(d0.a, (int64_t)M * C * 2);
    Frag fa[KS][RT];
#pragma unroll
    for (int s = 0; s < KS; ++s)
#pragma unroll
        for (int i = 0; i < RT; ++i) {
            const int row = m_w + i * 16 + r16, k = s * 32 + kg;
            fa[s][i].u = bl16(rA, (row < M && k < C) ? row * C + k : -1);
        }
    const int nrows = min(WROWS, M - m_w);
    // a problem's filter bank: loaded while the previous problem's tile is being stored (one bank in flight)
    auto load_bank = [&](const GemmDesc& d, Frag (&fb)[KS][NT]) {
        const int N = (int)d.N, K = (int)d.K;
        const rsrc_t rB = mkrsrc(d.b, (int64_t)N * K * 2);
        const int brow = min(r16, N - 1) * K;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            const int k = s * 32 + kg;
#pragma unroll
            for (int j = 0; j < NT; ++j) {
                const int n = j * 16 + r16;
                fb[s][j].u = bl16(rB, (k < K && n < N) ? brow + j * 16 * K + k : -1);
                if (k + 8 > K) fb[s][j].u = splice(fb[s][j].u, make_uint4(0, 0, 0, 0), K - k);
            }
        }
    };
    Frag fb[KS][NT];
    load_bank(d0, fb);
    for (int q = 0; q < nprob; ++q) {
        const GemmDesc& d = descs[td.x + q];
        const int N = (int)d.N, act = (int)d.act, flags = (int)d.flags;
        f32x4_t acc[RT][NT];
#pragma unroll
        for (int i = 0; i < RT; ++i)
#pragma unroll
            for (int j = 0; j < NT; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][i].v, fb[s][j].v, acc[i][j], 0, 0, 0);
        if (q + 1 < nprob) load_bank(descs[td.x + q + 1], fb);
        const float* bias = reinterpret_cast<const float*>(d.bias);
        if (flags & GF_BNUSTAT) {
            bn_ustat_flush<RT, NT, 1>(d, acc, [&](int i, int rr) { return m_w + i * 16 + rr < M; }, 0, N, bias, act,
                                      bnred, wave, lane, N);
            __syncthreads();                             // (bnred is re-used by the next problem)
        }
        if (nrows > 0)
            wave_store_rows<RT, NT>(&ostage[wave * WROWS * BNB], reinterpret_cast<bf16_t*>(d.out), m_w, nrows, N, false,
                                    acc, bias, act, lane);
    }
}

// part 3: narrow FWD, single-step and direct-fragment FWD / DGRAD
bool gemm3_launch_part3(int mode, int variant, dim3 grid, dim3 block, hipStream_t s, const GemmDesc* dp,
                          const int4* tp) {
    if (mode == MODE_FWD && variant >= 6000 && variant < 7000) {
        const int k = (variant - 6000) % 100;
        const bool st = (variant - 6000) >= 100, sr = (variant - 6000) >= 200;
#define NF(K_) if (k == K_) { if (sr) hipLaunchKernelGGL((g3_narrow_fwd_sr_kernel<K_>), grid, block, 0, s, dp, tp); \
                              else if (st) hipLaunchKernelGGL((g3_narrow_fwd_kernel<K_, true>), grid, block, 0, s, dp, tp); \
                              else hipLaunchKernelGGL((g3_narrow_fwd_kernel<K_, false>), grid, block, 0, s, dp, tp); }
        NF(1) else NF(2) else NF(3) else NF(4)
#undef NF
        else throw std::runtime_error("gemm3: unknown narrow FWD variant " + std::to_string(variant));
        SERANN_CHECK(hipGetLastError());
        return true;
    }
    if (mode == MODE_FWD && variant > 5100 && variant < 5200) {
        const int v = variant - 5100;
#define SH3(NT_, KS_)                                                                                   \
    if (v == NT_ + 10 * KS_) {                                                                          \
        hipLaunchKernelGGL((g3_shared_fwd_kernel<NT_, KS_>), grid, block, 0, s, dp, tp);                \
        SERANN_CHECK(hipGetLastError());                                                                \
        return true;                                                                                    \
    }
        SH3(1, 1) SH3(2, 1) SH3(4, 1) SH3(1, 2) SH3(2, 2) SH3(4, 2) SH3(1, 3) SH3(2, 3) SH3(4, 3)
#undef SH3
        throw std::runtime_error("gemm3: unknown shared-input FWD variant " + std::to_string(variant));
    }
    if (variant >= 5000) {
        const int v = variant - 5000;
#define S3(MODE_, NT_, RT_)                                                                             \
    if (mode == MODE_ && v == NT_ + 10 * RT_) {                                                         \
        hipLaunchKernelGGL((g3_direct_kernel<MODE_, NT_, RT_, false, false, true>), grid, block, 0, s, dp, tp); \
        SERANN_CHECK(hipGetLastError());                                                                \
        return true;                                                                                         \
    }
        S3(MODE_FWD, 1, 4) S3(MODE_FWD, 2, 4) S3(MODE_FWD, 4, 4) S3(MODE_FWD, 8, 2)
        S3(MODE_DGRAD, 1, 4) S3(MODE_DGRAD, 2, 4) S3(MODE_DGRAD, 4, 4) S3(MODE_DGRAD, 8, 2)
#undef S3
        throw std::runtime_error("gemm3: unknown single-step variant " + std::to_string(variant));
    }
    const bool gen = variant >= 1000;
    const bool kw = (variant % 1000) >= 100;
    const int rt = (variant / 10) % 10;
    const int nt = variant % 10;
#define D3(MODE_, NT_, RT_, KW_) \
    if (mode == MODE_ && nt == NT_ && rt == RT_ && kw == KW_) { \
        if (gen) hipLaunchKernelGGL((g3_direct_kernel<MODE_, NT_, RT_, KW_, true>), grid, block, 0, s, dp, tp); \
        else hipLaunchKernelGGL((g3_direct_kernel<MODE_, NT_, RT_, KW_, false>), grid, block, 0, s, dp, tp); \
        SERANN_CHECK(hipGetLastError()); return true; }
#define D3ALL(MODE_) \
    D3(MODE_, 1, 4, false) D3(MODE_, 2, 4, false) D3(MODE_, 4, 4, false) \
    D3(MODE_, 1, 2, false) D3(MODE_, 2, 2, false) D3(MODE_, 4, 2, false) D3(MODE_, 8, 2, false) \
    D3(MODE_, 1, 2, true) D3(MODE_, 2, 2, true) D3(MODE_, 4, 2, true) D3(MODE_, 8, 2, true)
    D3ALL(MODE_FWD)
    D3ALL(MODE_DGRAD)
    D3(MODE_DGRAD, 1, 8, false)          // DGRAD onto <= 16 channels, 8 row tiles per wave (hip_ops.DGRAD_NT1_RT)
#undef D3ALL
#undef D3
    return false;
}
#endif

#if G3_PART(0)
void launch_gemm3(int mode, int variant, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipStream_t s = as_stream(stream);
    const GemmDesc* dp = as_ptr<const GemmDesc>(descs);
    const int4* tp = as_ptr<const int4>(tiles);
    dim3 grid((unsigned)ntiles), block(256);
    if (gemm3_launch_part0(mode, variant, grid, block, s, dp, tp) || gemm3_launch_part1(mode, variant, grid, block, s, dp, tp) ||
        gemm3_launch_part2(mode, variant, grid, block, s, dp, tp) || gemm3_launch_part3(mode, variant, grid, block, s, dp, tp))
        return;
    throw std::runtime_error("gemm3: unknown variant " + std::to_string(variant));
}
#endif
