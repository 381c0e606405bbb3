// Fused first-layer Conv2D + MaxPool2D on the raw single-channel image (gfx950 / CDNA4).
//
// The genome grammar's commonest X-branch opening is ``X_layer = Conv2D(filters=F, kernel_size=k,
// strides=s)(X_layer)`` directly followed by ``X_layer = MaxPool2D(pool_size=p)(X_layer)``
// (layer_transitions.py:9-23, 61-72).  Unfused, the conv output [B][OH][OW][F] -- 9x the pooled
// size for p = 3 -- is written, read by the pool, and in the backward pass a dense dZ of the same
// size is written by the pool scatter and read again by WGRAD.  Here that tensor never exists:
//
// * FWD: per image, the block stages the 28x28 input in LDS and runs one bf16 MFMA per (window
//   offset, 16 pooled positions, 16 filters): A = the patches of the conv positions at that window
//   offset (gathered from LDS), B = the filter bank (registers).  The max over the window offsets is
//   an element-wise max of accumulators in registers (window code packed into the low mantissa bits:
//   2 VALU ops per conv output); bias + activation are applied after the max
//   (both are monotone non-decreasing, so max(act(z + b)) = act(max(z) + b)) and the pooled output
//   and the argmax window offset are the only stores.
// * WGRAD: dW[f][tap] = sum_{b,p} dz[b,p,f] [argmax == w] img[b][pos(p, w) + tap], one MFMA per
//   (window offset, 32 pooled positions, 16 filters, 16 taps): A = dz masked by the argmax (held in
//   registers across the window offsets), B = patches from LDS.  The bias gradient is the plain sum
//   of dz.  The waves' tiles are summed in LDS in wave order and flushed with one Q40 fixed-point
//   atomic per (block, weight) (deterministic).
// There is no DGRAD: the input is the raw image.
//
// One block = 4 waves = one organism x a chunk of images x a group of 64 filters.  Every wave owns
// one LDS image slot; the 4 waves stage their images together between two block barriers.
#include "common.h"
#include "serann_hip.h"

typedef __attribute__((ext_vector_type(8))) __bf16 cp_bf16x8_t;
typedef __attribute__((ext_vector_type(4))) float cp_f32x4_t;

union CpFrag {
    cp_bf16x8_t v;
    bf16_t h[8];
};

constexpr int CP_FWD_IMGS = 16;     // images per FWD block (4 per wave)
constexpr int CP_WGRAD_IMGS = 32;   // images per WGRAD block (8 per wave)
constexpr int CP_MAXPIX = 1024;     // LDS image slot (H * W <= 1024 bf16)

__device__ __forceinline__ void cp_stage_image(bf16_t* __restrict__ slot, const bf16_t* __restrict__ src, int HW,
                                               int lane) {
    if ((HW & 7) == 0 && ((reinterpret_cast<uintptr_t>(src) & 15) == 0)) {
        for (int e = lane * 8; e < HW; e += 512)
            *reinterpret_cast<uint4*>(slot + e) = *reinterpret_cast<const uint4*>(src + e);
    } else {
        for (int e = lane; e < HW; e += 64) slot[e] = src[e];
    }
}

// Image prefetch: the next image of a wave is loaded into registers while the current one is in use,
// so the global latency is off the critical path (H * W <= 1024 bf16 = 128 16-B vectors: 2 per lane).
struct CpImg {
    uint4 v[2];
};

__device__ __forceinline__ bool cp_vec_ok(const ConvPoolDesc& d) {
    return ((d.H * d.W) & 7) == 0 && (d.x & 15) == 0;
}

__device__ __forceinline__ void cp_load_image(CpImg& r, const bf16_t* __restrict__ src, int HW, int lane) {
    const int nv = HW >> 3;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = lane + q * 64;
        if (e < nv) r.v[q] = *reinterpret_cast<const uint4*>(src + e * 8);
    }
}

__device__ __forceinline__ void cp_store_image(bf16_t* __restrict__ slot, const CpImg& r, int HW, int lane) {
    const int nv = HW >> 3;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
        const int e = lane + q * 64;
        if (e < nv) *reinterpret_cast<uint4*>(slot + e * 8) = r.v[q];
    }
}

// Stage image b of this wave (vector path with a one-image register prefetch, or the scalar path).
struct CpStager {
    CpImg next;
    bool vec;
    __device__ __forceinline__ void start(const ConvPoolDesc& d, int b, int lane) {
        vec = cp_vec_ok(d);
        if (vec && b < (int)d.B)
            cp_load_image(next, reinterpret_cast<const bf16_t*>(d.x) + (int64_t)b * d.H * d.W, (int)(d.H * d.W), lane);
    }
    // write image b (prefetched) into the slot and prefetch image b_next
    __device__ __forceinline__ void stage(const ConvPoolDesc& d, bf16_t* slot, int b, int b_next, int lane) {
        const int HW = (int)(d.H * d.W);
        const bf16_t* x = reinterpret_cast<const bf16_t*>(d.x);
        if (vec) {
            if (b < (int)d.B) cp_store_image(slot, next, HW, lane);
            if (b_next < (int)d.B) cp_load_image(next, x + (int64_t)b_next * HW, HW, lane);
        } else if (b < (int)d.B) {
            cp_stage_image(slot, x + (int64_t)b * HW, HW, lane);
        }
    }
};

// Running max of one accumulator element over the window offsets in a few VALU ops: the window code is
// packed into the low 8 mantissa bits and the packed values are max-ed as floats.  On a tie the first
// window in (i, j) scan order wins, as in the reference's MaxPool gradient: for values >= 0 a larger
// mantissa is larger, so the field holds 255 - code; for negative values (sign bit set) a larger mantissa
// is smaller, so it holds the code itself.  The kept value is truncated by at most 2^-15 relative before
// its bf16 rounding.  maxNum drops NaN: a NaN conv output can only come from non-finite filter weights (the
// image is finite), which are flagged per filter instead (cp_nan).
__device__ __forceinline__ float cp_key(float v, int code) {
    const uint32_t u = __float_as_uint(v);
    const uint32_t field = (u >> 31) ? (uint32_t)code : (uint32_t)(255 - code);
    return __uint_as_float((u & 0xffffff00u) | field);
}
__device__ __forceinline__ float cp_key_value(float key) { return __uint_as_float(__float_as_uint(key) & 0xffffff00u); }
__device__ __forceinline__ int cp_key_code(float key) {
    const uint32_t u = __float_as_uint(key);
    return (u >> 31) ? (int)(u & 0xffu) : 255 - (int)(u & 0xffu);
}
__device__ __forceinline__ bf16_t cp_bf16(float v) { return __builtin_bit_cast(bf16_t, (__bf16)v); }

// KT: 32-tap k steps; NT: 16-filter tiles per block (<= 4); G: 16-position groups per pass (ILP)
template <int KT, int NT>
__global__ __launch_bounds__(256) void convpool_fwd_kernel(const ConvPoolDesc* __restrict__ descs,
                                                           const int2* __restrict__ tiles) {
    constexpr int G = 2;
    __shared__ __attribute__((aligned(16))) bf16_t img[4][CP_MAXPIX];
    const int2 td = tiles[blockIdx.x];
    const ConvPoolDesc& d = descs[td.x];
    const int F = (int)d.F, NG = (F + 63) >> 6;
    const int ic = td.y / NG, ng = td.y - ic * NG;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int Bn = (int)d.B, W = (int)d.W;
    const int KW = (int)d.KW, SH = (int)d.SH, SW = (int)d.SW;
    const int PH = (int)d.PH, PW = (int)d.PW, PSH = (int)d.PSH, PSW = (int)d.PSW;
    const int POW = (int)d.POW, npos = (int)(d.POH * d.POW);
    const int taps = (int)(d.KH * d.KW);
    const int f0 = ng * 64;
    const int act = (int)d.act;
    const bf16_t* __restrict__ w = reinterpret_cast<const bf16_t*>(d.w);
    const float* __restrict__ bias = reinterpret_cast<const float*>(d.bias);
    bf16_t* __restrict__ y = reinterpret_cast<bf16_t*>(d.y);
    uint8_t* __restrict__ idx = reinterpret_cast<uint8_t*>(d.idx);
    const int col = lane & 15, kg = lane >> 4;

    // filter bank fragments: B[k = tap][n = filter], lane holds taps 8*kg + j of filter col
    CpFrag bw[KT][NT];
    int toff[KT][8];
#pragma unroll
    for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int tap = kt * 32 + kg * 8 + j;
            const int ky = tap / KW, kx = tap - ky * KW;
            toff[kt][j] = tap < taps ? ky * W + kx : 0;
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int f = f0 + nt * 16 + col;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int tap = kt * 32 + kg * 8 + j;
                bw[kt][nt].h[j] = (tap < taps && f < F) ? w[(int64_t)f * taps + tap] : (bf16_t)0;
            }
        }
    }
    float bv[NT];
    bool cp_nan[NT];                                 // filter has a non-finite weight -> NaN outputs
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int f = f0 + nt * 16 + col;
        bv[nt] = (bias != nullptr && f < F) ? bias[f] : 0.f;
        float sw = 0.f;
#pragma unroll
        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
            for (int j = 0; j < 8; ++j) sw += fabsf(bf2f(bw[kt][nt].h[j]));
        sw += __shfl_xor(sw, 16, 64);
        sw += __shfl_xor(sw, 32, 64);
        cp_nan[nt] = !(sw <= 3.0e38f);
    }

    bf16_t* slot = img[wave];
    // images per block: d.flags when set (a multiple of 4, hip_ops.convpool_imgs), else CP_FWD_IMGS
    const int ipb = d.flags > 0 ? (int)d.flags : CP_FWD_IMGS;
    const int b0 = ic * ipb;
    CpStager st;
    st.start(d, b0 + wave, lane);
    for (int it = 0; it < ipb / 4; ++it) {
        const int b = b0 + it * 4 + wave;
        __syncthreads();
        st.stage(d, slot, b, it + 1 < ipb / 4 ? b + 4 : Bn, lane);
        __syncthreads();
        if (b >= Bn) continue;
        for (int pg = 0; pg < npos; pg += 16 * G) {
            // A rows: pooled positions pg + 16 g + col (clamped; rows past npos are computed and dropped)
            int base[G];
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const int pa = min(pg + g * 16 + col, npos - 1);
                const int poh = pa / POW, pw_ = pa - poh * POW;
                base[g] = poh * PSH * SH * W + pw_ * PSW * SW;
            }
            float best[G][NT][4];                    // packed (value, 255 - window code) keys
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) best[g][nt][r] = -3.0e38f;
            // window offsets in (i, j) scan order; the patches of window wi + 1 are read from LDS while
            // window wi runs its MFMAs and max updates (register double buffer)
            const int nwin = PH * PW;
            CpFrag a[G][KT], an[G][KT];
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int kt = 0; kt < KT; ++kt)
#pragma unroll
                    for (int j = 0; j < 8; ++j) a[g][kt].h[j] = slot[base[g] + toff[kt][j]];
            int wi_i = 0, wi_j = 0;
            for (int wi = 0; wi < nwin; ++wi) {
                {
                    // next window offset (clamped to the last one: a harmless re-read)
                    int ni = wi_i, nj = wi_j + 1;
                    if (nj == PW) { nj = 0; ++ni; }
                    if (ni == PH) { ni = PH - 1; nj = PW - 1; }
                    const int noff = ni * SH * W + nj * SW;
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int kt = 0; kt < KT; ++kt)
#pragma unroll
                            for (int j = 0; j < 8; ++j) an[g][kt].h[j] = slot[base[g] + noff + toff[kt][j]];
                }
                const int code = wi;
                {
                    cp_f32x4_t acc[G][NT];
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt) {
                            acc[g][nt] = cp_f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                            for (int kt = 0; kt < KT; ++kt)
                                acc[g][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[g][kt].v, bw[kt][nt].v,
                                                                                     acc[g][nt], 0, 0, 0);
                        }
#pragma unroll
                    for (int g = 0; g < G; ++g)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                            for (int r = 0; r < 4; ++r)
                                best[g][nt][r] = fmaxf(best[g][nt][r], cp_key(acc[g][nt][r], code));
                }
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int kt = 0; kt < KT; ++kt) a[g][kt] = an[g][kt];
                if (++wi_j == PW) { wi_j = 0; ++wi_i; }
            }
            // D[row = pooled position][col = filter]: lane holds rows 4*kg + r of column col
#pragma unroll
            for (int g = 0; g < G; ++g)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int f = f0 + nt * 16 + col;
                    if (f >= F) continue;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int p = pg + g * 16 + kg * 4 + r;
                        if (p >= npos) continue;
                        const int64_t o = ((int64_t)b * npos + p) * F + f;
                        const float key = best[g][nt][r];
                        const float v = cp_nan[nt] ? __builtin_nanf("") : cp_key_value(key);
                        y[o] = cp_bf16(apply_act(v + bv[nt], act));
                        if (idx != nullptr) idx[o] = (uint8_t)cp_key_code(key);
                    }
                }
        }
    }
}

template <int KT, int NT>
__global__ __launch_bounds__(256) void convpool_wgrad_kernel(const ConvPoolDesc* __restrict__ descs,
                                                             const int2* __restrict__ tiles) {
    constexpr int TT = 2 * KT;      // 16-tap output tiles
    __shared__ __attribute__((aligned(16))) bf16_t img[4][CP_MAXPIX];
    const int2 td = tiles[blockIdx.x];
    const ConvPoolDesc& d = descs[td.x];
    const int F = (int)d.F, NG = (F + 63) >> 6;
    const int ic = td.y / NG, ng = td.y - ic * NG;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int Bn = (int)d.B, W = (int)d.W;
    const int KW = (int)d.KW, SH = (int)d.SH, SW = (int)d.SW;
    const int PH = (int)d.PH, PW = (int)d.PW, PSH = (int)d.PSH, PSW = (int)d.PSW;
    const int POW = (int)d.POW, npos = (int)(d.POH * d.POW);
    const int taps = (int)(d.KH * d.KW);
    const int f0 = ng * 64;
    const int tts = min(TT, (taps + 15) >> 4);
    const int act = (int)d.act;
    const bf16_t* __restrict__ dy = reinterpret_cast<const bf16_t*>(d.dy);
    const bf16_t* __restrict__ y = reinterpret_cast<const bf16_t*>(d.y);
    const uint8_t* __restrict__ idx = reinterpret_cast<const uint8_t*>(d.idx);
    const int col = lane & 15, kg = lane >> 4;

    // B columns = taps tt*16 + col: their offsets inside the image
    int toff[TT];
#pragma unroll
    for (int tt = 0; tt < TT; ++tt) {
        const int tap = tt * 16 + col;
        const int ky = tap / KW, kx = tap - ky * KW;
        toff[tt] = tap < taps ? ky * W + kx : 0;
    }
    cp_f32x4_t acc[NT][TT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int tt = 0; tt < TT; ++tt) acc[nt][tt] = cp_f32x4_t{0.f, 0.f, 0.f, 0.f};
    float bsum[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) bsum[nt] = 0.f;

    bf16_t* slot = img[wave];
    // images per block: d.flags when set (a multiple of 4: hip_ops.convpool_imgs lowers it until the
    // problem has enough blocks to spread over the chip), else CP_WGRAD_IMGS
    const int ipb = d.flags > 0 ? (int)d.flags : CP_WGRAD_IMGS;
    const int b0 = ic * ipb;
    CpStager st;
    st.start(d, b0 + wave, lane);
    for (int it = 0; it < ipb / 4; ++it) {
        const int b = b0 + it * 4 + wave;
        __syncthreads();
        st.stage(d, slot, b, it + 1 < ipb / 4 ? b + 4 : Bn, lane);
        __syncthreads();
        if (b >= Bn) continue;
        for (int pk = 0; pk < npos; pk += 32) {
            // A operand (dz as bf16 bits, [row = filter][k = pooled position]) and its argmax codes for
            // the 8 positions pk + 8*kg + j of this lane: loaded once, masked per window offset.  The
            // loads are unconditional (clamped indices, masked after) so they issue back to back.
            bf16_t dz[NT][8];
            int code[NT][8];
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int fr = f0 + nt * 16 + col;
                const int f = min(fr, F - 1);
                bf16_t gv[8], yv[8];
                uint8_t cv[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int p = min(pk + kg * 8 + j, npos - 1);
                    const int64_t o = ((int64_t)b * npos + p) * F + f;
                    gv[j] = dy[o];
                    cv[j] = idx[o];
                    if (act != ACT_LINEAR) yv[j] = y[o];
                }
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const bool valid = fr < F && pk + kg * 8 + j < npos;
                    float g = bf2f(gv[j]);
                    if (act != ACT_LINEAR) g *= act_grad_from_y(bf2f(yv[j]), act);
                    g = valid ? g : 0.f;
                    dz[nt][j] = f2bf(g);
                    code[nt][j] = valid ? (int)cv[j] : -1;
                    bsum[nt] += g;
                }
            }
            // B rows: pooled positions pk + 8*kg + j (clamped; their dz is 0)
            int pbase[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const int p = min(pk + kg * 8 + j, npos - 1);
                const int poh = p / POW, pw_ = p - poh * POW;
                pbase[j] = poh * PSH * SH * W + pw_ * PSW * SW;
            }
            // window offsets in (i, j) scan order; the patches of window wi + 1 are read from LDS while
            // window wi runs (register double buffer)
            const int nwin = PH * PW;
            CpFrag bp[TT], bpn[TT];
#pragma unroll
            for (int tt = 0; tt < TT; ++tt)
#pragma unroll
                for (int j = 0; j < 8; ++j) bp[tt].h[j] = slot[pbase[j] + toff[tt]];
            int wi_i = 0, wi_j = 0;
            for (int wi = 0; wi < nwin; ++wi) {
                {
                    int ni = wi_i, nj = wi_j + 1;
                    if (nj == PW) { nj = 0; ++ni; }
                    if (ni == PH) { ni = PH - 1; nj = PW - 1; }
                    const int noff = ni * SH * W + nj * SW;
#pragma unroll
                    for (int tt = 0; tt < TT; ++tt)
#pragma unroll
                        for (int j = 0; j < 8; ++j) bpn[tt].h[j] = slot[pbase[j] + noff + toff[tt]];
                }
                CpFrag a[NT];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int j = 0; j < 8; ++j) a[nt].h[j] = code[nt][j] == wi ? dz[nt][j] : (bf16_t)0;
#pragma unroll
                for (int tt = 0; tt < TT; ++tt) {
                    if (tt >= tts) break;
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[nt][tt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[nt].v, bp[tt].v, acc[nt][tt], 0, 0, 0);
                }
#pragma unroll
                for (int tt = 0; tt < TT; ++tt) bp[tt] = bpn[tt];
                if (++wi_j == PW) { wi_j = 0; ++wi_i; }
            }
        }
    }
    // D[row = filter][col = tap]: lane holds filters 4*kg + r of tap column col.  The 4 waves' tiles are
    // summed in LDS in fixed wave order (deterministic), then flushed with one Q40 fixed-point atomic per
    // (block, weight): with one image per wave (4-image blocks) per-wave flushes would cost 4x the atomics.
    constexpr int RW = TT * 16;
    __shared__ float red[NT * 16 * RW];
    for (int w = 0; w < 4; ++w) {
        if (wave == w) {
#pragma unroll
            for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                for (int tt = 0; tt < TT; ++tt) {
                    if (tt >= tts) break;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int e = (nt * 16 + kg * 4 + r) * RW + tt * 16 + col;
                        red[e] = (w == 0 ? 0.f : red[e]) + acc[nt][tt][r];
                    }
                }
        }
        __syncthreads();
    }
    long long* __restrict__ dw = reinterpret_cast<long long*>(d.dw);     // Q40 gradient arena (common.h)
    const int tw = tts * 16;
    for (int e = threadIdx.x; e < NT * 16 * tw; e += 256) {
        const int row = e / tw, tap = e - row * tw;
        const int f = f0 + row;
        if (f < F && tap < taps) fx_add(dw + (int64_t)f * taps + tap, red[row * RW + tap]);
    }
    long long* __restrict__ dbias = reinterpret_cast<long long*>(d.dbias);
    if (dbias != nullptr) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            float s = bsum[nt];
            s += __shfl_xor(s, 16, 64);
            s += __shfl_xor(s, 32, 64);
            const int f = f0 + nt * 16 + col;
            if (kg == 0 && f < F) fx_add(dbias + f, s);
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Host-side limits mirrored in hip_ops.convpool_ok: H * W <= CP_MAXPIX, KH * KW <= 96.
// variant = kt * 8 + nt (hip_ops.convpool_variant): kt in 1..3 k steps, nt in 1..4 filter tiles per block.
template <int KT>
static void launch_convpool_kt(int backward, int nt, dim3 grid, hipStream_t s, const ConvPoolDesc* dp,
                               const int2* tp) {
    const dim3 block(256);
#define CP_LAUNCH(NT_)                                                                          \
    do {                                                                                       \
        if (backward) hipLaunchKernelGGL((convpool_wgrad_kernel<KT, NT_>), grid, block, 0, s, dp, tp); \
        else hipLaunchKernelGGL((convpool_fwd_kernel<KT, NT_>), grid, block, 0, s, dp, tp);     \
    } while (0)
    switch (nt) {
        case 1: CP_LAUNCH(1); break;
        case 2: CP_LAUNCH(2); break;
        case 3: CP_LAUNCH(3); break;
        default: CP_LAUNCH(4); break;
    }
#undef CP_LAUNCH
}

void launch_convpool(int backward, int variant, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    const int kt = variant >> 3, nt = variant & 7;
    if (kt < 1 || kt > 3 || nt < 1 || nt > 4) throw std::runtime_error("convpool: bad variant");
    const dim3 grid((unsigned)ntiles);
    const ConvPoolDesc* dp = as_ptr<const ConvPoolDesc>(descs);
    const int2* tp = as_ptr<const int2>(tiles);
    hipStream_t s = as_stream(stream);
    if (kt == 1) launch_convpool_kt<1>(backward, nt, grid, s, dp, tp);
    else if (kt == 2) launch_convpool_kt<2>(backward, nt, grid, s, dp, tp);
    else launch_convpool_kt<3>(backward, nt, grid, s, dp, tp);
    SERANN_CHECK(hipGetLastError());
}
