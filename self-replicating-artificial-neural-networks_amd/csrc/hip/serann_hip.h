// Host-side launcher declarations for the SeRANN-AMD HIP kernels (gfx950).
// All pointers/streams cross the Python boundary as uint64 integers (pybind11 module.hip).
#pragma once
#include <stdint.h>

// ---- descriptor layouts (all fields int64 so Python can build them as int64 arrays) ----------
// Grouped implicit-GEMM convolution problem (see gemm3.hip for the per-mode meaning of a/b/out).
struct GemmDesc {
    int64_t a, b, out, bias, aux;     // aux: DGRAD/FWD accumulate source (unused = 0)
    int64_t H, W, C, OH, OW, F, KH, KW, SH, SW;
    int64_t M, N, K;
    int64_t act, flags;
    // host-computed fast-division magics (low 32 bits: multiplier, bits 32..39: shift) of the
    // divisors the v3 kernels need: q = (umulhi(n, mul) + n) >> shift, exact for 0 <= n < 2^31.
    int64_t dvC, dvKW, dvOW, dvOHW, dvF, dvW, dvHW, dvSH, dvSW;
    int64_t dvCp;     // magic of Cp = C rounded up to 8 (LDS-halo conv kernels)
    int64_t kper;     // GF_SPLITWS: k steps (32) per split; split s writes aux + (sbase + s) * M * N (fp32)
    int64_t ldb;      // LDS-tiled kernel: B row stride (0: K) -- a K slice [.., col0 + K) of a wider [N][ldb] matrix
    int64_t sbase;    // GF_SPLITWS: first workspace slot of this problem (K slices of one output share a workspace)
    int64_t ldo;      // WGRAD (64-row LDS kernel): output row stride (0: N) -- a column slice of a wider dW
    int64_t adam;     // GF_ADAM: device AdamCtx of the parameter arenas (WGRAD applies Adam to its tile)
    int64_t ext;      // GF_NBNSUM: device NbnDesc of the fused raw-input Dense -> BN pair whose dY this DGRAD is
};
// The parameter / gradient / moment arenas of a population engine (same layout, element e of each is the
// same parameter) and the device Adam scalars, for WGRAD epilogues that apply the optimizer step (GF_ADAM).
struct AdamCtx {
    int64_t p, m, v, pbf, g, lr_t;   // fp32, m / v (fp32, or bf16 / log16: mode), bf16, Q40 int64 arenas; device lr_t (float)
    int64_t org_off, diverged, norg; // divergence flags (common.h flag_diverged; org_off = 0: none)
    float b1, b2, eps;
    int32_t mode;                    // common.h MOM_F32 / MOM_16: storage of the m and v arenas
};
enum GemmFlags : int64_t {
    GF_VEC_A = 1,         // A operand chunks are contiguous 8-element vectors
    GF_VEC_B = 2,         // B operand chunks are contiguous 8-element vectors
    GF_ACCUM = 4,         // out += result (bf16 read-modify-write)
    GF_OUT_F32 = 8,       // FWD: write fp32 output (heads)
    GF_WSTORE = 16,       // WGRAD: single m-split -> plain stores of the Q40 gradient instead of atomics
    GF_SPLITWS = 64,      // FWD (LDS-tiled kernel): k range split over blocks; each split stores its raw
                          // fp32 partial tile to the workspace aux[split][M][N]; splitk_finalize sums
                          // the splits in order and applies bias + activation (no atomics, no zeroing)
    GF_BNSTAT = 128,      // FWD narrow kernel: also accumulate the consuming BatchNorm's phase-0 statistics
                          // into aux (shifted sums, wide fixed point: the BN statistics workspace format)
    GF_ADAM = 256,        // WGRAD with GF_WSTORE (sole writer of its tile): apply Keras-Adam to the tile in the
                          // epilogue instead of storing the gradient; the arena-wide Adam pass skips it
    GF_NOSTORE = 32,      // FWD narrow kernel with GF_BNSTAT: statistics only, the output is never stored
                          // (its only consumer recomputes it: nbn.hip)
    GF_BNUSTAT = 1024,    // FWD (conv-halo, direct non-KW, LDS-tiled without k splits): also accumulate the consuming
                          // BatchNorm's phase-0 statistics, unshifted, into aux (its workspace; BnDesc flag 512)
    GF_WSLAB = 2048,      // WGRAD (Dense / 1x1 kernels), m-split problem: a block stores its fp32 partial tile to the
                          // slab of its split, ext + (kt0 / kper) * M * N (plain stores, every element written once
                          // per split); wgrad_finalize sums the S slabs in split order (WgFinDesc with C = Cp = N) and
                          // stores the Q40 gradient or applies Adam -- no fixed-point atomics, so the reduction can
                          // be split as finely as the grid needs
    GF_NBNSUM = 512,      // DGRAD (LDS-tiled kernel) producing the output gradient of a fused raw-input
                          // Dense (1 input channel) -> BN pair (ext = its NbnDesc): instead of storing dY, reduce the BN / Dense
                          // backward sums of every column over the block's rows into NbnDesc::part; nbn
                          // phase 6 finishes them (nbn.hip)
};
enum GemmMode : int { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

void launch_gemm3(int mode, int variant, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_transpose_weights(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);

// ---- optimizer --------------------------------------------------------------------------------
void launch_adam(uint64_t p, uint64_t g, uint64_t m, uint64_t v, uint64_t pbf, uint64_t step, uint64_t lr_t,
                 int64_t n, float lr, float b1, float b2, float eps, uint64_t stream, int mode);
void launch_f32_to_bf16(uint64_t x, uint64_t y, int64_t n, uint64_t stream);

// ---- auxiliary grouped kernels (aux.hip) ------------------------------------------------------
void launch_gather_batch(uint64_t x_all, uint64_t g_all, uint64_t y_all, uint64_t perm, uint64_t counter,
                         int64_t base, int64_t B, int64_t n_perm, int64_t x_cols, int64_t g_cols,
                         uint64_t x_out, uint64_t g_out, uint64_t y_out, uint64_t stream);
void launch_counter_add(uint64_t counter, int64_t value, uint64_t stream);
void launch_bn(int phase, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_pool(int backward, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_ew(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_copy2d(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_loss(int train, uint64_t descs, int64_t nprob, int64_t B, uint64_t stream, int64_t nvalid);
void launch_memset32(uint64_t ptr, int64_t n, uint64_t stream);
void launch_imcol(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_concrete_fwd(uint64_t logits, uint64_t u, uint64_t s, uint64_t z, uint64_t kl, int64_t B, int64_t G,
                         int64_t A, double t, double tp, uint64_t seed, uint64_t offset, uint64_t stream, uint64_t zb);
void launch_concrete_bwd(uint64_t s, uint64_t z, uint64_t gz, uint64_t gkl, uint64_t dlogits, int64_t B, int64_t G,
                         int64_t A, double t, double tp, uint64_t stream, int bf16);
void launch_cat_loglik_fwd(uint64_t z, uint64_t x, uint64_t out, int64_t B, int64_t L, int64_t V, uint64_t stream,
                           int bf16);
void launch_cat_loglik_bwd(uint64_t z, uint64_t x, uint64_t gout, uint64_t dz, int64_t B, int64_t L, int64_t V,
                           uint64_t stream, int bf16);
void launch_onehot(uint64_t tok, uint64_t out, int64_t rows, int64_t V, uint64_t stream);
void launch_splitk_finalize(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
// Split WGRAD finalize (aux.hip): a WGRAD problem split over S row ranges leaves one fp32 slab per split,
// ws[S][M][ldp] with ldp = (N / C) * Cp (the kernel's padded (tap, Cp) columns; Cp = C for Dense), written
// with plain stores; the finalize adds the S slabs IN SPLIT ORDER (bitwise reproducible, no atomics) and
// stores the Q40 gradient out[M][N] (N = taps * C) -- or, with adam != 0, applies Keras-Adam to those
// parameters (the gradient quantised as the Q40 arena would hold it; the arena-wide Adam pass skips them).
struct WgFinDesc { int64_t ws, out, adam, M, N, C, Cp, S, ldo, flags; };   // ldo: out row stride (0: N)
constexpr int WGFIN_ELEMS = 64;       // outputs per block
void launch_wgrad_finalize(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_embed_gather(uint64_t tokens, uint64_t table, uint64_t out, int64_t rows, int64_t E, int64_t V,
                         uint64_t stream);
void launch_group_argmax(uint64_t logits, uint64_t out, int64_t ngroups, int64_t V, uint64_t stream);

// ---- auxiliary descriptors (int64 fields) ----------------------------------------------------
struct TransDesc { int64_t src, dst, F, P, C; };                             // P = KH*KW
// BatchNorm statistics workspace: BN_WS_STRIPES copies of the [2C] sums, each a wide fixed-point pair
// (hi, lo) of int64 (common.h fxw_add), one copy per block-index residue (same-address atomics serialise
// in L2), summed in integer arithmetic by the readers (common.h fxw_sum): [stripe][2C][2] int64
constexpr int BN_WS_STRIPES = 8;
struct BnDesc {
    int64_t x, y, dy, dx, gamma, beta, mm, mv, mean, invstd, ws, dgamma, dbeta;
    int64_t pdb;              // phase 5: Q40 bias gradient of the GEMM producing x (0 = none), reduced from
                              // the fp32 dZ before it is rounded to bf16 (serann_hip.h note below)
    int64_t R, C, flags;      // flags: 1 has_gamma, 2 has_beta, 4 accumulate dx, 8 no dx, 64 moving variance
                              // with n / (n - 1) (standard BN) instead of BatchNormalizationF16's n / (n - 1 - eps),
                              // bits 4-5 (phase 5): act of the GEMM producing x -- dx is written as that
                              // GEMM's dZ = dx * act'(x) (x is its output), so its backward reads no Y.
                              // pdb: that GEMM's bias gradient sum(dZ) is taken here, in fp32: when the act
                              // is linear it is mathematically zero (BN removes the mean), and summing the
                              // bf16-rounded dZ over ~600k rows instead leaves O(sqrt(R) * 2^-9) noise.
                              // flags 128 / 256: pdb is ONE bias element that receives -/+ sum(dx) over all
                              // channels (a Dense(units=1) subtracted from / added to the BN input)
                              // flag 512: ws holds unshifted phase-0 sums from the producer (GF_BNUSTAT)
    double eps, momentum;
};
struct PoolDesc { int64_t x, y, idx, dy, dx, B, H, W, C, OH, OW, PH, PW, SH, SW, flags; };  // flags: 1 accum
struct CopyDesc { int64_t src, dst, rows, cols, src_stride, dst_stride, flags; };           // flags: 1 accum
// Strided elementwise map / reduction (ew.hip): out[j] (+)= sum_r (ca A[a(j,r)] + cb B[b(j,r)]) + c over a
// dense 4-d destination D and a 4-d reduction box R; strides in elements; b = 0: no B; flags: 1 accumulate
struct EwDesc {
    int64_t a, b, out;
    int64_t D[4], R[4], aJ[4], aR[4], bJ[4], bR[4];
    float ca, cb, c, pad;
    int64_t flags;
};
constexpr int EW_ELEMS = 2048;        // destination elements per block
struct SplitFinDesc { int64_t ws, out, bias, M, N, S, act, flags; };      // flags: 1 = fp32 output
// Fused first-layer Conv2D + MaxPool2D on a raw single-channel image (convpool.hip).  w: bf16 [F][KH*KW];
// bias / dw / dbias: fp32 (0 = none); y / dy: bf16 pooled [B][POH][POW][F]; idx: u8 argmax window offset.
struct ConvPoolDesc {
    int64_t x, w, bias, y, idx, dy, dw, dbias;
    int64_t B, H, W, F, KH, KW, SH, SW, OH, OW, PH, PW, PSH, PSW, POH, POW, act, flags;
};
void launch_convpool(int backward, int kt, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
// Fused genotype-branch chain Conv1D(raw genotype) -> Dense -> [BatchNormalization] (gchain.hip).
// g: bf16 [B][L0]; w1: bf16 [F1][T]; w2: bf16 [F2][F1]; biases / BN parameters / gradients fp32;
// y, dy: bf16 [B * L1][F2] (the BN output when GC_BN, else the Dense output); rows per block rpb.
struct GChainDesc {
    int64_t g, w1, b1, w2, b2, y, dy, dw1, db1, dw2, db2;
    int64_t gamma, beta, mm, mv, mean, invstd, ws, wsb, dgamma, dbeta;
    int64_t B, L0, L1, T, S, F1, F2, act1, act2, flags, rpb;
    int64_t dvL1;     // fast-division magic of L1 (hip_ops.fast_div_magic)
    double eps, momentum;
};
enum GChainFlags : int64_t { GC_BN = 1, GC_GAMMA = 2, GC_BETA = 4, GC_TRAIN = 8 };
void launch_gchain(int mode, int variant, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
struct ImcolDesc { int64_t x, out, B, H, W, OH, OW, KH, KW, SH, SW, K8; };   // single-channel input
// Replication epilogue (K16): rows [0, rows) of one organism's fp32 head logits [B][NC + L] -> offspring
// bits, packed MSB-first (numpy.packbits order) into out [rows][ceil(L / 8)] uint8.
struct RepBitsDesc { int64_t logits, out, rows, NC, L; };
// Fused raw-input Dense (K <= 4 input channels, 8 <= F <= 256 units) -> BatchNormalization, training
// (nbn.hip).  x: the raw input rows (bf16, row stride ldx); w: bf16 [F][K]; bias fp32 (0 = none); y: the BN
// output; dy: its gradient; ws / wsb: forward / backward wide statistics workspaces (BnDesc layout);
// dw, db, dgamma, dbeta: Q40 gradient arena (0 = none); flags as BnDesc (1 gamma, 2 beta, 64 n/(n-1)).
struct NbnDesc {
    int64_t x, w, bias, y, dy, gamma, beta, mm, mv, mean, invstd, ws, wsb, dw, db, dgamma, dbeta;
    int64_t R, F, K, ldx, act, flags;
    double eps, momentum;
    // GF_NBNSUM / phase 6 (K = 1 pairs): fp32 partial sums [mtiles][N][NBN_NSUM] written by the consumer's
    // DGRAD epilogue, one slot per 128-row m tile (N = np * F columns; BN row of (m, n) = m * np + n / F)
    int64_t part, mtiles, np;
};
constexpr int NBN_NSUM = 8;
// nbn tiles (int4): (problem, first super-row, end super-row, 1 for the problem's first block); the planner
// sizes the ranges (hip_ops.nbn_tiles)
void launch_adam_scalars(uint64_t step, uint64_t lr_t, float lr, float b1, float b2, uint64_t stream);
void launch_adam_update(uint64_t p, uint64_t g, uint64_t m, uint64_t v, uint64_t pbf, uint64_t lr_t, int64_t n,
                        float b1, float b2, float eps, uint64_t skip, uint64_t stream, int mode, uint64_t org_off,
                        uint64_t diverged, int64_t norg);
void launch_nbn(int phase, int k, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);
void launch_rep_bits(uint64_t descs, int64_t ndesc, int64_t max_rows, int64_t row_bytes, uint64_t stream);
struct LossDesc {
    int64_t logits, dlogits, labels, target, metrics, NC, L, B, flags;
    double lb;
};

// Binary-genotype factorisation of a raw-genotype Dense -> BN pair's merged-Dense K slice (bnbn.hip).  g: raw genotype
// bf16 [B][L] in {0, 1}; w / bias / act: the pair's Dense (K = 1); gamma / beta / mean / invstd: its BN (flags 1 gamma,
// 2 beta, 4 BIN_VEC4: bin_sw's 4-column lanes); wc: the consumer's bf16 weights at the slice (W[n][col + j], row stride ldw), Nc units; E fp32 [L][Nc],
// C0 fp32 [Nc]; slab: the slice's fp32 slot [B][Nc] of the consumer's split-K workspace; Hm, cs: Q40 H [Nc][L] and
// column sums of dZ [Nc] (written by a gemm3 WGRAD launch); part: NbnDesc::part slot 0 [L F][8]; dw: the slice's Q40
// gradient (row stride ldw); dbias: the consumer's Q40 bias gradient when the slice carries it; adam: AdamCtx (0: store)
struct BinDesc {
    int64_t g, w, bias, gamma, beta, mean, invstd, act, flags;
    int64_t wc, ldw, Nc, L, F, B;
    int64_t E, C0, slab, Hm, cs, part, dw, dbias, adam;
    int64_t ns;   // bin_sw row splits: split s sums rows [s Nc / ns, (s + 1) Nc / ns) into part slot s
};
// phase 0 bin_prep (problem, n), 1 bin_fwd (problem, 32 rows), 3 bin_sw (problem, column block * ns + split)
void launch_bin(int phase, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream);

