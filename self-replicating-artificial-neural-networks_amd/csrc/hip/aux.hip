// Auxiliary grouped kernels for the SeRANN population engine:
//   gather_batch (K14), act_bwd + bias grad (K04/K09 epilogue backward), fused BatchNormalizationF16
//   train/infer/backward (K05/K06), maxpool fwd/bwd (K03), concat copies (K08), fused heads loss
//   (softmax-CE + sigmoid-MSE + accuracy + dlogits, K10/K11/K12/K17), popstats (K20-K22).
// Grouped kernels take a descriptor array and an int2 tile table (problem, chunk).
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
// dz = dy * act'(y);  dbias += column sums of dz.   Chunk = 64 rows.
constexpr int ACT_ROWS = 64;
constexpr int SEG = 1024;

__global__ __launch_bounds__(256) void act_bwd_kernel(const ActBwdDesc* __restrict__ descs,
                                                      const int2* __restrict__ tiles) {
    __shared__ float colsum[SEG];
    const int2 td = tiles[blockIdx.x];
    const ActBwdDesc& d = descs[td.x];
    const int M = (int)d.M, N = (int)d.N, act = (int)d.act;
    const bool write = d.flags & 1;
    const bf16_t* dy = reinterpret_cast<const bf16_t*>(d.dy);
    const bf16_t* y = reinterpret_cast<const bf16_t*>(d.y);
    bf16_t* dz = reinterpret_cast<bf16_t*>(d.dz);
    float* dbias = reinterpret_cast<float*>(d.dbias);
    const int r0 = td.y * ACT_ROWS;
    const int r1 = min(M, r0 + ACT_ROWS);
    for (int seg = 0; seg < N; seg += SEG) {
        const int sn = min(SEG, N - seg);
        for (int i = threadIdx.x; i < sn; i += blockDim.x) colsum[i] = 0.f;
        __syncthreads();
        const int total = (r1 - r0) * sn;
        for (int e = threadIdx.x; e < total; e += blockDim.x) {
            const int r = r0 + e / sn, c = e % sn;
            const int64_t off = (int64_t)r * N + seg + c;
            float g = bf2f(dy[off]);
            if (act != ACT_LINEAR) g *= act_grad_from_y(bf2f(y[off]), act);
            if (write) dz[off] = f2bf(g);
            if (dbias) atomicAdd(&colsum[c], g);
        }
        __syncthreads();
        if (dbias)
            for (int i = threadIdx.x; i < sn; i += blockDim.x) atomicAdd(&dbias[seg + i], colsum[i]);
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// BatchNormalizationF16 (channel-last, rows x C).  Phases:
//   0: ws[c] += sum x            1: ws[C+c] += sum (x-mean)^2         2: train apply (+ moving stats)
//   3: inference apply           4: ws2: sum dy, sum dy*xhat          5: backward apply (+ dgamma/dbeta)
constexpr int BN_ROWS = 64;

__global__ __launch_bounds__(256) void bn_kernel(const BnDesc* __restrict__ descs, const int2* __restrict__ tiles,
                                                 int phase) {
    __shared__ float s0[SEG];
    __shared__ float s1[SEG];
    const int2 td = tiles[blockIdx.x];
    const BnDesc& d = descs[td.x];
    const int R = (int)d.R, C = (int)d.C;
    const int flags = (int)d.flags;
    const float eps = (float)d.eps;
    const bf16_t* x = reinterpret_cast<const bf16_t*>(d.x);
    float* ws = reinterpret_cast<float*>(d.ws);
    const float* gamma = reinterpret_cast<const float*>(d.gamma);
    const float* beta = reinterpret_cast<const float*>(d.beta);
    float* mean = reinterpret_cast<float*>(d.mean);
    float* invstd = reinterpret_cast<float*>(d.invstd);
    const int r0 = td.y * BN_ROWS, r1 = min(R, r0 + BN_ROWS);
    const float invR = 1.f / (float)R;

    if (phase == 0 || phase == 1 || phase == 4) {
        for (int seg = 0; seg < C; seg += SEG) {
            const int sn = min(SEG, C - seg);
            for (int i = threadIdx.x; i < sn; i += blockDim.x) { s0[i] = 0.f; s1[i] = 0.f; }
            __syncthreads();
            const int total = (r1 - r0) * sn;
            for (int e = threadIdx.x; e < total; e += blockDim.x) {
                const int r = r0 + e / sn, c = e % sn, ch = seg + c;
                const int64_t off = (int64_t)r * C + ch;
                const float xv = bf2f(x[off]);
                if (phase == 0) {
                    atomicAdd(&s0[c], xv);
                } else if (phase == 1) {
                    const float dv = xv - ws[ch] * invR;
                    atomicAdd(&s0[c], dv * dv);
                } else {
                    const float dyv = bf2f(reinterpret_cast<const bf16_t*>(d.dy)[off]);
                    const float xh = (xv - mean[ch]) * invstd[ch];
                    atomicAdd(&s0[c], dyv);
                    atomicAdd(&s1[c], dyv * xh);
                }
            }
            __syncthreads();
            for (int i = threadIdx.x; i < sn; i += blockDim.x) {
                if (phase == 0) atomicAdd(&ws[seg + i], s0[i]);
                else if (phase == 1) atomicAdd(&ws[C + seg + i], s0[i]);
                else { atomicAdd(&ws[seg + i], s0[i]); atomicAdd(&ws[C + seg + i], s1[i]); }
            }
            __syncthreads();
        }
        return;
    }
    bf16_t* y = reinterpret_cast<bf16_t*>(d.y);
    if (phase == 2 || phase == 3) {
        if (phase == 2 && td.y == 0) {
            // per-channel statistics, moving averages (K.moving_average_update), saved for backward
            const float mom = (float)d.momentum;
            float* mm = reinterpret_cast<float*>(d.mm);
            float* mv = reinterpret_cast<float*>(d.mv);
            for (int c = threadIdx.x; c < C; c += blockDim.x) {
                const float mu = ws[c] * invR;
                const float var = ws[C + c] * invR;
                const float n = (float)R;
                const float unbiased = var * (n / (n - (1.f + eps)));
                mm[c] = mm[c] * mom + mu * (1.f - mom);
                mv[c] = mv[c] * mom + unbiased * (1.f - mom);
            }
        }
        const int total = (r1 - r0) * C;
        for (int e = threadIdx.x; e < total; e += blockDim.x) {
            const int r = r0 + e / C, c = e % C;
            const int64_t off = (int64_t)r * C + c;
            float mu, is;
            if (phase == 2) {
                mu = ws[c] * invR;
                is = rsqrtf(ws[C + c] * invR + eps);
                if (td.y == 0 && r == r0) { mean[c] = mu; invstd[c] = is; }
            } else {
                mu = reinterpret_cast<const float*>(d.mm)[c];
                is = rsqrtf(reinterpret_cast<const float*>(d.mv)[c] + eps);
            }
            float v = (bf2f(x[off]) - mu) * is;
            if (flags & 1) v *= gamma[c];
            if (flags & 2) v += beta[c];
            y[off] = f2bf(v);
        }
        return;
    }
    // phase 5: backward apply
    if (td.y == 0) {
        float* dg = reinterpret_cast<float*>(d.dgamma);
        float* db = reinterpret_cast<float*>(d.dbeta);
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            if (flags & 1) dg[c] += ws[C + c];
            if (flags & 2) db[c] += ws[c];
        }
    }
    if (flags & 8) return;
    const bf16_t* dy = reinterpret_cast<const bf16_t*>(d.dy);
    bf16_t* dx = reinterpret_cast<bf16_t*>(d.dx);
    const int total = (r1 - r0) * C;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
        const int r = r0 + e / C, c = e % C;
        const int64_t off = (int64_t)r * C + c;
        const float g = (flags & 1) ? gamma[c] : 1.f;
        const float xh = (bf2f(x[off]) - mean[c]) * invstd[c];
        float v = g * invstd[c] * (bf2f(dy[off]) - ws[c] * invR - xh * ws[C + c] * invR);
        if (flags & 4) v += bf2f(dx[off]);
        dx[off] = f2bf(v);
    }
}

// ------------------------------------------------------------------------------------------------
// MaxPool2D valid.  Forward stores the argmax window offset (uint8); backward is a gather over the
// windows covering each input element (handles overlapping windows from explicit strides).
constexpr int POOL_ELEMS = 1024;

__global__ __launch_bounds__(256) void pool_fwd_kernel(const PoolDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const PoolDesc& d = descs[td.x];
    const int C = (int)d.C, OW = (int)d.OW, OH = (int)d.OH, W = (int)d.W, H = (int)d.H;
    const int PH = (int)d.PH, PW = (int)d.PW, SH = (int)d.SH, SW = (int)d.SW;
    const int64_t total = d.B * OH * OW * C;
    const bf16_t* x = reinterpret_cast<const bf16_t*>(d.x);
    bf16_t* y = reinterpret_cast<bf16_t*>(d.y);
    uint8_t* idx = reinterpret_cast<uint8_t*>(d.idx);
    const int64_t e0 = (int64_t)td.y * POOL_ELEMS;
    for (int64_t e = e0 + threadIdx.x; e < min(total, e0 + POOL_ELEMS); e += blockDim.x) {
        int64_t t = e;
        const int c = t % C; t /= C;
        const int ow = t % OW; t /= OW;
        const int oh = t % OH;
        const int64_t b = t / OH;
        float best = -INFINITY;
        int bi = 0;
        for (int i = 0; i < PH; ++i)
            for (int j = 0; j < PW; ++j) {
                const float v = bf2f(x[((b * H + oh * SH + i) * W + ow * SW + j) * C + c]);
                if (v > best || (v != v && best == best)) { best = v; bi = i * PW + j; }
            }
        y[e] = f2bf(best);
        idx[e] = (uint8_t)bi;
    }
}

__global__ __launch_bounds__(256) void pool_bwd_kernel(const PoolDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const PoolDesc& d = descs[td.x];
    const int C = (int)d.C, OW = (int)d.OW, OH = (int)d.OH, W = (int)d.W, H = (int)d.H;
    const int PH = (int)d.PH, PW = (int)d.PW, SH = (int)d.SH, SW = (int)d.SW;
    const int64_t total = d.B * H * W * C;
    const bf16_t* dy = reinterpret_cast<const bf16_t*>(d.dy);
    bf16_t* dx = reinterpret_cast<bf16_t*>(d.dx);
    const uint8_t* idx = reinterpret_cast<const uint8_t*>(d.idx);
    const int64_t e0 = (int64_t)td.y * POOL_ELEMS;
    for (int64_t e = e0 + threadIdx.x; e < min(total, e0 + POOL_ELEMS); e += blockDim.x) {
        int64_t t = e;
        const int c = t % C; t /= C;
        const int iw = t % W; t /= W;
        const int ih = t % H;
        const int64_t b = t / H;
        float acc = 0.f;
        const int oh_lo = max(0, (ih - PH + SH) / SH), oh_hi = min(OH - 1, ih / SH);
        const int ow_lo = max(0, (iw - PW + SW) / SW), ow_hi = min(OW - 1, iw / SW);
        for (int oh = oh_lo; oh <= oh_hi; ++oh) {
            const int i = ih - oh * SH;
            if (i < 0 || i >= PH) continue;
            for (int ow = ow_lo; ow <= ow_hi; ++ow) {
                const int j = iw - ow * SW;
                if (j < 0 || j >= PW) continue;
                const int64_t o = ((b * OH + oh) * OW + ow) * C + c;
                if (idx[o] == i * PW + j) acc += bf2f(dy[o]);
            }
        }
        if (d.flags & 1) acc += bf2f(dx[e]);
        dx[e] = f2bf(acc);
    }
}

// ------------------------------------------------------------------------------------------------
constexpr int COPY_ELEMS = 2048;

__global__ __launch_bounds__(256) void copy2d_kernel(const CopyDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const CopyDesc& d = descs[td.x];
    const int64_t total = d.rows * d.cols;
    const bf16_t* src = reinterpret_cast<const bf16_t*>(d.src);
    bf16_t* dst = reinterpret_cast<bf16_t*>(d.dst);
    const int64_t e0 = (int64_t)td.y * COPY_ELEMS;
    for (int64_t e = e0 + threadIdx.x; e < min(total, e0 + COPY_ELEMS); e += blockDim.x) {
        const int64_t r = e / d.cols, c = e - r * d.cols;
        float v = bf2f(src[r * d.src_stride + c]);
        bf16_t* o = dst + r * d.dst_stride + c;
        if (d.flags & 1) v += bf2f(*o);
        *o = f2bf(v);
    }
}

// ------------------------------------------------------------------------------------------------
// Fused heads loss: one wave per sample row.  logits fp32 [B][NC+L] (classification logits then
// replication logits), labels int [B], target bf16 [B][L].  Train: writes dlogits bf16 (d(lb*CE +
// (1-lb)*MSE)/dz, Keras mean reduction over the batch) and accumulates metrics[0]+=loss,
// metrics[1]+=correct, metrics[2]+=sum_row mean_j (sigmoid-g)^2, metrics[3]+=rows.
__global__ __launch_bounds__(256) void loss_kernel(const LossDesc* __restrict__ descs, int train, int nvalid) {
    const LossDesc& d = descs[blockIdx.y];
    const int B = (int)d.B, NC = (int)d.NC, L = (int)d.L;
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= B) return;
    const bool valid = train ? true : (row < nvalid);
    const float* z = reinterpret_cast<const float*>(d.logits) + (int64_t)row * (NC + L);
    const int label = reinterpret_cast<const int*>(d.labels)[row];
    const bf16_t* tg = reinterpret_cast<const bf16_t*>(d.target) + (int64_t)row * L;
    const float lb = (float)d.lb;
    const float invB = 1.f / (float)B;
    // --- softmax cross-entropy over NC <= 64 classes
    float zc = lane < NC ? z[lane] : -INFINITY;
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
        const float s = 1.f / (1.f + __expf(-z[NC + j]));
        const float err = s - bf2f(tg[j]);
        sq += err * err;
        if (train) {
            const float gr = (1.f - lb) * invB * 2.f * err / (float)L * s * (1.f - s);
            reinterpret_cast<bf16_t*>(d.dlogits)[(int64_t)row * (NC + L) + NC + j] = f2bf(gr);
        }
    }
    sq = warp_sum(sq);
    if (train && lane < NC) {
        const float p = ex / se;
        const float gc = lb * invB * (p - (lane == label ? 1.f : 0.f));
        reinterpret_cast<bf16_t*>(d.dlogits)[(int64_t)row * (NC + L) + lane] = f2bf(gc);
    }
    if (lane == 0 && valid) {
        float* m = reinterpret_cast<float*>(d.metrics);
        atomicAdd(&m[0], lb * ce + (1.f - lb) * sq / (float)L);
        atomicAdd(&m[1], amax == label ? 1.f : 0.f);
        atomicAdd(&m[2], sq / (float)L);
        atomicAdd(&m[3], 1.f);
    }
}

// ------------------------------------------------------------------------------------------------
// Pairwise genotype statistics over bit-packed genotypes: sum_{i<j} hamming, sum_{i<j} sqrt(hamming).
__global__ __launch_bounds__(256) void popstats_kernel(const uint64_t* __restrict__ bits, int n, int words,
                                                       double* __restrict__ out) {
    const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
    if (j0 + 63 < i0) return;
    double sh = 0.0, se = 0.0;
    for (int p = threadIdx.x; p < 64 * 64; p += blockDim.x) {
        const int i = i0 + p / 64, j = j0 + p % 64;
        if (i >= n || j >= n || j <= i) continue;
        int dsum = 0;
        for (int w = 0; w < words; ++w) dsum += __popcll(bits[(int64_t)i * words + w] ^ bits[(int64_t)j * words + w]);
        sh += dsum;
        se += sqrt((double)dsum);
    }
    // wave reduce then one atomic per wave
    for (int o = 32; o > 0; o >>= 1) {
        sh += __shfl_xor(sh, o, 64);
        se += __shfl_xor(se, o, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&out[0], sh);
        atomicAdd(&out[1], se);
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

void launch_act_bwd(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(act_bwd_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const ActBwdDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}

void launch_bn(int phase, uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(bn_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const BnDesc>(descs), as_ptr<const int2>(tiles), phase);
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
    dim3 grid((unsigned)((B + 3) / 4), (unsigned)nprob);
    hipLaunchKernelGGL(loss_kernel, grid, dim3(256), 0, as_stream(stream), as_ptr<const LossDesc>(descs), train,
                       (int)nvalid);
    SERANN_CHECK(hipGetLastError());
}

void launch_popstats(uint64_t bits, int64_t n, int64_t words, uint64_t partials, uint64_t stream) {
    if (n < 2) return;
    const unsigned t = (unsigned)((n + 63) / 64);
    hipLaunchKernelGGL(popstats_kernel, dim3(t, t), dim3(256), 0, as_stream(stream), as_ptr<const uint64_t>(bits),
                       (int)n, (int)words, as_ptr<double>(partials));
    SERANN_CHECK(hipGetLastError());
}
