// RiboAE training-path kernels.
//
// K36 (model.py:70-86, 95): binary-concrete sampling + softmax + KL(q || prior), fused.  Per genotype
// locus (b, g) over the alphabet a:
//   u        = Philox4x32-10(seed, counter = (row, a/4, offset)) -> (0,1)   (or a caller-supplied u)
//   s[a]     = logits[a]/t - (1/t) log(-log u[a])                 Gumbel(logits/t, 1/t) sample
//   logq[a]  = -(zq + e^-zq) + log t,  zq = -log(-log u[a])        posterior log-density
//   logp[a]  = -(zp + e^-zp) + log tp, zp = (s[a] - log(1/A)/tp) tp prior Gumbel(log(1/A)/tp, 1/tp)
//   z[a]     = softmax_a(s),   kl[b] = sum_{g,a} logq - logp (one block per b, fixed-order sum)
// (precise logf/expf: -log(-log u) for u near 1 needs log u accurate to relative, not absolute, error)
// backward (the reparameterised path; logq does not depend on the logits since s - loc = -log(-log u)/t):
//   dlogits[a] = (1/t) ( z[a] (gz[a] - sum_k z[k] gz[k]) + gkl[b] tp (1 - e^-zp[a]) )
//
// K37: fused log-softmax + target gather + per-sequence sum.
//
//   forward : out[b] = sum_l ( z[b,l,x[b,l]] - logsumexp_v z[b,l,v] )        (model.py:54-59, 45-46)
//   backward: dz[b,l,v] = g[b] * ( [v == x[b,l]] - softmax_v(z[b,l,:])[v] )
// z is the generative net's BatchNormalization output [B][L][V] (fp32, V = vocabulary, ~40), x the
// target tokens [B][L] (int64).  One block per sequence b: each lane owns positions l = lane, lane + 256,
// ... and walks their V logits (two passes: max, then sum-exp and the target logit); the per-sequence sum
// is a fixed-order block reduction (wave sums, then the 4 waves in order) and a plain store -- no atomics,
// so the loss is bitwise reproducible.  The log-probability tensor [B][L][V] is never materialised.

#include "common.h"
#include "serann_hip.h"

// Fixed-order sum of one value per thread over a 256-thread block; thread 0 returns the total.
__device__ __forceinline__ float block_sum256(float v, float* red) {
    v = warp_sum(v);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return threadIdx.x == 0 ? ((red[0] + red[1]) + red[2]) + red[3] : 0.f;
}

// Element access of the K37 kernels: z fp32 or bf16 (the generative BatchNormalization's own output, read in place
// by the HIP trainer), targets int64 or int32, dz fp32 or bf16 (the bf16 gradient buffer the next BN backward reads)
template <typename T> __device__ __forceinline__ float ld_f(const T* p, int64_t i);
template <> __device__ __forceinline__ float ld_f<float>(const float* p, int64_t i) { return p[i]; }
template <> __device__ __forceinline__ float ld_f<bf16_t>(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
__device__ __forceinline__ void st_f(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st_f(bf16_t* p, int64_t i, float v) { p[i] = f2bf(v); }

template <typename ZT, typename XT>
__global__ __launch_bounds__(256) void cat_loglik_fwd_kernel(const ZT* __restrict__ z, const XT* __restrict__ x,
                                                             float* __restrict__ out, int B, int L, int V) {
    __shared__ float red[4];
    const int b = blockIdx.x;
    float v = 0.f;
    for (int l = threadIdx.x; l < L; l += 256) {
        const int64_t row = ((int64_t)b * L + l) * V;
        float m = -INFINITY;
        for (int k = 0; k < V; ++k) m = fmaxf(m, ld_f(z, row + k));
        float s = 0.f;
        for (int k = 0; k < V; ++k) s += __expf(ld_f(z, row + k) - m);
        int t = (int)x[(int64_t)b * L + l];
        t = min(max(t, 0), V - 1);
        v += ld_f(z, row + t) - m - __logf(s);
    }
    v = block_sum256(v, red);
    if (threadIdx.x == 0) out[b] = v;
}

template <typename ZT, typename XT, typename DT>
__global__ __launch_bounds__(256) void cat_loglik_bwd_kernel(const ZT* __restrict__ z, const XT* __restrict__ x,
                                                             const float* __restrict__ gout, DT* __restrict__ dz,
                                                             int B, int L, int V) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)B * L) return;
    const int b = (int)(gid / L);
    const int64_t row = gid * V;
    float m = -INFINITY;
    for (int k = 0; k < V; ++k) m = fmaxf(m, ld_f(z, row + k));
    float s = 0.f;
    for (int k = 0; k < V; ++k) s += __expf(ld_f(z, row + k) - m);
    const float inv = 1.f / s, g = gout[b];
    int t = (int)x[gid];
    t = min(max(t, 0), V - 1);
    for (int k = 0; k < V; ++k) st_f(dz, row + k, g * ((k == t ? 1.f : 0.f) - __expf(ld_f(z, row + k) - m) * inv));
}

// One-hot rows of the target tokens (the embedding WGRAD's A operand), bf16 [rows][V]: written by a kernel from the
// int32 tokens instead of a host-side int64 one_hot + cast (57 MB of int64 per RiboAE step at B = 512)
__global__ __launch_bounds__(256) void onehot_kernel(const int* __restrict__ tok, bf16_t* __restrict__ out, int64_t rows,
                                                     int V) {
    const int64_t total = rows * V;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = i / V;
        const int v = (int)(i - r * V);
        out[i] = v == min(max(tok[r], 0), V - 1) ? (bf16_t)0x3f80 : (bf16_t)0;
    }
}

// ---- K36 -------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1;
        c[1] = (uint32_t)p1;
        c[3] = (uint32_t)p0;
        c[0] = n0;
        c[2] = n2;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}

constexpr int CONCRETE_MAX_A = 16;

__global__ __launch_bounds__(256) void concrete_fwd_kernel(const float* __restrict__ logits, const float* __restrict__ u_in,
                                                           float* __restrict__ s_out, float* __restrict__ z_out,
                                                           bf16_t* __restrict__ zb_out,
                                                           float* __restrict__ kl, int B, int G, int A, float t, float tp,
                                                           uint32_t k0, uint32_t k1, uint32_t off) {
    __shared__ float red[4];
    const int b = blockIdx.x;                    // one block per sequence; loci g = thread, thread + 256, ...
    float klv = 0.f;
    for (int g = threadIdx.x; g < G; g += 256) {
        const int64_t row = (int64_t)b * G + g;
        const float inv_t = 1.f / t, ploc = logf(1.f / (float)A) / tp, log_t = logf(t), log_tp = logf(tp);
        float s[CONCRETE_MAX_A];
        uint32_t c[4];
        float m = -INFINITY;
        for (int a = 0; a < A; ++a) {
            float u;
            if (u_in) {
                u = u_in[row * A + a];
            } else {
                if ((a & 3) == 0) {
                    c[0] = (uint32_t)row;
                    c[1] = (uint32_t)(row >> 32) ^ ((uint32_t)a << 24);
                    c[2] = off;
                    c[3] = 0x5EA7A11Eu;
                    philox4x32_10(c, k0, k1);
                }
                u = ((float)(c[a & 3] >> 8) + 0.5f) * (1.f / 16777216.f);
            }
            u = fminf(fmaxf(u, 1e-20f), 1.f - 1e-7f);
            const float zq = -logf(-logf(u));
            const float sa = logits[row * A + a] * inv_t + zq * inv_t;
            const float zp = (sa - ploc) * tp;
            klv += (-(zq + expf(-zq)) + log_t) - (-(zp + expf(-zp)) + log_tp);
            s[a] = sa;
            m = fmaxf(m, sa);
        }
        float den = 0.f;
        for (int a = 0; a < A; ++a) den += expf(s[a] - m);
        const float inv = 1.f / den;
        for (int a = 0; a < A; ++a) {
            s_out[row * A + a] = s[a];
            const float za = expf(s[a] - m) * inv;
            z_out[row * A + a] = za;
            if (zb_out) zb_out[row * A + a] = f2bf(za);     // the decoder's bf16 input
        }
    }
    klv = block_sum256(klv, red);
    if (threadIdx.x == 0) kl[b] = klv;           // fixed-order block sum: no atomics (deterministic)
}

template <typename GT, typename DT>
__global__ __launch_bounds__(256) void concrete_bwd_kernel(const float* __restrict__ s_in, const float* __restrict__ z_in,
                                                           const GT* __restrict__ gz, const float* __restrict__ gkl,
                                                           DT* __restrict__ dlogits, int B, int G, int A, float t,
                                                           float tp) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= (int64_t)B * G) return;
    const int b = (int)(row / G);
    const float ploc = logf(1.f / (float)A) / tp, inv_t = 1.f / t;
    const float gk = gkl ? gkl[b] : 0.f;
    float dot = 0.f;
    if (gz)
        for (int a = 0; a < A; ++a) dot += z_in[row * A + a] * ld_f(gz, row * A + a);
    for (int a = 0; a < A; ++a) {
        const float za = z_in[row * A + a];
        const float ds = gz ? za * (ld_f(gz, row * A + a) - dot) : 0.f;
        const float zp = (s_in[row * A + a] - ploc) * tp;
        st_f(dlogits, row * A + a, inv_t * (ds + gk * tp * (1.f - expf(-zp))));
    }
}

void launch_concrete_fwd(uint64_t logits, uint64_t u, uint64_t s, uint64_t z, uint64_t kl, int64_t B, int64_t G,
                         int64_t A, double t, double tp, uint64_t seed, uint64_t offset, uint64_t stream, uint64_t zb) {
    if (B <= 0 || G <= 0) return;
    if (A < 1 || A > CONCRETE_MAX_A) throw std::runtime_error("concrete: alphabet size must be in [1, 16]");
    hipLaunchKernelGGL(concrete_fwd_kernel, dim3((unsigned)B), dim3(256), 0, as_stream(stream),
                       as_ptr<const float>(logits), as_ptr<const float>(u), as_ptr<float>(s), as_ptr<float>(z),
                       as_ptr<bf16_t>(zb), as_ptr<float>(kl), (int)B, (int)G, (int)A, (float)t, (float)tp, (uint32_t)seed,
                       (uint32_t)(seed >> 32), (uint32_t)offset);
    SERANN_CHECK(hipGetLastError());
}

// bf16: 1 = gz is bf16 and dlogits is written as bf16 (the HIP trainer's buffers), 0 = both fp32
void launch_concrete_bwd(uint64_t s, uint64_t z, uint64_t gz, uint64_t gkl, uint64_t dlogits, int64_t B, int64_t G,
                         int64_t A, double t, double tp, uint64_t stream, int bf16) {
    if (B <= 0 || G <= 0) return;
    const dim3 grid((unsigned)((B * G + 255) / 256));
    if (bf16)
        hipLaunchKernelGGL((concrete_bwd_kernel<bf16_t, bf16_t>), grid, dim3(256), 0, as_stream(stream),
                           as_ptr<const float>(s), as_ptr<const float>(z), as_ptr<const bf16_t>(gz),
                           as_ptr<const float>(gkl), as_ptr<bf16_t>(dlogits), (int)B, (int)G, (int)A, (float)t, (float)tp);
    else
        hipLaunchKernelGGL((concrete_bwd_kernel<float, float>), grid, dim3(256), 0, as_stream(stream),
                           as_ptr<const float>(s), as_ptr<const float>(z), as_ptr<const float>(gz),
                           as_ptr<const float>(gkl), as_ptr<float>(dlogits), (int)B, (int)G, (int)A, (float)t, (float)tp);
    SERANN_CHECK(hipGetLastError());
}

// ---- K37 -------------------------------------------------------------------------------------------
// bf16: 1 = z bf16, x int32, dz bf16 (the HIP trainer); 0 = z fp32, x int64, dz fp32 (riboae_ops autograd)
void launch_cat_loglik_fwd(uint64_t z, uint64_t x, uint64_t out, int64_t B, int64_t L, int64_t V, uint64_t stream,
                           int bf16) {
    if (B <= 0 || L <= 0) return;
    if (bf16)
        hipLaunchKernelGGL((cat_loglik_fwd_kernel<bf16_t, int>), dim3((unsigned)B), dim3(256), 0, as_stream(stream),
                           as_ptr<const bf16_t>(z), as_ptr<const int>(x), as_ptr<float>(out), (int)B, (int)L, (int)V);
    else
        hipLaunchKernelGGL((cat_loglik_fwd_kernel<float, int64_t>), dim3((unsigned)B), dim3(256), 0, as_stream(stream),
                           as_ptr<const float>(z), as_ptr<const int64_t>(x), as_ptr<float>(out), (int)B, (int)L, (int)V);
    SERANN_CHECK(hipGetLastError());
}

void launch_cat_loglik_bwd(uint64_t z, uint64_t x, uint64_t gout, uint64_t dz, int64_t B, int64_t L, int64_t V,
                           uint64_t stream, int bf16) {
    if (B <= 0 || L <= 0) return;
    const dim3 grid((unsigned)((B * L + 255) / 256));
    if (bf16)
        hipLaunchKernelGGL((cat_loglik_bwd_kernel<bf16_t, int, bf16_t>), grid, dim3(256), 0, as_stream(stream),
                           as_ptr<const bf16_t>(z), as_ptr<const int>(x), as_ptr<const float>(gout), as_ptr<bf16_t>(dz),
                           (int)B, (int)L, (int)V);
    else
        hipLaunchKernelGGL((cat_loglik_bwd_kernel<float, int64_t, float>), grid, dim3(256), 0, as_stream(stream),
                           as_ptr<const float>(z), as_ptr<const int64_t>(x), as_ptr<const float>(gout), as_ptr<float>(dz),
                           (int)B, (int)L, (int)V);
    SERANN_CHECK(hipGetLastError());
}

void launch_onehot(uint64_t tok, uint64_t out, int64_t rows, int64_t V, uint64_t stream) {
    if (rows <= 0) return;
    int64_t blocks = (rows * V + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(onehot_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), as_ptr<const int>(tok),
                       as_ptr<bf16_t>(out), rows, (int)V);
    SERANN_CHECK(hipGetLastError());
}
