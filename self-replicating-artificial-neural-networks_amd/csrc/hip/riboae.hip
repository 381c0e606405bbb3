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

__global__ __launch_bounds__(256) void cat_loglik_fwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ x,
                                                             float* __restrict__ out, int B, int L, int V) {
    __shared__ float red[4];
    const int b = blockIdx.x;
    float v = 0.f;
    for (int l = threadIdx.x; l < L; l += 256) {
        const float* row = z + ((int64_t)b * L + l) * V;
        float m = -INFINITY;
        for (int k = 0; k < V; ++k) m = fmaxf(m, row[k]);
        float s = 0.f;
        for (int k = 0; k < V; ++k) s += __expf(row[k] - m);
        int t = (int)x[(int64_t)b * L + l];
        t = min(max(t, 0), V - 1);
        v += row[t] - m - __logf(s);
    }
    v = block_sum256(v, red);
    if (threadIdx.x == 0) out[b] = v;
}

__global__ __launch_bounds__(256) void cat_loglik_bwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ x,
                                                             const float* __restrict__ gout, float* __restrict__ dz,
                                                             int B, int L, int V) {
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (int64_t)B * L) return;
    const int b = (int)(gid / L);
    const float* row = z + gid * V;
    float* drow = dz + gid * V;
    float m = -INFINITY;
    for (int k = 0; k < V; ++k) m = fmaxf(m, row[k]);
    float s = 0.f;
    for (int k = 0; k < V; ++k) s += __expf(row[k] - m);
    const float inv = 1.f / s, g = gout[b];
    int t = (int)x[gid];
    t = min(max(t, 0), V - 1);
    for (int k = 0; k < V; ++k) drow[k] = g * ((k == t ? 1.f : 0.f) - __expf(row[k] - m) * inv);
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
            z_out[row * A + a] = expf(s[a] - m) * inv;
        }
    }
    klv = block_sum256(klv, red);
    if (threadIdx.x == 0) kl[b] = klv;           // fixed-order block sum: no atomics (deterministic)
}

__global__ __launch_bounds__(256) void concrete_bwd_kernel(const float* __restrict__ s_in, const float* __restrict__ z_in,
                                                           const float* __restrict__ gz, const float* __restrict__ gkl,
                                                           float* __restrict__ dlogits, int B, int G, int A, float t,
                                                           float tp) {
    const int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= (int64_t)B * G) return;
    const int b = (int)(row / G);
    const float ploc = logf(1.f / (float)A) / tp, inv_t = 1.f / t;
    const float gk = gkl ? gkl[b] : 0.f;
    float dot = 0.f;
    if (gz)
        for (int a = 0; a < A; ++a) dot += z_in[row * A + a] * gz[row * A + a];
    for (int a = 0; a < A; ++a) {
        const float za = z_in[row * A + a];
        const float ds = gz ? za * (gz[row * A + a] - dot) : 0.f;
        const float zp = (s_in[row * A + a] - ploc) * tp;
        dlogits[row * A + a] = inv_t * (ds + gk * tp * (1.f - expf(-zp)));
    }
}

void launch_concrete_fwd(uint64_t logits, uint64_t u, uint64_t s, uint64_t z, uint64_t kl, int64_t B, int64_t G,
                         int64_t A, double t, double tp, uint64_t seed, uint64_t offset, uint64_t stream) {
    if (B <= 0 || G <= 0) return;
    if (A < 1 || A > CONCRETE_MAX_A) throw std::runtime_error("concrete: alphabet size must be in [1, 16]");
    hipLaunchKernelGGL(concrete_fwd_kernel, dim3((unsigned)B), dim3(256), 0, as_stream(stream),
                       as_ptr<const float>(logits), as_ptr<const float>(u), as_ptr<float>(s), as_ptr<float>(z),
                       as_ptr<float>(kl), (int)B, (int)G, (int)A, (float)t, (float)tp, (uint32_t)seed,
                       (uint32_t)(seed >> 32), (uint32_t)offset);
    SERANN_CHECK(hipGetLastError());
}

void launch_concrete_bwd(uint64_t s, uint64_t z, uint64_t gz, uint64_t gkl, uint64_t dlogits, int64_t B, int64_t G,
                         int64_t A, double t, double tp, uint64_t stream) {
    if (B <= 0 || G <= 0) return;
    hipLaunchKernelGGL(concrete_bwd_kernel, dim3((unsigned)((B * G + 255) / 256)), dim3(256), 0, as_stream(stream),
                       as_ptr<const float>(s), as_ptr<const float>(z), as_ptr<const float>(gz),
                       as_ptr<const float>(gkl), as_ptr<float>(dlogits), (int)B, (int)G, (int)A, (float)t, (float)tp);
    SERANN_CHECK(hipGetLastError());
}

// ---- K37 -------------------------------------------------------------------------------------------
void launch_cat_loglik_fwd(uint64_t z, uint64_t x, uint64_t out, int64_t B, int64_t L, int64_t V, uint64_t stream) {
    if (B <= 0 || L <= 0) return;
    hipLaunchKernelGGL(cat_loglik_fwd_kernel, dim3((unsigned)B), dim3(256), 0, as_stream(stream),
                       as_ptr<const float>(z), as_ptr<const int64_t>(x), as_ptr<float>(out), (int)B, (int)L, (int)V);
    SERANN_CHECK(hipGetLastError());
}

void launch_cat_loglik_bwd(uint64_t z, uint64_t x, uint64_t gout, uint64_t dz, int64_t B, int64_t L, int64_t V,
                           uint64_t stream) {
    if (B <= 0 || L <= 0) return;
    hipLaunchKernelGGL(cat_loglik_bwd_kernel, dim3((unsigned)((B * L + 255) / 256)), dim3(256), 0, as_stream(stream),
                       as_ptr<const float>(z), as_ptr<const int64_t>(x), as_ptr<const float>(gout), as_ptr<float>(dz),
                       (int)B, (int)L, (int)V);
    SERANN_CHECK(hipGetLastError());
}
