// RiboAE training-path kernels: fused log-softmax + target gather + per-sequence sum.
//
//   forward : out[b] = sum_l ( z[b,l,x[b,l]] - logsumexp_v z[b,l,v] )        (model.py:54-59, 45-46)
//   backward: dz[b,l,v] = g[b] * ( [v == x[b,l]] - softmax_v(z[b,l,:])[v] )
// z is the generative net's BatchNormalization output [B][L][V] (fp32, V = vocabulary, ~40), x the
// target tokens [B][L] (int64).  One wave per (b, l-block of 64 positions): each lane owns one position
// and walks its V logits (two passes: max, then sum-exp and the target logit); the per-sequence sum is
// a wave reduction + one atomic per wave.  The log-probability tensor [B][L][V] is never materialised.
#include "common.h"
#include "serann_hip.h"

__global__ __launch_bounds__(256) void cat_loglik_fwd_kernel(const float* __restrict__ z, const int64_t* __restrict__ x,
                                                             float* __restrict__ out, int B, int L, int V) {
    const int lanes_per_b = ((L + 63) / 64) * 64;
    const int64_t gid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int b = (int)(gid / lanes_per_b);
    const int l = (int)(gid - (int64_t)b * lanes_per_b);
    float v = 0.f;
    if (b < B && l < L) {
        const float* row = z + ((int64_t)b * L + l) * V;
        float m = -INFINITY;
        for (int k = 0; k < V; ++k) m = fmaxf(m, row[k]);
        float s = 0.f;
        for (int k = 0; k < V; ++k) s += __expf(row[k] - m);
        int t = (int)x[(int64_t)b * L + l];
        t = min(max(t, 0), V - 1);
        v = row[t] - m - __logf(s);
    }
    v = warp_sum(v);
    if ((threadIdx.x & 63) == 0 && b < B) atomicAdd(out + b, v);
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

void launch_cat_loglik_fwd(uint64_t z, uint64_t x, uint64_t out, int64_t B, int64_t L, int64_t V, uint64_t stream) {
    if (B <= 0 || L <= 0) return;
    const int64_t threads = B * (((L + 63) / 64) * 64);
    hipLaunchKernelGGL(cat_loglik_fwd_kernel, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, as_stream(stream),
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
