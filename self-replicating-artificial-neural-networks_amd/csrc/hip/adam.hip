// Fused multi-tensor Keras-Adam over a flat fp32 parameter arena (K13 / K38).  The gradients arrive in
// the deterministic Q40 fixed-point arena (common.h fx_*: int64, 2^-40 units) and are converted here.
//
// TF ResourceApplyAdam semantics (experiment_worker.py:80): lr_t = lr*sqrt(1-b2^t)/(1-b1^t),
// m = b1 m + (1-b1) g, v = b2 v + (1-b2) g^2, p -= lr_t m / (sqrt(v) + eps).
// One launch per training step for the whole population shard; the step counter and lr_t live in
// device memory so the launch can be captured once in a hipGraph and replayed every step.  The
// kernel also refreshes the bf16 compute copy of the weights and zeroes the gradient arena for the
// next step's atomic accumulation.  Pure HBM streaming: 3x float4 + 2x int64x2 in, the same + bf16 out.
#include "common.h"
#include "serann_hip.h"

__global__ void adam_scalars_kernel(int* step, float* lr_t, float lr, float b1, float b2) {
    int t = *step + 1;
    *step = t;
    *lr_t = lr * sqrtf(1.f - powf(b2, (float)t)) / (1.f - powf(b1, (float)t));
}

// skip (optional): one byte per 4-parameter group, bit j set = parameter 4i + j was already updated by its
// WGRAD epilogue (GF_ADAM) this step; fully skipped groups are not even read.  MM: moment storage (common.h).
template <int MM>
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ p, long long* __restrict__ g,
                                                   void* __restrict__ m, void* __restrict__ v,
                                                   bf16_t* __restrict__ pbf, const float* __restrict__ lr_t_ptr,
                                                   int64_t n, float b1, float b2, float eps,
                                                   const uint8_t* __restrict__ skip, const int64_t* __restrict__ org_off,
                                                   int* __restrict__ diverged, int norg) {
    const float lr_t = *lr_t_ptr;
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        const unsigned sk = skip ? skip[i] : 0u;
        if (sk == 0xfu) continue;
        float4 pv = reinterpret_cast<float4*>(p)[i];
        const longlong2 g01 = reinterpret_cast<longlong2*>(g)[2 * i];
        const longlong2 g23 = reinterpret_cast<longlong2*>(g)[2 * i + 1];
        float4 gv = make_float4(fx_f(g01.x), fx_f(g01.y), fx_f(g23.x), fx_f(g23.y));
        if (org_off && fmaxf(fmaxf(fabsf(gv.x), fabsf(gv.y)), fmaxf(fabsf(gv.z), fabsf(gv.w))) > FX_DIVERGE)
            flag_diverged(org_off, diverged, norg, 4 * i);
        float4 mv = m_ld4<MM>(m, 4 * i);
        float4 vv = v_ld4<MM>(v, 4 * i);
        float* pp = &pv.x; float* gg = &gv.x; float* mm = &mv.x; float* vvv = &vv.x;
        ushort4 ob = reinterpret_cast<ushort4*>(pbf)[i];
        uint16_t* o = &ob.x;
        if (sk == 0u) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                adam_elem(pp[k], mm[k], vvv[k], gg[k], lr_t, b1, b2, eps);
                o[k] = f2bf(pp[k]);
            }
            reinterpret_cast<float4*>(p)[i] = pv;
            m_st4<MM>(m, 4 * i, mv);
            v_st4<MM>(v, 4 * i, vv);
            reinterpret_cast<longlong2*>(g)[2 * i] = make_longlong2(0, 0);
            reinterpret_cast<longlong2*>(g)[2 * i + 1] = make_longlong2(0, 0);
            reinterpret_cast<ushort4*>(pbf)[i] = ob;
        } else {
            // a group straddling a fused tile's edge: element by element
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                if (sk & (1u << k)) continue;
                const int64_t e = 4 * i + k;
                adam_elem(pp[k], mm[k], vvv[k], gg[k], lr_t, b1, b2, eps);
                p[e] = pp[k]; m_st<MM>(m, e, mm[k]); v_st<MM>(v, e, vvv[k]); g[e] = 0; pbf[e] = f2bf(pp[k]);
            }
        }
    }
    // tail
    for (int64_t i = n4 * 4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        if (skip && ((skip[i >> 2] >> (i & 3)) & 1u)) continue;
        float pp = p[i], mm = m_ld<MM>(m, i), vv = v_ld<MM>(v, i);
        if (org_off && fabsf(fx_f(g[i])) > FX_DIVERGE) flag_diverged(org_off, diverged, norg, i);
        adam_elem(pp, mm, vv, fx_f(g[i]), lr_t, b1, b2, eps);
        m_st<MM>(m, i, mm); v_st<MM>(v, i, vv); p[i] = pp; g[i] = 0; pbf[i] = f2bf(pp);
    }
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) y[i] = f2bf(x[i]);
}

void launch_adam_scalars(uint64_t step, uint64_t lr_t, float lr, float b1, float b2, uint64_t stream) {
    hipLaunchKernelGGL(adam_scalars_kernel, dim3(1), dim3(1), 0, as_stream(stream), as_ptr<int>(step),
                       as_ptr<float>(lr_t), lr, b1, b2);
}

void launch_adam_update(uint64_t p, uint64_t g, uint64_t m, uint64_t v, uint64_t pbf, uint64_t lr_t, int64_t n,
                        float b1, float b2, float eps, uint64_t skip, uint64_t stream, int mode, uint64_t org_off,
                        uint64_t diverged, int64_t norg) {
    if (n <= 0) return;
    if (mode != MOM_F32 && mode != MOM_16) throw std::runtime_error("adam_update: unknown moment mode");
    int64_t blocks = ((n >> 2) + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    auto kern = mode == MOM_16 ? adam_kernel<MOM_16> : adam_kernel<MOM_F32>;
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream), as_ptr<float>(p),
                       as_ptr<long long>(g), as_ptr<void>(m), as_ptr<void>(v), as_ptr<bf16_t>(pbf),
                       as_ptr<const float>(lr_t), n, b1, b2, eps, as_ptr<const uint8_t>(skip),
                       as_ptr<const int64_t>(norg > 0 ? org_off : 0), as_ptr<int>(diverged), (int)norg);
    SERANN_CHECK(hipGetLastError());
}

void launch_adam(uint64_t p, uint64_t g, uint64_t m, uint64_t v, uint64_t pbf, uint64_t step, uint64_t lr_t,
                 int64_t n, float lr, float b1, float b2, float eps, uint64_t stream, int mode) {
    launch_adam_scalars(step, lr_t, lr, b1, b2, stream);
    launch_adam_update(p, g, m, v, pbf, lr_t, n, b1, b2, eps, 0, stream, mode, 0, 0, 0);
}

void launch_f32_to_bf16(uint64_t x, uint64_t y, int64_t n, uint64_t stream) {
    if (n <= 0) return;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(f32_to_bf16_kernel, dim3((unsigned)blocks), dim3(256), 0, as_stream(stream),
                       as_ptr<const float>(x), as_ptr<bf16_t>(y), n);
    SERANN_CHECK(hipGetLastError());
}
