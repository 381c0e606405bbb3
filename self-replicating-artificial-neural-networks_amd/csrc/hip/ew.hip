// Grouped strided elementwise kernel for the interpreter's rare ops (mutants reach unary and
// binary minus and BatchNormalization on a non-last axis; reference common/logic.py:17-35 runs them inside
// the Keras graph).  One descriptor form covers all of them:
//
//   out[j] (+)= sum_{r in R} ( ca * A[a(j, r)] + cb * B[b(j, r)] ) + c
//
// j runs over the dense 4-d destination D (row-major), r over the 4-d reduction box R (all ones for a pure
// map); every operand address is a stride dot-product of (j, r), so broadcasting (stride 0), permutations
// (BatchNormalization's [outer][C][inner] <-> [outer][inner][C] transposes) and reductions over broadcast
// dimensions (the gradient of a broadcast operand of `sub`) need no special cases.
//   neg         : ca = -1
//   sub (t - t) : ca = 1, cb = -1, B broadcast by zero strides
//   sub (t - c) : ca = 1, c = -k;  (c - t): ca = -1, c = k
//   backward    : dA = sum over A's broadcast dimensions of ca * dOut (R = those dimensions)
// Each thread owns whole destination elements and walks its reduction in a fixed order: no atomics, so the
// result is bitwise reproducible.  bf16 in / out, fp32 arithmetic.
#include "common.h"
#include "serann_hip.h"

namespace {

__device__ __forceinline__ void unravel4(int64_t j, const int64_t (&D)[4], int64_t (&q)[4]) {
    q[3] = j % D[3];
    j /= D[3];
    q[2] = j % D[2];
    j /= D[2];
    q[1] = j % D[1];
    q[0] = j / D[1];
}

}  // namespace

__global__ __launch_bounds__(256) void ew_kernel(const EwDesc* __restrict__ descs, const int2* __restrict__ tiles) {
    const int2 td = tiles[blockIdx.x];
    const EwDesc& d = descs[td.x];
    const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(d.a);
    const bf16_t* __restrict__ Bv = reinterpret_cast<const bf16_t*>(d.b);
    bf16_t* __restrict__ out = reinterpret_cast<bf16_t*>(d.out);
    const int64_t D[4] = {d.D[0], d.D[1], d.D[2], d.D[3]};
    const int64_t R[4] = {d.R[0], d.R[1], d.R[2], d.R[3]};
    const int64_t n = D[0] * D[1] * D[2] * D[3];
    const int64_t j0 = (int64_t)td.y * EW_ELEMS;
    const int64_t j1 = min(n, j0 + (int64_t)EW_ELEMS);
    const bool acc = d.flags & 1;
    for (int64_t j = j0 + threadIdx.x; j < j1; j += blockDim.x) {
        int64_t q[4];
        unravel4(j, D, q);
        int64_t ab = 0, bb = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ab += q[k] * d.aJ[k];
            bb += q[k] * d.bJ[k];
        }
        float s = 0.f;
        for (int64_t r0 = 0; r0 < R[0]; ++r0)
            for (int64_t r1 = 0; r1 < R[1]; ++r1)
                for (int64_t r2 = 0; r2 < R[2]; ++r2)
                    for (int64_t r3 = 0; r3 < R[3]; ++r3) {
                        const int64_t ao = ab + r0 * d.aR[0] + r1 * d.aR[1] + r2 * d.aR[2] + r3 * d.aR[3];
                        float v = d.ca * bf2f(A[ao]);
                        if (Bv) {
                            const int64_t bo = bb + r0 * d.bR[0] + r1 * d.bR[1] + r2 * d.bR[2] + r3 * d.bR[3];
                            v += d.cb * bf2f(Bv[bo]);
                        }
                        s += v;
                    }
        s += d.c;
        if (acc) s += bf2f(out[j]);
        out[j] = f2bf(s);
    }
}

void launch_ew(uint64_t descs, uint64_t tiles, int64_t ntiles, uint64_t stream) {
    if (ntiles <= 0) return;
    hipLaunchKernelGGL(ew_kernel, dim3((unsigned)ntiles), dim3(256), 0, as_stream(stream),
                       as_ptr<const EwDesc>(descs), as_ptr<const int2>(tiles));
    SERANN_CHECK(hipGetLastError());
}
