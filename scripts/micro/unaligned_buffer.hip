// Microtest: raw buffer_load_dwordx4 at 2-byte-aligned byte offsets on gfx950, and range checking.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
__global__ void k(const unsigned short* src, unsigned short* dst, int n, int shift, int nrec) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, nrec, 0x00020000);
    u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (i * 8 + shift) * 2, 0, 0);
    *reinterpret_cast<u32x4*>(dst + i * 8) = v;
}
int main() {
    const int n = 1 << 16;
    std::vector<unsigned short> h(n);
    for (int i = 0; i < n; ++i) h[i] = (unsigned short)(i * 7 + 3);
    unsigned short *s, *d;
    hipMalloc(&s, n * 2 + 64); hipMalloc(&d, n * 2 + 64);
    hipMemcpy(s, h.data(), n * 2, hipMemcpyHostToDevice);
    for (int shift = 0; shift < 8; ++shift) {
        hipMemset(d, 0, n * 2);
        hipLaunchKernelGGL(k, dim3(n / 8 / 256), dim3(256), 0, 0, s, d, n, shift, n * 2);
        hipError_t e = hipDeviceSynchronize();
        std::vector<unsigned short> o(n);
        hipMemcpy(o.data(), d, n * 2, hipMemcpyDeviceToHost);
        int bad = 0, first = -1;
        for (int i = 0; i + 8 + shift <= n; ++i) if (o[i] != h[i + shift]) { ++bad; if (first < 0) first = i; }
        printf("shift %d: err=%s mismatches=%d", shift, hipGetErrorString(e), bad);
        if (first >= 0) printf(" first=%d got=%u want=%u (want-1=%u want+1=%u)", first, o[first], h[first + shift], h[first+shift-1], h[first+shift+1]);
        // tail: elements beyond nrec must read as 0
        int tail_nonzero = 0;
        for (int i = n - shift; i < n; ++i) if (o[i] != 0) ++tail_nonzero;
        printf(" tail_nonzero=%d\n", tail_nonzero);
    }
    return 0;
}
