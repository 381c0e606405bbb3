// Microtest: are 16-byte global loads at 2-byte-aligned addresses handled correctly on gfx950?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
__global__ void k(const unsigned short* src, unsigned short* dst, int n, int shift) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i * 8 + 8 + shift <= n) {
        uint4 v = *reinterpret_cast<const uint4*>(src + i * 8 + shift);
        *reinterpret_cast<uint4*>(dst + i * 8) = v;
    }
}
int main() {
    const int n = 1 << 16;
    std::vector<unsigned short> h(n);
    for (int i = 0; i < n; ++i) h[i] = (unsigned short)(i * 7 + 3);
    unsigned short *s, *d;
    hipMalloc(&s, n * 2); hipMalloc(&d, n * 2);
    hipMemcpy(s, h.data(), n * 2, hipMemcpyHostToDevice);
    int bad_total = 0;
    for (int shift = 0; shift < 8; ++shift) {
        hipMemset(d, 0, n * 2);
        hipLaunchKernelGGL(k, dim3(n / 8 / 256), dim3(256), 0, 0, s, d, n, shift);
        hipError_t e = hipDeviceSynchronize();
        std::vector<unsigned short> o(n);
        hipMemcpy(o.data(), d, n * 2, hipMemcpyDeviceToHost);
        int bad = 0;
        for (int i = 0; i + 8 + shift <= n; ++i) if (o[i] != h[i + shift]) ++bad;
        printf("shift %d: err=%s mismatches=%d\n", shift, hipGetErrorString(e), bad);
        bad_total += bad;
    }
    printf(bad_total == 0 ? "UNALIGNED_OK\n" : "UNALIGNED_BAD\n");
    return 0;
}
