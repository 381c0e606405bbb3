// Microbenchmark: streaming read bandwidth of 16-B buffer loads whose byte offsets follow a [rows][F] bf16
// tensor's row starts (F = 64 aligned vs F = 69 / 75: every row start 2-B aligned), 8 chunks of 8 elements
// per row as the WGRAD A loader issues them, plus a flat aligned read of the same bytes.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
__global__ void rows_kernel(const unsigned short* src, unsigned* out, int rows, int F, long long nrec) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)src, (short)0, (int)nrec, 0x00020000);
    const int chunks = (F + 7) / 8;
    unsigned acc = 0;
    const long long total = (long long)rows * chunks;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
        const long long row = i / chunks, c = i - row * chunks;
        u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)((row * F + c * 8) * 2), 0, 0);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
__global__ void flat_kernel(const unsigned short* src, unsigned* out, long long n8) {
    unsigned acc = 0;
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n8; i += (long long)gridDim.x * blockDim.x) {
        u32x4 v = reinterpret_cast<const u32x4*>(src)[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}
int main() {
    const int rows = 1 << 20;
    unsigned short* s; unsigned* o;
    hipMalloc(&s, (size_t)rows * 80 * 2 + 64); hipMalloc(&o, 64);
    hipMemset(s, 1, (size_t)rows * 80 * 2);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    int Fs[] = {64, 69, 75, 16, 9};
    for (int F : Fs) {
        float best = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(rows_kernel, dim3(4096), dim3(256), 0, 0, s, o, rows, F, (long long)rows * F * 2);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        const double bytes = (double)rows * F * 2;
        float bf = 1e9;
        for (int rep = 0; rep < 5; ++rep) {
            hipEventRecord(a);
            hipLaunchKernelGGL(flat_kernel, dim3(4096), dim3(256), 0, 0, s, o, (long long)rows * F / 8);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < bf) bf = ms;
        }
        printf("F=%3d rows-pattern %.3f ms %.2f TB/s | flat aligned %.3f ms %.2f TB/s\n", F, best, bytes / best / 1e9,
               bf, bytes / bf / 1e9);
    }
    return 0;
}
