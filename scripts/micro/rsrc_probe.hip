// Probe: how gfx950 range-checks a partially out-of-range raw buffer_load_dwordx4.
// A 64-B buffer holds dwords 1..16; the resource covers only the first NREC bytes.  Each lane loads 16 B at
// byte offset 4 * lane (lanes 0..15) and stores the 4 dwords it got.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;

__global__ void probe(const unsigned* buf, int nrec, unsigned* out) {
    const int lane = threadIdx.x;
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, nrec, 0x00020000);
    if (lane < 16) {
        u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, lane * 4, 0, 0);
        for (int j = 0; j < 4; ++j) out[lane * 4 + j] = v[j];
    }
}

int main() {
    unsigned h[32];
    for (int i = 0; i < 32; ++i) h[i] = i + 1;
    unsigned *d, *o;
    hipMalloc(&d, sizeof(h));
    hipMalloc(&o, 64 * sizeof(unsigned));
    hipMemcpy(d, h, sizeof(h), hipMemcpyHostToDevice);
    for (int nrec : {40, 42, 48}) {
        hipMemset(o, 0xff, 64 * sizeof(unsigned));
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, nrec, o);
        unsigned r[64];
        hipMemcpy(r, o, sizeof(r), hipMemcpyDeviceToHost);
        printf("num_records=%d bytes\n", nrec);
        for (int l = 0; l < 12; ++l) printf("  byte offset %2d -> %u %u %u %u\n", 4 * l, r[4 * l], r[4 * l + 1], r[4 * l + 2], r[4 * l + 3]);
    }
    hipFree(d);
    hipFree(o);
    return 0;
}
