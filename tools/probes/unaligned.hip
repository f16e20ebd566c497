// Probe: 16-byte loads and stores at any byte offset from global memory
// (one global_load_dwordx4 / global_store_dwordx4 under the unaligned access
// mode), checked against byte copies.  Build: hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

struct __attribute__((packed, aligned(1))) U16 { uint32_t a, b, c, d; };
typedef __attribute__((address_space(1))) U16 gU16;

__global__ void probe(const uint8_t *in, uint8_t *out, uint8_t *out2)
{
    const uint32_t t = threadIdx.x;            // offset t
    const gU16 *src = (const gU16 *)(uintptr_t)(in + t);
    U16 v;
    v.a = src->a, v.b = src->b, v.c = src->c, v.d = src->d;
    *reinterpret_cast<U16 *>(out + t * 16) = v;  // aligned store of what was read
    U16 w; w.a = v.a; w.b = v.b; w.c = v.c; w.d = v.d;
    gU16 *dst = (gU16 *)(uintptr_t)(out2 + 1 + t * 17); // unaligned store
    dst->a = w.a, dst->b = w.b, dst->c = w.c, dst->d = w.d;
}

int main()
{
    uint8_t h[4096], o[4096], o2[8192];
    for (int i = 0; i < 4096; i++) h[i] = (uint8_t)(i * 7 + 3);
    uint8_t *din, *dout, *dout2;
    hipMalloc(&din, 4096); hipMalloc(&dout, 4096); hipMalloc(&dout2, 8192);
    hipMemcpy(din, h, 4096, hipMemcpyHostToDevice);
    hipMemset(dout2, 0, 8192);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, din, dout, dout2);
    hipMemcpy(o, dout, 4096, hipMemcpyDeviceToHost);
    hipMemcpy(o2, dout2, 8192, hipMemcpyDeviceToHost);
    int bad = 0, bad2 = 0;
    for (int t = 0; t < 64; t++)
        for (int k = 0; k < 16; k++) {
            bad += o[t * 16 + k] != h[t + k];
            bad2 += o2[1 + t * 17 + k] != h[t + k];
        }
    printf("unaligned dwordx4 probe: load mismatches %d, store mismatches %d\n", bad, bad2);
    return bad || bad2;
}
