// Probe: do gfx950's VOP2 16-bit ops (v_add_u16, v_sub_u16, v_min_u16) zero
// the upper half of their destination?  Sources carry garbage in bits 31:16.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k(uint32_t *out)
{
    const uint32_t t = threadIdx.x;
    uint32_t a = 0xABCD0000u | (100u + t), b = 0x12340000u | 7u, r0, r1, r2;
    asm volatile("v_add_u16 %0, %1, %2" : "=v"(r0) : "v"(a), "v"(b));
    asm volatile("v_sub_u16 %0, %1, %2" : "=v"(r1) : "v"(a), "v"(b));
    asm volatile("v_min_u16 %0, %1, %2" : "=v"(r2) : "v"(a), "v"(b));
    // destination preloaded with garbage, written by a 16-bit op
    uint32_t r3 = 0x55550000u | t;
    asm volatile("v_add_u16 %0, %1, %2" : "+v"(r3) : "v"(a), "v"(b));
    if (t == 0) {
        out[0] = r0;
        out[1] = r1;
        out[2] = r2;
        out[3] = r3;
    }
}

int main()
{
    uint32_t *d, h[4];
    if (hipMalloc(&d, 16) != hipSuccess)
        return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, 16, hipMemcpyDeviceToHost) != hipSuccess)
        return 1;
    printf("add %08x sub %08x min %08x add(dst preloaded) %08x\n", h[0], h[1], h[2], h[3]);
    printf("upper half zeroed: %s\n", ((h[0] | h[1] | h[2] | h[3]) >> 16) ? "no" : "yes");
    return 0;
}
