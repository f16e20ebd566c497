// Probe: ds_read past the end of a 64 KiB workgroup allocation on gfx950,
// with two 1024-thread workgroups per CU (the split decode kernels' shape).
// Each workgroup fills its LDS with a workgroup-specific nonzero byte; lane i
// of wave 0 reads offset offs[i]; the host reports, per offset, how many
// workgroups read 0, their own byte, or anything else.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define NOFF 16
#ifdef FINE
__constant__ unsigned offs[NOFF] = {65536u, 69632u, 73728u, 77824u, 81920u, 86016u, 90112u, 94208u,
                                    96256u, 97280u, 98300u, 98304u, 102400u, 114688u, 122880u, 131068u};
#else
__constant__ unsigned offs[NOFF] = {65532u, 65535u, 65536u, 65540u, 98304u, 131071u, 131072u, 163840u,
                                    196608u, 262144u, 300000u, 524288u, 1048576u, 1u << 24, 1u << 28, 0xFFFFFFF0u};
#endif

__global__ __launch_bounds__(1024) void probe(unsigned *out)
{
    __shared__ unsigned char lds[65536];
    const unsigned char pat = (unsigned char)((blockIdx.x % 254) + 1);
    for (int i = threadIdx.x; i < 65536; i += 1024)
        lds[i] = pat;
    __syncthreads();
    if (threadIdx.x < NOFF) {
        unsigned o = offs[threadIdx.x] + (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char *)lds;
        unsigned w = 0;
        asm volatile("ds_read_u8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(o));
        out[blockIdx.x * NOFF + threadIdx.x] = (w == 0) ? 0u : (w == pat ? 1u : 2u);
    }
    __syncthreads();
}

int main()
{
    const int nb = 2048;
    unsigned *d, *h = (unsigned *)malloc(nb * NOFF * 4);
    unsigned hoffs[NOFF];
    if (hipMalloc(&d, nb * NOFF * 4) != hipSuccess)
        return 2;
    hipLaunchKernelGGL(probe, dim3(nb), dim3(1024), 0, 0, d);
    if (hipMemcpy(h, d, nb * NOFF * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return 3;
    if (hipMemcpyFromSymbol(hoffs, HIP_SYMBOL(offs), sizeof(hoffs)) != hipSuccess)
        return 4;
    for (int i = 0; i < NOFF; i++) {
        int z = 0, own = 0, other = 0;
        for (int b = 0; b < nb; b++) {
            unsigned v = h[b * NOFF + i];
            z += v == 0;
            own += v == 1;
            other += v == 2;
        }
        printf("offset %10u (0x%08x): zero %d  own %d  other %d\n", hoffs[i], hoffs[i], z, own, other);
    }
    return 0;
}
