// Probe: what does a ds_read return past the end of the workgroup's LDS
// allocation on gfx950?  (The correction kernel's zero-sentinel lookups rely
// on it.)  Prints the values read at offsets past 160 KiB.
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ __launch_bounds__(256) void probe(unsigned *out)
{
    __shared__ unsigned char lds[163840];
    for (int i = threadIdx.x; i < 163840; i += 256)
        lds[i] = 0xA5;
    __syncthreads();
    const unsigned offs[8] = {163836u, 163840u, 163844u, 163840u + 4096u, 196608u, 229376u, 262140u, 300000u};
    if (threadIdx.x < 8) {
        volatile unsigned char *p = lds;
        unsigned o = offs[threadIdx.x];
        unsigned v = p[o];
        unsigned w = 0;
        asm volatile("ds_read_u8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(w) : "v"(o));
        out[threadIdx.x * 2] = v;
        out[threadIdx.x * 2 + 1] = w;
    }
}

int main()
{
    unsigned *d, h[16];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess)
        return 2;
    hipLaunchKernelGGL(probe, dim3(1), dim3(256), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess)
        return 3;
    const char *names[8] = {"163836 (last dword, in range)", "163840", "163844", "167936", "196608", "229376", "262140", "300000"};
    for (int i = 0; i < 8; i++)
        printf("offset %-30s C-read 0x%02x  asm-read 0x%02x\n", names[i], h[2 * i], h[2 * i + 1]);
    return 0;
}
