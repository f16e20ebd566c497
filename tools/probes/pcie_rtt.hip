/*
 * pcie_rtt.hip -- diagnostic probe (not part of the product): the latencies
 * the single-call server (rs_serve_k) is made of, on this box.
 *
 *   1. GPU-side: dependent system-scope loads of a word in coherent host
 *      memory (the server's poll), in s_memrealtime ticks (10 ns).
 *   2. Ping-pong: the host writes a sequence number into coherent host
 *      memory, one GPU lane polls it (system-scope loads) and writes it back
 *      to another word, the host polls that -- the floor of a server call
 *      without any work (reported per round trip, host clock).
 *   3. The same ping-pong with the poll word and the answer in device memory
 *      visible to the host (hipExtMallocWithFlags fine-grained), if the host
 *      can map it.
 *
 * Build: hipcc --offload-arch=gfx950 -O2 -o tools/probes/pcie_rtt tools/probes/pcie_rtt.hip
 * Every GPU loop is bounded (a lifetime in ticks), so no run can hang.
 */
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdint>

__global__ void rtt_k(uint32_t *w, uint64_t *out, int n)
{
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
    for (int i = 0; i < n; ++i)
        acc += __hip_atomic_load(w + (acc & 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint64_t t1 = __builtin_amdgcn_s_memrealtime();
    out[0] = t1 - t0;
    out[1] = acc;
}

/* polls in[0] for values 1..n, echoing each to out[0]; leaves after `life` ticks */
__global__ void pong_k(uint32_t *in, uint32_t *outw, int n, uint64_t life)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t last = 0;
    while (last < (uint32_t)n) {
        const uint32_t v = __hip_atomic_load(in, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v != last) {
            __hip_atomic_store(outw, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            last = v;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > life)
            break;
    }
}

static double pingpong(uint32_t *hin, uint32_t *hout, uint32_t *din, uint32_t *dout, int n)
{
    hipLaunchKernelGGL(pong_k, dim3(1), dim3(1), 0, 0, din, dout, n, (uint64_t)300000000ull);
    volatile uint32_t *vi = hin, *vo = hout;
    /* warm: first exchange */
    *vi = 1;
    auto t_start = std::chrono::steady_clock::now();
    while (*vo != 1) {
        if (std::chrono::steady_clock::now() - t_start > std::chrono::seconds(5))
            return -1;
    }
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 2; i <= n; ++i) {
        std::atomic_thread_fence(std::memory_order_release);
        *vi = (uint32_t)i;
        while (*vo != (uint32_t)i) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
                return -1;
        }
    }
    auto t1 = std::chrono::steady_clock::now();
    hipDeviceSynchronize();
    return std::chrono::duration<double>(t1 - t0).count() / (n - 1) * 1e6;
}

int main()
{
    uint32_t *h = nullptr;
    uint64_t *o = nullptr;
    hipHostMalloc((void **)&h, 4096, hipHostMallocCoherent);
    hipMalloc((void **)&o, 64);
    h[0] = 0;
    h[1] = 0;
    void *dh = nullptr;
    hipHostGetDevicePointer(&dh, h, 0);
    const int n = 2000;
    hipLaunchKernelGGL(rtt_k, dim3(1), dim3(1), 0, 0, (uint32_t *)dh, o, n);
    uint64_t r[2];
    hipMemcpy(r, o, 16, hipMemcpyDeviceToHost);
    printf("{\"probe\": \"gpu load of coherent host memory\", \"ns_per_dependent_load\": %.1f}\n", r[0] * 10.0 / n);

    uint32_t *hin = h + 64, *hout = h + 128; /* separate cache lines */
    uint32_t *din = (uint32_t *)dh + 64, *dout = (uint32_t *)dh + 128;
    *hin = 0;
    *hout = 0;
    double us = pingpong(hin, hout, din, dout, 5000);
    printf("{\"probe\": \"host->gpu->host ping-pong, both words in coherent host memory\", \"us_per_round_trip\": %.3f}\n",
           us);

    /* poll word in fine-grained device memory written by the host (if mappable) */
    uint32_t *dev = nullptr;
    if (hipExtMallocWithFlags((void **)&dev, 4096, hipDeviceMallocFinegrained) == hipSuccess) {
        hipPointerAttribute_t at;
        bool host_ok = hipPointerGetAttributes(&at, dev) == hipSuccess;
        printf("{\"probe\": \"fine-grained device alloc\", \"attr_ok\": %d, \"hostPointer\": \"%p\"}\n", (int)host_ok,
               host_ok ? at.hostPointer : nullptr);
    }
    hipHostFree(h);
    hipFree(o);
    return 0;
}
