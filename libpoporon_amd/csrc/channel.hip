/*
 * channel.hip -- symbol-error channel for tests and benchmarks (not part of
 * the codec): XOR per-codeword magnitudes into per-codeword positions of a
 * device-resident batch of codeword rows, in place.
 *
 * One thread per (codeword, error): byte loads/stores only, so errors at
 * distinct positions of one row never race (positions within a row must be
 * distinct, as the benchmark's error patterns are).
 */
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void channel_xor_k(const uint8_t *__restrict__ pos, const uint8_t *__restrict__ mag,
                                                      uint32_t nper, uint8_t *cw, size_t stride, size_t total)
{
    const size_t t = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= total)
        return;
    const size_t c = t / nper;
    uint8_t *p = cw + c * stride + pos[t];
    *p = (uint8_t)(*p ^ mag[t]);
}

extern "C" __attribute__((visibility("default"))) bool
poporon_amd_channel_xor_device(const uint8_t *d_positions, const uint8_t *d_magnitudes, size_t per_codeword,
                               uint8_t *d_codewords, size_t stride, size_t count, void *stream)
{
    if (!d_positions || !d_magnitudes || !d_codewords || per_codeword == 0 || per_codeword > 255)
        return count == 0 || per_codeword == 0;
    const size_t total = per_codeword * count;
    if (total == 0)
        return true;
    const size_t blocks = (total + 255) / 256;
    if (blocks > 0x7fffffffu)
        return false;
    hipLaunchKernelGGL(channel_xor_k, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream, d_positions,
                       d_magnitudes, (uint32_t)per_codeword, d_codewords, stride, total);
    return hipGetLastError() == hipSuccess;
}
