/*
 * testutil.hip -- test and benchmark utilities for libpoporon_amd (NOT part
 * of the codec; built as libpoporon_testutil.so, never linked into
 * libpoporon_amd.so).
 *
 *   ptu_synth_rows      counter-hash payload bytes, keyed by (seed, global row)
 *   ptu_synth_errors    per-row unique error positions + nonzero magnitudes
 *   ptu_channel_xor     symbol-error channel (XOR magnitudes into positions)
 *   ptu_checksum        order-independent 64-bit checksum of a row batch
 *   ptu_time_encode / ptu_time_decode
 *                       a C loop of single-codeword calls through function
 *                       pointers (poporon_encode / poporon_decode of
 *                       whichever library the caller resolved): the
 *                       reference's calling pattern timed without any
 *                       interpreter overhead, as the CPU baseline's C loop is
 *
 * Every value depends only on (seed, global row index), so any sharding of a
 * batch over ranks produces the same rows; testutil/__init__.py restates each
 * formula in numpy (the CPU side of the tests), and tests check the two agree.
 */
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <chrono>

#define PTU_EXPORT extern "C" __attribute__((visibility("default")))

__device__ __forceinline__ uint32_t fmix32(uint32_t x)
{
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    return x ^ (x >> 16);
}

__device__ __forceinline__ uint64_t fmix64(uint64_t x)
{
    x ^= x >> 33;
    x *= 0xFF51AFD7ED558CCDull;
    x ^= x >> 33;
    x *= 0xC4CEB9FE1A85EC53ull;
    return x ^ (x >> 33);
}

/* byte j of row i = fmix32(((first + i) * width + j) * 0x9E3779B1 + seed) & 255 */
__global__ __launch_bounds__(256) void synth_rows_k(uint32_t seed, uint64_t first, uint64_t count, uint32_t width,
                                                    uint8_t *__restrict__ out, uint64_t stride)
{
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    const uint64_t row = t / width;
    if (row >= count)
        return;
    const uint32_t j = (uint32_t)(t - row * width);
    const uint32_t ctr = (uint32_t)((first + row) * width + j);
    out[row * stride + j] = (uint8_t)fmix32(ctr * 0x9E3779B1u + seed);
}

/* Positions: the nerr columns c < span with the largest keys
 * fmix32(((first + i) * span + c) * 0x9E3779B1 + seed), in descending key
 * order (or ascending position order when sorted != 0, magnitudes moving
 * with their positions).  Magnitudes: fmix32(((first + i) * nerr + e) *
 * 0x9E3779B1 + seed + 0x1234567) % 255 + 1 for the e-th key. */
__global__ __launch_bounds__(256) void synth_errors_k(uint32_t seed, uint64_t first, uint64_t count, uint32_t nerr,
                                                      uint32_t span, int sorted, uint8_t *__restrict__ pos,
                                                      uint8_t *__restrict__ mag)
{
    const uint64_t row = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (row >= count)
        return;
    uint32_t key[64];
    uint8_t col[64];
    uint32_t n = 0;
    const uint32_t base = (uint32_t)((first + row) * span);
    for (uint32_t c = 0; c < span; ++c) {
        const uint32_t k = fmix32((base + c) * 0x9E3779B1u + seed);
        if (n == nerr && k <= key[n - 1])
            continue;
        uint32_t p = n < nerr ? n++ : n - 1; /* insertion: descending keys */
        while (p > 0 && key[p - 1] < k) {
            key[p] = key[p - 1];
            col[p] = col[p - 1];
            --p;
        }
        key[p] = k;
        col[p] = (uint8_t)c;
    }
    uint8_t m[64];
    const uint32_t mb = (uint32_t)((first + row) * nerr);
    for (uint32_t e = 0; e < nerr; ++e)
        m[e] = (uint8_t)(fmix32((mb + e) * 0x9E3779B1u + seed + 0x1234567u) % 255u + 1u);
    if (sorted) {
        for (uint32_t a = 1; a < nerr; ++a) { /* insertion sort by position, magnitudes follow */
            const uint8_t pc = col[a], pm = m[a];
            uint32_t b = a;
            while (b > 0 && col[b - 1] > pc) {
                col[b] = col[b - 1];
                m[b] = m[b - 1];
                --b;
            }
            col[b] = pc;
            m[b] = pm;
        }
    }
    for (uint32_t e = 0; e < nerr; ++e) {
        pos[row * nerr + e] = col[e];
        mag[row * nerr + e] = m[e];
    }
}

/* one thread per (row, error): byte read-modify-write, positions of a row distinct */
__global__ __launch_bounds__(256) void channel_xor_k(const uint8_t *__restrict__ pos, const uint8_t *__restrict__ mag,
                                                     uint32_t nper, uint8_t *cw, uint64_t stride, uint64_t total)
{
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= total)
        return;
    const uint64_t c = t / nper;
    uint8_t *p = cw + c * stride + pos[t];
    *p = (uint8_t)(*p ^ mag[t]);
}

/* sum over rows of H(first + i, row bytes): FNV-1a-64 over the bytes seeded by
 * fmix64 of the global row index, finished by fmix64 (sum mod 2^64) */
__global__ __launch_bounds__(256) void checksum_k(const uint8_t *__restrict__ rows, uint64_t stride, uint32_t width,
                                                  uint64_t first, uint64_t count, unsigned long long *sum)
{
    const uint64_t row = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    uint64_t h = 0;
    if (row < count) {
        const uint8_t *r = rows + row * stride;
        h = fmix64((first + row) * 0x9E3779B97F4A7C15ull + width);
        for (uint32_t j = 0; j < width; ++j)
            h = (h ^ r[j]) * 0x100000001B3ull;
        h = fmix64(h);
    }
    for (int o = 32; o > 0; o >>= 1)
        h += __shfl_xor(h, o, 64);
    if ((threadIdx.x & 63u) == 0u && h)
        atomicAdd(sum, (unsigned long long)h);
}

static bool grid_of(uint64_t threads, uint32_t *g)
{
    const uint64_t b = (threads + 255) / 256;
    if (b > 0x7fffffffull)
        return false;
    *g = (uint32_t)(b ? b : 1);
    return true;
}

PTU_EXPORT bool ptu_synth_rows(uint32_t seed, uint64_t first, uint64_t count, uint32_t width, uint8_t *d_out,
                               uint64_t stride, void *stream)
{
    uint32_t g;
    if (!count || !width)
        return true;
    if (!d_out || stride < width || !grid_of(count * width, &g))
        return false;
    hipLaunchKernelGGL(synth_rows_k, dim3(g), dim3(256), 0, (hipStream_t)stream, seed, first, count, width, d_out,
                       stride);
    return hipGetLastError() == hipSuccess;
}

PTU_EXPORT bool ptu_synth_errors(uint32_t seed, uint64_t first, uint64_t count, uint32_t nerr, uint32_t span,
                                 int sorted, uint8_t *d_pos, uint8_t *d_mag, void *stream)
{
    uint32_t g;
    if (!count)
        return true;
    if (!d_pos || !d_mag || nerr == 0 || nerr > 64 || nerr > span || span > 256 || !grid_of(count, &g))
        return false;
    hipLaunchKernelGGL(synth_errors_k, dim3(g), dim3(256), 0, (hipStream_t)stream, seed, first, count, nerr, span,
                       sorted, d_pos, d_mag);
    return hipGetLastError() == hipSuccess;
}

PTU_EXPORT bool ptu_channel_xor(const uint8_t *d_positions, const uint8_t *d_magnitudes, uint64_t per_row,
                                uint8_t *d_rows, uint64_t stride, uint64_t count, void *stream)
{
    uint32_t g;
    if (!count || !per_row)
        return true;
    if (!d_positions || !d_magnitudes || !d_rows || per_row > 255 || !grid_of(per_row * count, &g))
        return false;
    hipLaunchKernelGGL(channel_xor_k, dim3(g), dim3(256), 0, (hipStream_t)stream, d_positions, d_magnitudes,
                       (uint32_t)per_row, d_rows, stride, per_row * count);
    return hipGetLastError() == hipSuccess;
}

/* *d_sum += checksum of the rows (d_sum: one device u64, caller-initialised) */
PTU_EXPORT bool ptu_checksum(const uint8_t *d_rows, uint64_t stride, uint32_t width, uint64_t first, uint64_t count,
                             uint64_t *d_sum, void *stream)
{
    uint32_t g;
    if (!count)
        return true;
    if (!d_rows || !d_sum || !grid_of(count, &g))
        return false;
    hipLaunchKernelGGL(checksum_k, dim3(g), dim3(256), 0, (hipStream_t)stream, d_rows, stride, width, first, count,
                       (unsigned long long *)d_sum);
    return hipGetLastError() == hipSuccess;
}

/* ------------------------------------------------------------------------ */
/* single-call latency loops (host code)                                    */
/* ------------------------------------------------------------------------ */
typedef bool (*ptu_enc_fn)(void *, uint8_t *, size_t, uint8_t *);
typedef bool (*ptu_dec_fn)(void *, uint8_t *, size_t, uint8_t *, size_t *);

/* calls x enc(h, msgs + c * size, size, par + c * pstride); seconds, or -1
 * if a call failed */
PTU_EXPORT double ptu_time_encode(void *fn, void *h, uint8_t *msgs, uint64_t size, uint8_t *par, uint64_t pstride,
                                  uint64_t calls)
{
    const ptu_enc_fn enc = (ptu_enc_fn)fn;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t c = 0; c < calls; ++c)
        if (!enc(h, msgs + c * size, size, par + c * pstride))
            return -1.0;
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

/* calls x dec(h, data + c * dstride, size, par + c * pstride, &n), ok / corrected
 * recorded per call; seconds */
PTU_EXPORT double ptu_time_decode(void *fn, void *h, uint8_t *data, uint64_t dstride, uint8_t *par, uint64_t pstride,
                                  uint64_t size, uint64_t calls, uint8_t *ok, uint8_t *cor)
{
    const ptu_dec_fn dec = (ptu_dec_fn)fn;
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t c = 0; c < calls; ++c) {
        size_t n = 0;
        ok[c] = dec(h, data + c * dstride, size, par + c * pstride, &n) ? 1 : 0;
        /* a device failure (corrected_num = POPORON_AMD_DEVICE_ERROR, past
         * every count the reference reports) is recorded as 255, never
         * truncated into an ordinary count */
        cor[c] = n > 254u ? (uint8_t)255u : (uint8_t)n;
    }
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
