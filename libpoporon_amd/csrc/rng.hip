/*
 * rng.hip -- the reference's byte source, xoshiro128++ seeded through
 * splitmix32 (src/rng.c:17-132): host API (include/poporon/rng.h) and a
 * device fill (include/poporon_amd.h) that writes the same byte stream into
 * device memory.
 *
 * Device fill.  The xoshiro128 state update is linear over GF(2) (128-bit
 * state, s' = M s; only the output function is nonlinear), so the state
 * after k steps is M^k s.  The fill cuts the word stream into blocks of
 * RNG_BLOCK words; the host derives the start state of every block by
 * repeated application of M^RNG_BLOCK (a 128 x 128 bit matrix, built by
 * squaring), and one lane generates each block with the plain recurrence.
 * The handle's state then advances by the number of words written
 * (M^n s, square-and-multiply), exactly as poporon_rng_next would.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "poporon/rng.h"
#include "rs_device.h" /* RS_LAUNCH */

#define EXPORT extern "C" __attribute__((visibility("default")))
#define RNG_BLOCK 1024u /* words per lane */

struct _poporon_rng_t {
    poporon_rng_type_t type;
    uint32_t s[4];
    /* device-fill cache: block start states */
    uint32_t *d_starts = nullptr;
    size_t starts_cap = 0;
    int device = -1;
};

__host__ __device__ static inline uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

static inline uint32_t splitmix32(uint32_t z)
{
    z = (z ^ (z >> 16)) * 0x85EBCA6Bu;
    z = (z ^ (z >> 13)) * 0xC2B2AE35u;
    return z ^ (z >> 16);
}

/* one output and one state step (src/rng.c:62-76) */
__host__ __device__ static inline uint32_t xo_next(uint32_t (&s)[4])
{
    const uint32_t r = rotl32(s[0] + s[3], 7) + s[0];
    const uint32_t t = s[1] << 9;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl32(s[3], 11);
    return r;
}

EXPORT poporon_rng_t *poporon_rng_create(poporon_rng_type_t type, void *seed, size_t seed_size)
{
    poporon_rng_t *r = new (std::nothrow) _poporon_rng_t();
    if (!r)
        return nullptr;
    r->type = type;
    /* every type seeds xoshiro128++ (src/rng.c:88-93) */
    uint32_t s = 0;
    if (seed && seed_size > 0)
        memcpy(&s, seed, seed_size < sizeof(uint32_t) ? seed_size : sizeof(uint32_t));
    r->s[0] = splitmix32(s + 0x6C078965u);
    r->s[1] = splitmix32(r->s[0] + 0x9D2C5680u);
    r->s[2] = splitmix32(r->s[1] + 0xEFC60000u);
    r->s[3] = splitmix32(r->s[2] + 0x12345678u);
    return r;
}

EXPORT void poporon_rng_destroy(poporon_rng_t *r)
{
    if (!r)
        return;
    if (r->d_starts) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        (void)hipSetDevice(r->device);
        (void)hipFree(r->d_starts);
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
    delete r;
}

EXPORT bool poporon_rng_next(poporon_rng_t *r, void *dest, size_t size)
{
    if (!r || !dest || size == 0)
        return false;
    uint8_t *p = (uint8_t *)dest;
    size_t i = 0;
    for (; i + 4 <= size; i += 4) {
        const uint32_t v = xo_next(r->s);
        memcpy(p + i, &v, 4);
    }
    if (i < size) {
        const uint32_t v = xo_next(r->s);
        memcpy(p + i, &v, size - i);
    }
    return true;
}

/* ---- GF(2) jump-ahead: 128 x 128 matrices as 128 column images ---- */
struct Mat {
    uint32_t c[128][4]; /* c[j] = M e_j */
};

static void apply(const Mat &m, const uint32_t (&x)[4], uint32_t (&y)[4])
{
    uint32_t o[4] = {0, 0, 0, 0};
    for (int j = 0; j < 128; j++)
        if ((x[j >> 5] >> (j & 31)) & 1u)
            for (int w = 0; w < 4; w++)
                o[w] ^= m.c[j][w];
    memcpy(y, o, sizeof(o));
}

static void mul(const Mat &a, const Mat &b, Mat &out) /* out = a b */
{
    Mat t;
    for (int j = 0; j < 128; j++)
        apply(a, b.c[j], t.c[j]);
    out = t;
}

static void step_matrix(Mat &m)
{
    for (int j = 0; j < 128; j++) {
        uint32_t s[4] = {0, 0, 0, 0};
        s[j >> 5] = 1u << (j & 31);
        (void)xo_next(s);
        memcpy(m.c[j], s, sizeof(s));
    }
}

/* m = M^(2^k) */
static void pow2_matrix(unsigned k, Mat &m)
{
    step_matrix(m);
    for (unsigned i = 0; i < k; i++)
        mul(m, m, m);
}

static void advance(uint32_t (&s)[4], uint64_t n)
{
    Mat p;
    step_matrix(p);
    while (n) {
        if (n & 1u)
            apply(p, s, s);
        n >>= 1;
        if (n)
            mul(p, p, p);
    }
}

__global__ __launch_bounds__(256) void rng_fill_k(const uint32_t *__restrict__ starts, uint8_t *__restrict__ dst,
                                                   size_t size, size_t nblocks)
{
    const size_t b = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (b >= nblocks)
        return;
    uint32_t s[4] = {starts[4 * b], starts[4 * b + 1], starts[4 * b + 2], starts[4 * b + 3]};
    const size_t w0 = b * RNG_BLOCK;
    const size_t nwords = (size + 3) / 4;
    const size_t w1 = w0 + RNG_BLOCK < nwords ? w0 + RNG_BLOCK : nwords;
    const bool aligned = (reinterpret_cast<uintptr_t>(dst) & 3u) == 0;
    for (size_t w = w0; w < w1; ++w) {
        const uint32_t v = xo_next(s);
        const size_t off = 4 * w;
        if (aligned && off + 4 <= size) {
            *reinterpret_cast<uint32_t *>(dst + off) = v;
        } else {
            for (size_t k = 0; k < 4 && off + k < size; ++k)
                dst[off + k] = (uint8_t)(v >> (8 * k));
        }
    }
}

extern "C" __attribute__((visibility("default"))) bool poporon_amd_rng_fill_device(poporon_rng_t *r, void *d_dest,
                                                                                     size_t size, void *stream)
{
    if (!r || !d_dest || size == 0)
        return false;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess)
        return false;
    const uint64_t nwords = (size + 3) / 4;
    const size_t nblocks = (size_t)((nwords + RNG_BLOCK - 1) / RNG_BLOCK);
    std::vector<uint32_t> starts(4 * nblocks);
    {
        static const Mat jump = [] { /* M^RNG_BLOCK (RNG_BLOCK = 2^10), built once */
            Mat m;
            pow2_matrix(10, m);
            return m;
        }();
        uint32_t s[4] = {r->s[0], r->s[1], r->s[2], r->s[3]};
        for (size_t b = 0; b < nblocks; b++) {
            memcpy(&starts[4 * b], s, sizeof(s));
            if (b + 1 < nblocks)
                apply(jump, s, s);
        }
    }
    if (r->d_starts && (r->starts_cap < nblocks || r->device != dev)) {
        if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
            return false;
        (void)hipFree(r->d_starts);
        r->d_starts = nullptr;
        r->starts_cap = 0;
    }
    if (!r->d_starts) {
        if (hipMalloc((void **)&r->d_starts, std::max<size_t>(nblocks, 64) * 16) != hipSuccess)
            return false;
        r->starts_cap = std::max<size_t>(nblocks, 64);
        r->device = dev;
    }
    /* the copy from pageable memory completes before hipMemcpyAsync returns */
    if (hipMemcpyAsync(r->d_starts, starts.data(), nblocks * 16, hipMemcpyHostToDevice, (hipStream_t)stream) !=
        hipSuccess)
        return false;
    if (hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return false;
    RS_LAUNCH(rng_fill_k, dim3((uint32_t)((nblocks + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       r->d_starts, (uint8_t *)d_dest, size, nblocks);
    if (hipGetLastError() != hipSuccess)
        return false;
    advance(r->s, nwords);
    return true;
}
