/*
 * bch.hip -- binary BCH codec of libpoporon on gfx950 (codewords of up to
 * 31 bits: symbol_size 3..5), batched, one codeword per lane.
 *
 *   bch_encode_k   poporon_encode for PPLN_FEC_BCH    src/encode.c:199-233,
 *                  systematic division by g(x)        src/bch.c:359-384
 *   bch_decode_k   poporon_decode for PPLN_FEC_BCH    src/decode.c:542-590,
 *                  syndromes / BM / Chien / re-check  src/bch.c:25-165, :386-436
 *
 * The reference's arithmetic is restated with its exact loop bounds and
 * update rules (its BM keeps 64-entry polynomials and a "shift" counter; the
 * results, including miscorrections and failures, are bit-exact).  The
 * per-codeword arrays (2t syndromes, three 64-entry polynomial buffers, the
 * error positions) live in LDS laid out [index][lane]; the GF(2^m) tables
 * (<= 32 entries each) sit in LDS in front of them.  Polynomial loops run
 * only up to tracked degree bounds: entries past them are zero and would
 * contribute nothing.
 */
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bch_device.h"
#include "rs_device.h" /* RS_LAUNCH */

#define B_WG 256
#define B_POLY 64 /* BCH_MAX_POLY, src/bch.c:12 */
#define B_SLOTS (32 + 3 * B_POLY + 16)

struct BLane {
    uint8_t *p;
    __device__ __forceinline__ uint8_t &operator[](uint32_t i) const { return p[i * B_WG]; }
};

__device__ __forceinline__ void bch_tables(const BchParams &P, uint8_t *alog, uint8_t *lg)
{
    if (threadIdx.x < 32u) {
        alog[threadIdx.x] = P.alog[threadIdx.x];
        lg[threadIdx.x] = P.log[threadIdx.x];
    }
    __syncthreads();
}

/* big-endian byte image <-> value, src/encode.c:214-219 / src/decode.c:558-570 */
__device__ __forceinline__ uint32_t be_read(const uint8_t *p, uint32_t nbytes, uint32_t bits)
{
    uint32_t v = 0;
    for (uint32_t i = 0; i < nbytes && i < 4u; ++i)
        v |= (uint32_t)p[i] << (8u * (nbytes - 1u - i));
    if (bits < 32u)
        v &= (1u << bits) - 1u;
    return v;
}

__global__ __launch_bounds__(B_WG) void bch_encode_k(BchParams P, const uint8_t *__restrict__ data, size_t dstride,
                                                      uint8_t *__restrict__ parity, size_t pstride, size_t count)
{
    for (size_t cw = (size_t)blockIdx.x * B_WG + threadIdx.x; cw < count; cw += (size_t)gridDim.x * B_WG) {
        const uint32_t dv = be_read(data + cw * dstride, P.dbytes, P.k);
        const uint32_t sh = dv << P.pbits;
        uint32_t r = sh;
        for (int i = (int)P.nn - 1; i >= (int)P.gdeg; --i)
            if (r & (1u << i))
                r ^= P.gen << (i - (int)P.gdeg);
        const uint32_t pv = (sh ^ r) & ((1u << P.pbits) - 1u);
        uint8_t *o = parity + cw * pstride;
        for (uint32_t i = 0; i < P.pbytes; ++i)
            o[P.pbytes - 1u - i] = i < 4u ? (uint8_t)(pv >> (8u * i)) : (uint8_t)0;
    }
}

/* syndromes S_i = r(alpha^(i+1)), i < 2t (src/bch.c:25-50); returns any nonzero */
__device__ __forceinline__ bool bch_syn(const BchParams &P, const uint8_t *alog, uint32_t w, const BLane &S)
{
    bool nz = false;
    for (uint32_t i = 0; i < 2u * P.t; ++i) {
        const uint32_t step = (i + 1u) % P.nn;
        uint32_t s = 0, e = 0; /* e = (i+1) j mod nn, stepped with j */
        for (uint32_t j = 0; j < P.nn; ++j) {
            if (w & (1u << j))
                s ^= alog[e];
            e += step;
            e = e >= P.nn ? e - P.nn : e;
        }
        S[i] = (uint8_t)s;
        nz |= s != 0u;
    }
    return nz;
}

__global__ __launch_bounds__(B_WG) void bch_decode_k(BchParams P, uint8_t *data, size_t dstride,
                                                      const uint8_t *__restrict__ parity, size_t pstride,
                                                      size_t count, uint8_t *__restrict__ ok,
                                                      uint8_t *__restrict__ corrected)
{
    __shared__ uint8_t alog[32], lg[32];
    __shared__ uint8_t lane_mem[B_SLOTS * B_WG];
    bch_tables(P, alog, lg);
    const uint32_t nn = P.nn;
    const BLane S{lane_mem + threadIdx.x};
    /* polynomial buffer `slot` (0..2) of this lane */
    auto buf = [&](uint32_t slot) { return BLane{lane_mem + (32u + slot * B_POLY) * B_WG + threadIdx.x}; };
    const BLane pos{lane_mem + (32u + 3u * B_POLY) * B_WG + threadIdx.x};
    for (size_t cw = (size_t)blockIdx.x * B_WG + threadIdx.x; cw < count; cw += (size_t)gridDim.x * B_WG) {
        uint8_t *d = data + cw * dstride;
        const uint32_t dv = be_read(d, P.dbytes, P.k);
        const uint32_t pv = be_read(parity + cw * pstride, P.pbytes, P.pbits);
        const uint32_t rx = ((dv << P.pbits) | pv) & ((1u << nn) - 1u);
        bool good = true;
        uint32_t out = rx, nerr = 0;
        if (bch_syn(P, alog, rx, S)) {
            /* ---- Berlekamp-Massey, src/bch.c:77-141 ---- */
            uint32_t ic = 0, ip = 1, is = 2; /* current, previous, scratch buffers */
            const BLane b0 = buf(0), b1 = buf(1);
            for (uint32_t i = 0; i < B_POLY; ++i) {
                b0[i] = 0;
                b1[i] = 0;
            }
            b0[0] = 1;
            b1[0] = 1;
            uint32_t cdeg = 0, pdeg = 0; /* bounds of the nonzero entries */
            int ec = 0, shift = 1;
            uint32_t pd = 1;
            for (int it = 0; it < (int)(2u * P.t); ++it) {
                const BLane cur = buf(ic), prev = buf(ip);
                uint32_t dsc = S[(uint32_t)it];
                for (int i = 1; i <= ec; ++i) {
                    const uint32_t ci = cur[(uint32_t)i], si = S[(uint32_t)(it - i)];
                    if (ci && si)
                        dsc ^= alog[(lg[ci] + lg[si]) % nn];
                }
                if (dsc == 0u) {
                    ++shift;
                    continue;
                }
                const uint32_t lmult = lg[alog[(nn - lg[pd] + lg[dsc]) % nn]];
                const uint32_t top = (uint32_t)(B_POLY - shift); /* i < top */
                const uint32_t lim = min(pdeg + 1u, top);
                if (2 * ec <= it) {
                    /* scratch = cur + mult x^shift prev; prev <- cur; cur <- scratch */
                    const BLane nw = buf(is);
                    for (uint32_t i = 0; i < B_POLY; ++i)
                        nw[i] = cur[i];
                    for (uint32_t i = 0; i < lim; ++i) {
                        const uint32_t pi = prev[i];
                        if (pi)
                            nw[i + (uint32_t)shift] = (uint8_t)(nw[i + (uint32_t)shift] ^ alog[(lg[pi] + lmult) % nn]);
                    }
                    const uint32_t ndeg = lim ? max(cdeg, lim - 1u + (uint32_t)shift) : cdeg;
                    const uint32_t t0 = ip;
                    ip = ic;
                    ic = is;
                    is = t0;
                    pdeg = cdeg;
                    cdeg = ndeg;
                    ec = it + 1 - ec;
                    pd = dsc;
                    shift = 1;
                } else {
                    for (uint32_t i = 0; i < lim; ++i) {
                        const uint32_t pi = prev[i];
                        if (pi)
                            cur[i + (uint32_t)shift] =
                                (uint8_t)(cur[i + (uint32_t)shift] ^ alog[(lg[pi] + lmult) % nn]);
                    }
                    if (lim)
                        cdeg = max(cdeg, lim - 1u + (uint32_t)shift);
                    ++shift;
                }
            }
            if (ec > (int)P.t) {
                good = false;
            } else {
                /* ---- Chien over i < nn: Lambda(alpha^-i), src/bch.c:52-75, :143-165 ---- */
                const BLane loc = buf(ic);
                int found = 0;
                for (uint32_t i = 0; i < nn; ++i) {
                    const uint32_t x = alog[(nn - i) % nn];
                    const uint32_t lx = lg[x];
                    uint32_t sum = 0;
                    for (int j = 0; j <= ec; ++j) {
                        const uint32_t pj = loc[(uint32_t)j];
                        if (pj)
                            sum ^= alog[(lg[pj] + (lx * (uint32_t)j) % nn) % nn];
                    }
                    if (sum == 0u) {
                        pos[(uint32_t)found++] = (uint8_t)i;
                        if (found >= ec)
                            break;
                    }
                }
                if (found != ec) {
                    good = false;
                } else {
                    uint32_t fixed = rx;
                    for (int i = 0; i < found; ++i)
                        fixed ^= 1u << pos[(uint32_t)i];
                    if (bch_syn(P, alog, fixed, S)) {
                        good = false;
                    } else {
                        out = fixed;
                        nerr = (uint32_t)found;
                    }
                }
            }
        }
        if (good) {
            const uint32_t cd = (out >> P.pbits) & ((1u << P.k) - 1u);
            for (uint32_t i = 0; i < P.dbytes && i < 4u; ++i)
                d[P.dbytes - 1u - i] = (uint8_t)(cd >> (8u * i));
        }
        ok[cw] = good ? 1 : 0;
        if (corrected)
            corrected[cw] = good ? (uint8_t)nerr : (uint8_t)0;
    }
}

static dim3 bch_grid(size_t count, int num_cu)
{
    const size_t need = (count + B_WG - 1) / B_WG;
    const size_t cap = (size_t)(num_cu > 0 ? num_cu : 256) * 8;
    return dim3((uint32_t)std::max<size_t>(1, std::min(need, cap)));
}

extern "C" hipError_t bchk_encode(const BchParams *prm, const uint8_t *data, size_t dstride, uint8_t *parity,
                                  size_t pstride, size_t count, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(bch_encode_k, bch_grid(count, num_cu), dim3(B_WG), 0, stream, *prm, data, dstride, parity,
                       pstride, count);
    return hipGetLastError();
}

extern "C" hipError_t bchk_decode(const BchParams *prm, uint8_t *data, size_t dstride, const uint8_t *parity,
                                  size_t pstride, size_t count, uint8_t *ok, uint8_t *corrected, int num_cu,
                                  hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(bch_decode_k, bch_grid(count, num_cu), dim3(B_WG), 0, stream, *prm, data, dstride, parity,
                       pstride, count, ok, corrected);
    return hipGetLastError();
}
