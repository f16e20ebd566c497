/*
 * rs_kernels.hip -- RS(n, n-32) over GF(2^8) on CDNA4 (gfx950).
 *
 * Kernels
 *   rs_lfsr_k<MODE_ENCODE>  encode: parity = m(x) x^32 mod g(x)        (src/encode.c:120-143)
 *   rs_lfsr_k<MODE_REMAINDER>   remainder of the received word mod g(x); the syndromes
 *                     of src/decode.c:375-415 are r(beta_i) since g(beta_i)=0
 *   rs_correct_k      syndromes from the remainder, erasure locator, BM,
 *                     Chien, Omega, Forney, re-syndrome check and apply
 *                     (src/decode.c:17-230), one codeword per lane
 *
 * LFSR layout.  One codeword per lane; the 32-byte shift register lives in 8
 * VGPRs.  A feedback byte fb selects a 32-byte row (fb * g(x), pre-shifted)
 * that is XORed into the register after a one-byte funnel shift.  The 8 KB
 * row table is replicated 16 times in LDS (128 KB): lane l reads copy l & 15,
 * and copy c of every 16-byte half-row sits in bank slot c, so each
 * ds_read_b128 lane group (16 lanes, one per slot) is conflict-free whatever
 * the data (MI355X_MICROARCH.md §LDS).  1024-thread workgroups, one per CU,
 * persistent over the batch.
 */
#include <hip/hip_runtime.h>

#include "rs_device.h"

#define LFSR_WG 1024
#define LFSR_REPL 16

/* ------------------------------------------------------------------------ */
/* LFSR (encode / remainder)                                                */
/* ------------------------------------------------------------------------ */

__device__ __forceinline__ void lfsr_step(uint32_t (&P)[8], uint32_t in_byte, const uint4 *__restrict__ tab)
{
    const uint32_t fb = (P[0] ^ in_byte) & 0xffu;
    const uint4 a = tab[fb * (2 * LFSR_REPL)];
    const uint4 b = tab[fb * (2 * LFSR_REPL) + LFSR_REPL];
    P[0] = __builtin_amdgcn_alignbyte(P[1], P[0], 1) ^ a.x;
    P[1] = __builtin_amdgcn_alignbyte(P[2], P[1], 1) ^ a.y;
    P[2] = __builtin_amdgcn_alignbyte(P[3], P[2], 1) ^ a.z;
    P[3] = __builtin_amdgcn_alignbyte(P[4], P[3], 1) ^ a.w;
    P[4] = __builtin_amdgcn_alignbyte(P[5], P[4], 1) ^ b.x;
    P[5] = __builtin_amdgcn_alignbyte(P[6], P[5], 1) ^ b.y;
    P[6] = __builtin_amdgcn_alignbyte(P[7], P[6], 1) ^ b.z;
    P[7] = (P[7] >> 8) ^ b.w;
}

__device__ __forceinline__ void lfsr_word(uint32_t (&P)[8], uint32_t w, const uint4 *__restrict__ tab)
{
    lfsr_step(P, w & 0xffu, tab);
    lfsr_step(P, (w >> 8) & 0xffu, tab);
    lfsr_step(P, (w >> 16) & 0xffu, tab);
    lfsr_step(P, w >> 24, tab);
}

/* Feed n bytes starting at p (any alignment).  Only aligned dwords that
 * contain at least one message byte are loaded, so no load can cross into an
 * unmapped page. */
__device__ __forceinline__ void lfsr_feed(uint32_t (&P)[8], const uint8_t *p, uint32_t n, const uint4 *__restrict__ tab)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
    const uint32_t sh = static_cast<uint32_t>(a & 3u);
    const uint32_t nd = (sh + n + 3u) >> 2; /* dwords holding message bytes */
    if (n == 0)
        return;
    uint32_t cur = w[0];
    uint32_t q = 0;
    uint32_t i = 0;
    for (; i + 16u <= n; i += 16u, q += 4u) {
        const uint32_t w1 = (q + 1u < nd) ? w[q + 1u] : 0u;
        const uint32_t w2 = (q + 2u < nd) ? w[q + 2u] : 0u;
        const uint32_t w3 = (q + 3u < nd) ? w[q + 3u] : 0u;
        const uint32_t w4 = (q + 4u < nd) ? w[q + 4u] : 0u;
        lfsr_word(P, __builtin_amdgcn_alignbyte(w1, cur, sh), tab);
        lfsr_word(P, __builtin_amdgcn_alignbyte(w2, w1, sh), tab);
        lfsr_word(P, __builtin_amdgcn_alignbyte(w3, w2, sh), tab);
        lfsr_word(P, __builtin_amdgcn_alignbyte(w4, w3, sh), tab);
        cur = w4;
    }
    if (i < n) {
        const uint32_t w1 = (q + 1u < nd) ? w[q + 1u] : 0u;
        const uint32_t w2 = (q + 2u < nd) ? w[q + 2u] : 0u;
        const uint32_t w3 = (q + 3u < nd) ? w[q + 3u] : 0u;
        const uint32_t w4 = (q + 4u < nd) ? w[q + 4u] : 0u;
        const uint32_t m[4] = {__builtin_amdgcn_alignbyte(w1, cur, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                               __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
        const uint32_t rem = n - i;
#pragma unroll
        for (uint32_t b = 0; b < 16u; ++b)
            if (b < rem)
                lfsr_step(P, (m[b >> 2] >> (8u * (b & 3u))) & 0xffu, tab);
    }
}

#define MODE_ENCODE 0
#define MODE_REMAINDER 1
#define MODE_CHECK 2

template <int MODE>
__global__ __launch_bounds__(LFSR_WG) void rs_lfsr_k(const uint4 *__restrict__ rows, const uint8_t *__restrict__ data,
                                                      size_t dstride, uint8_t *__restrict__ parity, size_t pstride,
                                                      uint32_t size, size_t count, uint8_t *__restrict__ rem,
                                                      int par_aligned)
{
    __shared__ uint4 lds[512 * LFSR_REPL];
    for (uint32_t t = threadIdx.x; t < 512u * LFSR_REPL; t += LFSR_WG)
        lds[t] = rows[t / LFSR_REPL];
    __syncthreads();
    const uint4 *tab = lds + (threadIdx.x & (LFSR_REPL - 1));

    for (size_t cw = (size_t)blockIdx.x * LFSR_WG + threadIdx.x; cw < count; cw += (size_t)gridDim.x * LFSR_WG) {
        uint32_t P[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        lfsr_feed(P, data + cw * dstride, size, tab);
        if (MODE == MODE_REMAINDER) {
            lfsr_feed(P, parity + cw * pstride, RS_NR, tab);
            uint4 *o = reinterpret_cast<uint4 *>(rem + cw * RS_NR);
            o[0] = make_uint4(P[0], P[1], P[2], P[3]);
            o[1] = make_uint4(P[4], P[5], P[6], P[7]);
        } else if (MODE == MODE_CHECK) {
            lfsr_feed(P, parity + cw * pstride, RS_NR, tab);
            rem[cw] = (P[0] | P[1] | P[2] | P[3] | P[4] | P[5] | P[6] | P[7]) != 0u;
        } else {
            uint8_t *o = parity + cw * pstride;
            if (par_aligned) {
                uint32_t *o4 = reinterpret_cast<uint32_t *>(o);
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    o4[k] = P[k];
            } else {
#pragma unroll
                for (int k = 0; k < 32; ++k)
                    o[k] = (uint8_t)(P[k >> 2] >> (8 * (k & 3)));
            }
        }
    }
}

static int lfsr_grid(size_t count, int num_cu)
{
    size_t need = (count + LFSR_WG - 1) / LFSR_WG;
    size_t g = (size_t)(num_cu > 0 ? num_cu : 256);
    return (int)(need < g ? (need ? need : 1) : g);
}

extern "C" hipError_t rsk_encode(const RsDevTables *tab, const uint8_t *data, size_t dstride, uint8_t *parity,
                                 size_t pstride, uint32_t size, size_t count, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const int aligned = ((reinterpret_cast<uintptr_t>(parity) | pstride) & 3u) == 0;
    hipLaunchKernelGGL(rs_lfsr_k<MODE_ENCODE>, dim3(lfsr_grid(count, num_cu)), dim3(LFSR_WG), 0, stream, tab->lfsr, data,
                       dstride, parity, pstride, size, count, nullptr, aligned);
    return hipGetLastError();
}

extern "C" hipError_t rsk_remainder(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                    size_t pstride, uint32_t size, size_t count, uint8_t *rem, int num_cu,
                                    hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(rs_lfsr_k<MODE_REMAINDER>, dim3(lfsr_grid(count, num_cu)), dim3(LFSR_WG), 0, stream, tab->lfsr, data,
                       dstride, const_cast<uint8_t *>(parity), pstride, size, count, rem, 1);
    return hipGetLastError();
}

extern "C" hipError_t rsk_check(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                size_t pstride, uint32_t size, size_t count, uint8_t *flag, int num_cu,
                                hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(rs_lfsr_k<MODE_CHECK>, dim3(lfsr_grid(count, num_cu)), dim3(LFSR_WG), 0, stream, tab->lfsr,
                       data, dstride, const_cast<uint8_t *>(parity), pstride, size, count, flag, 1);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* Correction: one codeword per lane                                        */
/* ------------------------------------------------------------------------ */

#define CORR_WG 256

/* per-lane scratch rows in LDS, row-major [row][lane] so that a row access
 * by the whole wave is conflict-free */
#define ROW_S 0      /* 32 log-form syndromes      */
#define ROW_LAM 32   /* 33 locator coefficients    */
#define ROW_B 65     /* 33 BM correction poly (log) */
#define ROW_OM 98    /* 32 evaluator (log)          */
#define ROW_ROOT 130 /* 32 Chien roots              */
#define ROW_LOC 162  /* 32 locations                */
#define ROW_MAG 194  /* 32 magnitudes               */
#define ROWS 226

struct Lane {
    uint8_t *base;
    __device__ __forceinline__ uint32_t get(uint32_t row) const { return base[row * CORR_WG]; }
    __device__ __forceinline__ void put(uint32_t row, uint32_t v) const { base[row * CORR_WG] = (uint8_t)v; }
};

/* gf_mod of src/internal/common.h:102-110 on a value already truncated to
 * uint16 (equal to v % 255 there) */
__device__ __forceinline__ uint32_t mod255(uint32_t v) { return (v & 0xffffu) % 255u; }
/* reduce x < 510 */
__device__ __forceinline__ uint32_t red510(uint32_t x) { return x >= 255u ? x - 255u : x; }

template <typename PosT>
__device__ bool correct_one(const uint8_t *__restrict__ EXP, const uint8_t *__restrict__ LOG, const Lane &ln,
                            const RsCorrParams &P, uint8_t *data, uint8_t *parity, size_t size, uint32_t ne,
                            const PosT *pos, bool eras_apply, uint32_t &corrected)
{
    const int32_t pad = P.pad;

    /* --- erasure locator prod(1 + X_l x), src/decode.c:31-47 --- */
    ln.put(ROW_LAM + 0, 1);
    for (uint32_t i = 1; i <= RS_NR; ++i)
        ln.put(ROW_LAM + i, 0);
    if (ne > 0) {
        uint32_t t = (uint32_t)(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[0] + (uint32_t)pad)));
        ln.put(ROW_LAM + 1, EXP[mod255(t)]);
        for (uint32_t i = 1; i < ne; ++i) {
            t = (uint32_t)(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[i] + (uint32_t)pad)));
            const uint32_t xl = mod255(t);
            for (uint32_t j = i + 1; j > 0; --j) {
                const uint32_t lg = LOG[ln.get(ROW_LAM + j - 1)];
                if (lg != RS_A0)
                    ln.put(ROW_LAM + j, ln.get(ROW_LAM + j) ^ EXP[xl + lg]);
            }
        }
    }
    for (uint32_t i = 0; i <= RS_NR; ++i)
        ln.put(ROW_B + i, LOG[ln.get(ROW_LAM + i)]);

    /* --- Berlekamp-Massey, src/decode.c:53-96 --- */
    uint32_t L = ne;
    for (uint32_t r = ne + 1; r <= RS_NR; ++r) {
        uint32_t disc = 0;
        for (uint32_t i = 0; i < r; ++i) {
            const uint32_t li = ln.get(ROW_LAM + i);
            const uint32_t s = ln.get(ROW_S + r - i - 1);
            if (li != 0 && s != RS_A0)
                disc ^= EXP[LOG[li] + s];
        }
        disc = LOG[disc];
        const bool lengthen = (disc != RS_A0) && (2u * L <= r + ne - 1u);
        if (disc != RS_A0) {
            /* downward in place: T_i = lam_i + disc*B_{i-1}; B from OLD lam */
            for (uint32_t i = RS_NR; i > 0; --i) {
                const uint32_t bim1 = ln.get(ROW_B + i - 1);
                const uint32_t li = ln.get(ROW_LAM + i);
                const uint32_t t = (bim1 != RS_A0) ? EXP[disc + bim1] : 0u;
                ln.put(ROW_B + i, lengthen ? (li == 0 ? RS_A0 : red510(LOG[li] + RS_NN - disc)) : bim1);
                ln.put(ROW_LAM + i, li ^ t);
            }
            ln.put(ROW_B + 0, lengthen ? red510(LOG[ln.get(ROW_LAM + 0)] + RS_NN - disc) : RS_A0);
            if (lengthen)
                L = r + ne - L;
        } else {
            for (uint32_t i = RS_NR; i > 0; --i)
                ln.put(ROW_B + i, ln.get(ROW_B + i - 1));
            ln.put(ROW_B + 0, RS_A0);
        }
    }

    /* --- degree, log form, src/decode.c:98-110 --- */
    uint32_t deg = 0;
    uint32_t reg[RS_NR + 1];
#pragma unroll
    for (uint32_t i = 0; i <= RS_NR; ++i) {
        const uint32_t v = LOG[ln.get(ROW_LAM + i)];
        ln.put(ROW_LAM + i, v);
        reg[i] = v;
        if (v != RS_A0)
            deg = i;
    }
    if (deg == 0)
        return false;

    /* --- Chien search, src/decode.c:112-145 --- */
    uint32_t cnt = 0;
    int32_t k = (int32_t)P.iprim - 1;
    for (uint32_t i = 1; i <= RS_NN; ++i) {
        uint32_t acc = 1;
#pragma unroll
        for (uint32_t j = 1; j <= RS_NR; ++j) {
            if (j <= deg && reg[j] != RS_A0) {
                reg[j] = red510(reg[j] + j);
                acc ^= EXP[reg[j]];
            }
        }
        if (acc == 0) {
            if (k < pad)
                return false;
            ln.put(ROW_ROOT + cnt, i);
            ln.put(ROW_LOC + cnt, (uint32_t)k);
            if (++cnt == deg)
                break;
        }
        k = (int32_t)mod255((uint32_t)(k + (int32_t)P.iprim));
    }
    if (cnt != deg)
        return false;

    /* --- Omega, src/decode.c:147-158 --- */
    for (uint32_t i = 0; i < deg; ++i) {
        uint32_t acc = 0;
        for (uint32_t j = 0; j <= i; ++j) {
            const uint32_t s = ln.get(ROW_S + i - j), l = ln.get(ROW_LAM + j);
            if (s != RS_A0 && l != RS_A0)
                acc ^= EXP[s + l];
        }
        ln.put(ROW_OM + i, LOG[acc]);
    }

    /* --- Forney, src/decode.c:159-191 --- */
    corrected = 0;
    const uint32_t dtop = (deg < RS_NR - 1 ? deg : RS_NR - 1) & ~1u;
    for (uint32_t jj = 0; jj < cnt; ++jj) {
        const uint32_t root = ln.get(ROW_ROOT + jj);
        uint32_t num = 0, ir = 0; /* ir = i*root mod 255 */
        for (uint32_t i = 0; i < deg; ++i) {
            const uint32_t om = ln.get(ROW_OM + i);
            if (om != RS_A0)
                num ^= EXP[om + ir];
            ir = red510(ir + root);
        }
        if (num == 0) {
            ln.put(ROW_MAG + jj, 0);
            continue;
        }
        const uint32_t num2 = EXP[mod255((uint32_t)((int32_t)root * ((int32_t)P.fcr - 1) + (int32_t)RS_NN))];
        uint32_t den = 0;
        ir = 0;
        for (uint32_t i = 0; i <= dtop; i += 2) {
            const uint32_t l = ln.get(ROW_LAM + i + 1);
            if (l != RS_A0)
                den ^= EXP[l + ir];
            ir = red510(red510(ir + root) + root);
        }
        ln.put(ROW_MAG + jj, EXP[mod255(LOG[num] + LOG[num2] + RS_NN - LOG[den])]);
        ++corrected;
    }

    /* --- the pattern must reproduce every syndrome, src/decode.c:193-209 --- */
    for (uint32_t i = 0; i < RS_NR; ++i) {
        uint32_t acc = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t mg = ln.get(ROW_MAG + j);
            if (mg == 0)
                continue;
            const int32_t kk = (int16_t)((int32_t)(P.fcr + i) * (int32_t)P.prim * (int32_t)(RS_NN - ln.get(ROW_LOC + j) - 1u));
            acc ^= EXP[mod255((uint32_t)((int32_t)LOG[mg] + kk))];
        }
        const uint32_t s = ln.get(ROW_S + i);
        if (acc != (s == RS_A0 ? 0u : EXP[s]))
            return false;
    }

    /* --- apply, src/decode.c:211-227 --- */
    if (eras_apply) {
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t p = (uint32_t)pos[j];
            const uint8_t mg = (uint8_t)ln.get(ROW_MAG + j);
            if (p < size)
                data[p] ^= mg;
            else if (p < size + RS_NR)
                parity[p - size] ^= mg;
        }
    } else {
        for (uint32_t j = 0; j < cnt; ++j) {
            const int32_t p = (int32_t)ln.get(ROW_LOC + j) - pad;
            const uint8_t mg = (uint8_t)ln.get(ROW_MAG + j);
            if (p >= 0 && p < (int32_t)size)
                data[p] ^= mg;
            else if (p >= (int32_t)size && p < (int32_t)(size + RS_NR))
                parity[p - (int32_t)size] ^= mg;
            else
                return false;
        }
    }
    return true;
}

template <typename PosT>
__global__ __launch_bounds__(CORR_WG) void rs_correct_k(const RsDevTables *__restrict__ tab, RsCorrParams P,
                                                        uint8_t *data, size_t dstride, uint8_t *parity,
                                                        size_t pstride, size_t count,
                                                        const uint8_t *__restrict__ rem,
                                                        const uint8_t *__restrict__ ext_syn,
                                                        const PosT *__restrict__ pos, size_t pos_stride,
                                                        const uint8_t *__restrict__ cnt, uint8_t *__restrict__ ok,
                                                        uint8_t *__restrict__ corrected)
{
    __shared__ uint8_t EXP[512];
    __shared__ uint8_t LOG[256];
    __shared__ uint8_t scratch[ROWS * CORR_WG];
    for (uint32_t t = threadIdx.x; t < 512u; t += CORR_WG)
        EXP[t] = tab->exp2[t];
    LOG[threadIdx.x] = tab->log[threadIdx.x];
    __syncthreads();

    const size_t cw = (size_t)blockIdx.x * CORR_WG + threadIdx.x;
    if (cw >= count)
        return;
    const Lane ln{scratch + threadIdx.x};

    /* syndromes (log form) */
    bool any = false;
    if (ext_syn) {
        for (uint32_t i = 0; i < RS_NR; ++i) {
            const uint32_t s = ext_syn[cw * RS_NR + i];
            ln.put(ROW_S + i, s);
            any |= s != RS_A0;
        }
    } else {
        const uint4 *r4 = reinterpret_cast<const uint4 *>(rem + cw * RS_NR);
        const uint4 ra = r4[0], rb = r4[1];
        const uint32_t rw[8] = {ra.x, ra.y, ra.z, ra.w, rb.x, rb.y, rb.z, rb.w};
        if ((ra.x | ra.y | ra.z | ra.w | rb.x | rb.y | rb.z | rb.w) != 0u) {
            uint32_t s[RS_NR];
#pragma unroll
            for (uint32_t i = 0; i < RS_NR; ++i)
                s[i] = 0;
#pragma unroll
            for (uint32_t m = 0; m < RS_NR; ++m) {
                const uint32_t rm = (rw[m >> 2] >> (8 * (m & 3))) & 0xffu;
                if (rm) {
                    uint32_t e = red510(LOG[rm] + P.tr_start[m]);
                    const uint32_t inc = P.tr_inc[m];
#pragma unroll
                    for (uint32_t i = 0; i < RS_NR; ++i) {
                        s[i] ^= EXP[e];
                        e = red510(e + inc);
                    }
                }
            }
#pragma unroll
            for (uint32_t i = 0; i < RS_NR; ++i) {
                any |= s[i] != 0;
                ln.put(ROW_S + i, LOG[s[i]]);
            }
        }
    }
    uint32_t fixed = 0;
    bool good = true;
    uint8_t *d = data + cw * dstride;
    uint8_t *p = parity + cw * pstride;
    const bool eras = pos != nullptr;
    uint32_t ne = eras ? cnt[cw] : 0u;
    if (ne > RS_NR) {
        good = false; /* undefined behaviour in the reference (quirk Q5): refused */
    } else if (any) {
        good = correct_one<PosT>(EXP, LOG, ln, P, d, p, P.size, ne, eras ? pos + cw * pos_stride : nullptr, eras,
                                 fixed);
    }
    ok[cw] = good ? 1 : 0;
    if (corrected)
        corrected[cw] = (uint8_t)fixed;
}

extern "C" hipError_t rsk_correct(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride,
                                  uint8_t *parity, size_t pstride, size_t count, const uint8_t *rem,
                                  const uint8_t *ext_syn, const uint8_t *pos8, const uint32_t *pos32,
                                  size_t pos_stride, const uint8_t *cnt, uint8_t *ok, uint8_t *corrected,
                                  hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const dim3 grid((unsigned)((count + CORR_WG - 1) / CORR_WG));
    if (pos32)
        hipLaunchKernelGGL(rs_correct_k<uint32_t>, grid, dim3(CORR_WG), 0, stream, tab, *prm, data, dstride, parity,
                           pstride, count, rem, ext_syn, pos32, pos_stride, cnt, ok, corrected);
    else
        hipLaunchKernelGGL(rs_correct_k<uint8_t>, grid, dim3(CORR_WG), 0, stream, tab, *prm, data, dstride, parity,
                           pstride, count, rem, ext_syn, pos8, pos_stride, cnt, ok, corrected);
    return hipGetLastError();
}
