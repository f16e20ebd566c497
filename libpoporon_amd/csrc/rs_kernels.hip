/*
 * rs_kernels.hip -- RS(n, n-32) over GF(2^8) on CDNA4 (gfx950).
 *
 * Kernels
 *   rs_lfsr_k<MODE_ENCODE>    parity = m(x) x^32 mod g(x)          (src/encode.c:120-143)
 *   rs_lfsr_k<MODE_SYNDROME>  the 32 syndromes of the received word (src/decode.c:375-415),
 *                             as S_i = r(beta_i) beta_i^-32 with r = c(x) x^32 mod g(x)
 *   rs_lfsr_k<MODE_CHECK>     the "any syndrome nonzero" flag only
 *   rs_correct_k              erasure locator, Berlekamp-Massey, Chien, Omega,
 *                             Forney, re-syndrome check, apply   (src/decode.c:17-230)
 *
 * All kernels put one codeword on one lane and are persistent over the batch
 * (one 1024-thread workgroup per CU), because their LDS tables are large:
 *
 * LFSR kernels.  The 32-byte shift register lives in 8 VGPRs.  A feedback
 * byte fb selects a 32-byte row (fb * g(x), pre-shifted) that is XORed into
 * the register after a one-byte funnel shift.  The 8 KB row table is
 * replicated 16 times in LDS (128 KB): lane l reads copy l & 15, and copy c of
 * every 16-byte half-row sits in bank slot c, so each ds_read_b128 lane group
 * (16 lanes, one per slot) is conflict-free whatever the data
 * (MI355X_MICROARCH.md, LDS).  The syndrome kernel adds 32 KB of nibble
 * tables that turn the remainder into syndromes with 128 ds_read_b128 per
 * codeword: 160 KB, the whole LDS.
 *
 * Correction kernel.  LDS holds (a) the GF(256) exp/log tables replicated 32
 * times so that lane l's ds_read_u8 always hits bank l & 31 (conflict-free
 * random lookups), (b) the Chien chunk table (16 locator terms x 255 logs x
 * 16 consecutive points, ds_read_b128), (c) each lane's 32 log-syndromes,
 * row-major [row][lane] -- 163,584 of the 163,840 bytes.  BM keeps the
 * locator and correction polynomials in VGPRs (unrolled, degree-guarded
 * loops: a block runs only when some lane of the wave needs it).
 */
#include <hip/hip_runtime.h>

#include "rs_device.h"

#define LFSR_WG 1024
#define LFSR_REPL 16

/* ------------------------------------------------------------------------ */
/* LFSR (encode / syndromes / check)                                        */
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
        const uint32_t left = n - i;
#pragma unroll
        for (uint32_t b = 0; b < 16u; ++b)
            if (b < left)
                lfsr_step(P, (m[b >> 2] >> (8u * (b & 3u))) & 0xffu, tab);
    }
}

#define MODE_ENCODE 0
#define MODE_SYNDROME 1
#define MODE_CHECK 2

template <int MODE>
__global__ __launch_bounds__(LFSR_WG) void rs_lfsr_k(const RsDevTables *__restrict__ T,
                                                      const uint8_t *__restrict__ data, size_t dstride,
                                                      uint8_t *__restrict__ parity, size_t pstride, uint32_t size,
                                                      size_t count, uint8_t *__restrict__ out, int par_aligned)
{
    __shared__ uint4 lds[512 * LFSR_REPL + (MODE == MODE_SYNDROME ? 32 * 2 * 2 * 16 : 0)];
    for (uint32_t t = threadIdx.x; t < 512u * LFSR_REPL; t += LFSR_WG)
        lds[t] = T->lfsr[t / LFSR_REPL];
    if (MODE == MODE_SYNDROME)
        for (uint32_t t = threadIdx.x; t < 32u * 2 * 2 * 16; t += LFSR_WG)
            lds[512 * LFSR_REPL + t] = T->synt[t];
    __syncthreads();
    const uint4 *tab = lds + (threadIdx.x & (LFSR_REPL - 1));
    const uint4 *synt = lds + 512 * LFSR_REPL;

    for (size_t cw = (size_t)blockIdx.x * LFSR_WG + threadIdx.x; cw < count; cw += (size_t)gridDim.x * LFSR_WG) {
        uint32_t P[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        lfsr_feed(P, data + cw * dstride, size, tab);
        if (MODE == MODE_SYNDROME) {
            lfsr_feed(P, parity + cw * pstride, RS_NR, tab);
            /* S = sum over remainder bytes m of T_m,lo[r_m & 15] ^ T_m,hi[r_m >> 4] */
            uint32_t S[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if ((P[0] | P[1] | P[2] | P[3] | P[4] | P[5] | P[6] | P[7]) != 0u) {
#pragma unroll
                for (uint32_t m = 0; m < RS_NR; ++m) {
                    const uint32_t rm = (P[m >> 2] >> (8u * (m & 3u))) & 0xffu;
                    const uint4 *t0 = synt + (m * 4u) * 16u;
                    const uint4 l0 = t0[rm & 15u], l1 = t0[16u + (rm & 15u)];
                    const uint4 h0 = t0[32u + (rm >> 4)], h1 = t0[48u + (rm >> 4)];
                    S[0] ^= l0.x ^ h0.x;
                    S[1] ^= l0.y ^ h0.y;
                    S[2] ^= l0.z ^ h0.z;
                    S[3] ^= l0.w ^ h0.w;
                    S[4] ^= l1.x ^ h1.x;
                    S[5] ^= l1.y ^ h1.y;
                    S[6] ^= l1.z ^ h1.z;
                    S[7] ^= l1.w ^ h1.w;
                }
            }
            uint4 *o = reinterpret_cast<uint4 *>(out + cw * RS_NR);
            o[0] = make_uint4(S[0], S[1], S[2], S[3]);
            o[1] = make_uint4(S[4], S[5], S[6], S[7]);
        } else if (MODE == MODE_CHECK) {
            lfsr_feed(P, parity + cw * pstride, RS_NR, tab);
            out[cw] = (P[0] | P[1] | P[2] | P[3] | P[4] | P[5] | P[6] | P[7]) != 0u;
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

static int persistent_grid(size_t count, int wg, int num_cu)
{
    size_t need = (count + wg - 1) / wg;
    size_t g = (size_t)(num_cu > 0 ? num_cu : 256);
    return (int)(need < g ? (need ? need : 1) : g);
}

extern "C" hipError_t rsk_encode(const RsDevTables *tab, const uint8_t *data, size_t dstride, uint8_t *parity,
                                 size_t pstride, uint32_t size, size_t count, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const int aligned = ((reinterpret_cast<uintptr_t>(parity) | pstride) & 3u) == 0;
    hipLaunchKernelGGL(rs_lfsr_k<MODE_ENCODE>, dim3(persistent_grid(count, LFSR_WG, num_cu)), dim3(LFSR_WG), 0,
                       stream, tab, data, dstride, parity, pstride, size, count, nullptr, aligned);
    return hipGetLastError();
}

extern "C" hipError_t rsk_syndrome(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                   size_t pstride, uint32_t size, size_t count, uint8_t *syn, int num_cu,
                                   hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(rs_lfsr_k<MODE_SYNDROME>, dim3(persistent_grid(count, LFSR_WG, num_cu)), dim3(LFSR_WG), 0,
                       stream, tab, data, dstride, const_cast<uint8_t *>(parity), pstride, size, count, syn, 1);
    return hipGetLastError();
}

extern "C" hipError_t rsk_check(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                size_t pstride, uint32_t size, size_t count, uint8_t *flag, int num_cu,
                                hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    hipLaunchKernelGGL(rs_lfsr_k<MODE_CHECK>, dim3(persistent_grid(count, LFSR_WG, num_cu)), dim3(LFSR_WG), 0,
                       stream, tab, data, dstride, const_cast<uint8_t *>(parity), pstride, size, count, flag, 1);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* Correction: one codeword per lane                                        */
/* ------------------------------------------------------------------------ */

#define COR_WG 1024
#define GF_REPL 32
#define A0 RS_A0

/* GF(256) lookups from the bank-replicated table: entry x is the dword
 * {exp2[x], log[x & 255], 0, 0} stored 32 times, copy b in bank b. */
struct Gf {
    const uint8_t *p; /* table base + (lane & 31) * 4 */
    __device__ __forceinline__ uint32_t exp(uint32_t x) const { return p[x * (GF_REPL * 4)]; }     /* x < 512 */
    __device__ __forceinline__ uint32_t log(uint32_t v) const { return p[v * (GF_REPL * 4) + 1]; } /* v < 256 */
};

/* gf_mod of src/internal/common.h:102-110 applied to the uint16 truncation of
 * v (equal to (v & 0xffff) % 255) */
__device__ __forceinline__ uint32_t mod255(uint32_t v) { return (v & 0xffffu) % 255u; }
/* reduce x < 510 modulo 255 */
__device__ __forceinline__ uint32_t red(uint32_t x) { return x >= 255u ? x - 255u : x; }

/* byte-wise zero test of 4 dwords (16 points) -> 16-bit mask, bit b = byte b is zero */
__device__ __forceinline__ uint32_t zero_bytes16(const uint32_t (&v)[4])
{
    uint32_t m = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t z = ~(((v[d] & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v[d] | 0x7F7F7F7Fu); /* bit 8b+7 */
        const uint32_t t = (z >> 7) & 0x01010101u;
        m |= ((t * 0x10204080u) >> 28) << (4 * d);
    }
    return m;
}

__device__ __forceinline__ uint32_t pick8(const uint32_t (&r)[8], uint32_t w)
{
    uint32_t v = r[0];
#pragma unroll
    for (uint32_t k = 1; k < 8; ++k)
        v = (w == k) ? r[k] : v;
    return v;
}

template <typename PosT>
__device__ __forceinline__ bool correct_one(const Gf &gf, const uint4 *__restrict__ chien, const uint8_t *srow,
                                            const RsCorrParams &P, uint8_t *data, uint8_t *parity, uint32_t ne,
                                            const PosT *pos, uint32_t &corrected)
{
    const int32_t pad = P.pad;
    const uint32_t size = P.size;
    /* srow[q * COR_WG] = log S_(31-q) */
#define SLOG(k) ((uint32_t)srow[(31u - (k)) * COR_WG])

    /* ---- erasure locator prod(1 + X_l x), src/decode.c:31-47 ---- */
    uint32_t lam[RS_NR + 1];
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i)
        lam[i] = 0;
    lam[0] = 1;
    if (ne > 0) {
        lam[1] = gf.exp(mod255(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[0] + (uint32_t)pad))));
        for (uint32_t i = 1; i < ne; ++i) {
            const uint32_t xl = mod255(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[i] + (uint32_t)pad)));
#pragma unroll
            for (int j = RS_NR; j >= 1; --j) {
                if ((uint32_t)j <= i + 1) {
                    const uint32_t lg = gf.log(lam[j - 1]);
                    if (lg != A0)
                        lam[j] ^= gf.exp(xl + lg);
                }
            }
        }
    }

    /* ---- Berlekamp-Massey, src/decode.c:49-96 ----
     * dl / db: upper bounds of the nonzero indices of lam / B (exactness is
     * kept by the per-coefficient zero tests, the bounds only skip work). */
    uint32_t B[RS_NR + 1];
    uint32_t dl = ne, db = ne, L = ne;
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i)
        B[i] = ((uint32_t)i <= dl) ? gf.log(lam[i]) : A0;
    for (uint32_t r = ne + 1; r <= RS_NR; ++r) {
        const uint8_t *sr = srow + (RS_NR - r) * COR_WG; /* sr[i*COR_WG] = log S_(r-1-i) */
        uint32_t disc = 0;
#pragma unroll
        for (int i = 0; i < RS_NR; ++i) {
            if ((uint32_t)i < r && (uint32_t)i <= dl) {
                const uint32_t li = lam[i], s = sr[i * COR_WG];
                if (li != 0 && s != A0)
                    disc ^= gf.exp(gf.log(li) + s);
            }
        }
        disc = gf.log(disc);
        if (disc != A0) {
            const bool lengthen = 2u * L <= r + ne - 1u;
            const uint32_t up = min(RS_NR, max(dl, db + 1u));
#pragma unroll
            for (int i = RS_NR; i >= 1; --i) {
                if ((uint32_t)i <= up) {
                    const uint32_t bim1 = B[i - 1], li = lam[i];
                    const uint32_t t = (bim1 != A0) ? gf.exp(disc + bim1) : 0u;
                    B[i] = lengthen ? (li ? red(gf.log(li) + RS_NN - disc) : A0) : bim1;
                    lam[i] = li ^ t;
                }
            }
            B[0] = lengthen ? red(RS_NN - disc) : A0; /* lam[0] == 1 */
            db = lengthen ? dl : min(db + 1u, (uint32_t)RS_NR);
            dl = up;
            if (lengthen)
                L = r + ne - L;
        } else {
#pragma unroll
            for (int i = RS_NR; i >= 1; --i)
                if ((uint32_t)i <= db + 1u)
                    B[i] = B[i - 1];
            B[0] = A0;
            db = min(db + 1u, (uint32_t)RS_NR);
        }
    }

    /* ---- log form and degree, src/decode.c:98-110 ---- */
    uint32_t ll[RS_NR + 1]; /* log lambda */
    uint32_t deg = 0;
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i) {
        ll[i] = ((uint32_t)i <= dl) ? gf.log(lam[i]) : A0;
        if (ll[i] != A0)
            deg = i;
    }
    if (deg == 0)
        return false;

    /* ---- Chien search over all 255 points -> root bitmap over i' = i mod 255 ---- */
    uint32_t rb[8];
    if (deg <= 16) {
        /* chunk a holds points i' = 16a + b, b = 0..15: lambda = 1 + sum_j T_j[e_j] */
        uint32_t ej[17];
#pragma unroll
        for (int j = 1; j <= 16; ++j)
            ej[j] = ll[j];
#pragma unroll
        for (int a = 0; a < 16; ++a) {
            uint32_t acc[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
#pragma unroll
            for (int j = 1; j <= 16; ++j) {
                if (ej[j] != A0) {
                    const uint4 row = chien[(j - 1) * 255 + ej[j]];
                    acc[0] ^= row.x;
                    acc[1] ^= row.y;
                    acc[2] ^= row.z;
                    acc[3] ^= row.w;
                    ej[j] = red(ej[j] + (16u * j) % 255u);
                }
            }
            const uint32_t m16 = zero_bytes16(acc);
            if (a & 1)
                rb[a >> 1] |= m16 << 16;
            else
                rb[a >> 1] = m16;
        }
        rb[7] &= 0x7FFFFFFFu; /* i' = 255 repeats i' = 0 */
    } else {
        /* Karn's register form, src/decode.c:117-141 (beyond-capacity locators) */
        uint32_t reg[RS_NR + 1];
#pragma unroll
        for (int j = 1; j <= RS_NR; ++j)
            reg[j] = ll[j];
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            uint32_t bits = 0;
            for (uint32_t b = (w == 0 ? 1u : 0u); b < 32u; ++b) {
                if (w == 7 && b == 31u)
                    break;
                uint32_t acc = 1;
#pragma unroll
                for (int j = 1; j <= RS_NR; ++j) {
                    if (reg[j] != A0) {
                        reg[j] = red(reg[j] + j);
                        acc ^= gf.exp(reg[j]);
                    }
                }
                bits |= (acc == 0 ? 1u : 0u) << b;
            }
            rb[w] = bits;
        }
        /* point i = 255 (alpha^0) */
        uint32_t acc = 1;
#pragma unroll
        for (int j = 1; j <= RS_NR; ++j)
            if (reg[j] != A0)
                acc ^= gf.exp(red(reg[j] + j));
        rb[0] |= (acc == 0 ? 1u : 0u);
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w)
        cnt += __popc(rb[w]);
    if (cnt != deg)
        return false; /* src/decode.c:143-145 */

    /* root i (1..255) -> location k = (i*iprim - 1) mod 255 (src/decode.c:117-118) */
    if (pad > 0) {
        for (uint32_t w = 0; w < 9; ++w) {
            uint32_t bits = w < 8 ? pick8(rb, w) : (rb[0] & 1u);
            if (w == 0)
                bits &= ~1u;
            const uint32_t base = w < 8 ? 32u * w : 255u;
            while (bits) {
                const uint32_t i = base + __builtin_ctz(bits);
                bits &= bits - 1u;
                if ((int32_t)((i * P.iprim + 254u) % 255u) < pad)
                    return false; /* src/decode.c:132-134 */
            }
        }
    }

    /* ---- Omega = S * Lambda mod x^deg (log form), src/decode.c:147-158 ---- */
    uint32_t om[RS_NR];
#pragma unroll
    for (int m = 0; m < RS_NR; ++m) {
        om[m] = A0;
        if ((uint32_t)m < deg) {
            uint32_t acc = 0;
#pragma unroll
            for (int j = 0; j <= m; ++j) {
                const uint32_t s = SLOG((uint32_t)(m - j)), l = ll[j];
                if (s != A0 && l != A0)
                    acc ^= gf.exp(s + l);
            }
            om[m] = gf.log(acc);
        }
    }
    const uint32_t dtop = (deg < RS_NR - 1 ? deg : RS_NR - 1) & ~1u;

    /* ---- Forney per root + apply + re-syndrome accumulation ----
     * Corrections are applied as they are computed; if the re-syndrome check
     * fails, a second pass XORs the same magnitudes again (undo), so a failed
     * decode leaves data/parity untouched as in src/decode.c:206-208. */
    bool good = true;
    for (uint32_t pass = 0; pass < 2; ++pass) {
        uint32_t V[RS_NR / 4]; /* re-syndromes, 4 bytes per dword */
#pragma unroll
        for (int q = 0; q < RS_NR / 4; ++q)
            V[q] = 0;
        uint32_t nth = 0;
        for (uint32_t w = 0; w < 9; ++w) {
            uint32_t bits = w < 8 ? pick8(rb, w) : (rb[0] & 1u);
            if (w == 0)
                bits &= ~1u;
            const uint32_t base = w < 8 ? 32u * w : 255u;
            while (bits) {
                const uint32_t i = base + __builtin_ctz(bits); /* root, ascending as in the reference */
                bits &= bits - 1u;
                const uint32_t slot = nth++;
                uint32_t num = 0, ir = 0;
#pragma unroll
                for (int m = 0; m < RS_NR; ++m) {
                    if ((uint32_t)m < deg) {
                        if (om[m] != A0)
                            num ^= gf.exp(om[m] + ir);
                        ir = red(ir + i);
                    }
                }
                if (num == 0)
                    continue; /* magnitude 0: not counted, not applied (src/decode.c:170-173) */
                const uint32_t ln2 = mod255((uint32_t)((int32_t)i * ((int32_t)P.fcr - 1) + (int32_t)RS_NN));
                const uint32_t i2 = red(i + i);
                uint32_t den = 0;
                ir = 0;
#pragma unroll
                for (int m = 0; m < RS_NR; m += 2) {
                    if ((uint32_t)m <= dtop) {
                        const uint32_t l = ll[m + 1];
                        if (l != A0)
                            den ^= gf.exp(l + ir);
                        ir = red(ir + i2);
                    }
                }
                const uint32_t lmag = (gf.log(num) + ln2 + RS_NN - gf.log(den)) % 255u;
                const uint8_t mag = (uint8_t)gf.exp(lmag);
                if (pass == 0)
                    ++corrected;
                const uint32_t k = (i * P.iprim + 254u) % 255u;
                /* apply: src/decode.c:211-227 */
                uint32_t p;
                if (pos) {
                    p = (uint32_t)pos[slot]; /* quirk Q1/Q2: list slot by root ordinal */
                } else {
                    p = (uint32_t)((int32_t)k - pad);
                }
                if (p < size)
                    data[p] ^= mag;
                else if (p < size + RS_NR)
                    parity[p - size] ^= mag;
                if (pass == 1)
                    continue;
                /* re-syndrome contribution: mag * alpha^((fcr+q)*prim*(254-k)) */
                if (P.vfast) {
                    uint32_t e = (lmag + P.fcr * P.prim * (254u - k)) % 255u;
                    const uint32_t st = (P.prim * (254u - k)) % 255u;
#pragma unroll
                    for (int q = 0; q < RS_NR; ++q) {
                        V[q >> 2] ^= gf.exp(e) << (8 * (q & 3));
                        e = red(e + st);
                    }
                } else {
#pragma unroll
                    for (int q = 0; q < RS_NR; ++q) {
                        const int32_t kk = (int16_t)((int32_t)(P.fcr + q) * (int32_t)P.prim * (int32_t)(254u - k));
                        V[q >> 2] ^= gf.exp(mod255((uint32_t)((int32_t)lmag + kk))) << (8 * (q & 3));
                    }
                }
            }
        }
        if (pass == 1)
            break;
#pragma unroll
        for (int q = 0; q < RS_NR; ++q) {
            const uint32_t s = SLOG((uint32_t)q);
            V[q >> 2] ^= (s == A0 ? 0u : gf.exp(s)) << (8 * (q & 3));
        }
#pragma unroll
        for (int q = 0; q < RS_NR / 4; ++q)
            good = good && V[q] == 0u;
        if (good)
            break; /* else: second pass undoes the applied corrections */
    }
#undef SLOG
    return good;
}

template <typename PosT>
__global__ __launch_bounds__(COR_WG) void rs_correct_k(const RsDevTables *__restrict__ T, RsCorrParams P,
                                                       uint8_t *data, size_t dstride, uint8_t *parity, size_t pstride,
                                                       size_t count, const uint8_t *__restrict__ syn, int syn_is_log,
                                                       const PosT *__restrict__ pos, size_t pos_stride,
                                                       const uint8_t *__restrict__ cnt, uint8_t *__restrict__ ok,
                                                       uint8_t *__restrict__ corrected)
{
    __shared__ uint32_t lgf[512 * GF_REPL];    /* 64 KB */
    __shared__ uint4 lch[16 * 255];            /* 65,280 B */
    __shared__ uint8_t lsyn[RS_NR * COR_WG];   /* 32 KB */
    for (uint32_t t = threadIdx.x; t < 512u * GF_REPL; t += COR_WG) {
        const uint32_t x = t / GF_REPL;
        lgf[t] = (uint32_t)T->exp2[x] | ((uint32_t)T->log[x & 255u] << 8);
    }
    for (uint32_t t = threadIdx.x; t < 16u * 255u; t += COR_WG)
        lch[t] = T->chien[t];
    __syncthreads();
    const Gf gf{reinterpret_cast<const uint8_t *>(lgf) + (threadIdx.x & (GF_REPL - 1)) * 4};
    uint8_t *srow = lsyn + threadIdx.x;

    for (size_t cw = (size_t)blockIdx.x * COR_WG + threadIdx.x; cw < count; cw += (size_t)gridDim.x * COR_WG) {
        const uint4 *s4 = reinterpret_cast<const uint4 *>(syn + cw * RS_NR);
        const uint4 sa = s4[0], sb = s4[1];
        const uint32_t sw[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
        bool any = false;
#pragma unroll
        for (uint32_t q = 0; q < RS_NR; ++q) {
            const uint32_t v = (sw[q >> 2] >> (8u * (q & 3u))) & 0xffu;
            const uint32_t lv = syn_is_log ? v : gf.log(v);
            any |= lv != A0;
            srow[(31u - q) * COR_WG] = (uint8_t)lv;
        }
        uint32_t fixed = 0;
        bool good = true;
        const uint32_t ne = pos ? cnt[cw] : 0u;
        if (ne > RS_NR)
            good = false; /* undefined behaviour in the reference (quirk Q5): refused */
        else if (any)
            good = correct_one<PosT>(gf, lch, srow, P, data + cw * dstride, parity + cw * pstride, ne,
                                     pos ? pos + cw * pos_stride : nullptr, fixed);
        ok[cw] = good ? 1 : 0;
        if (corrected)
            corrected[cw] = (uint8_t)fixed;
    }
}

extern "C" hipError_t rsk_correct(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride,
                                  uint8_t *parity, size_t pstride, size_t count, const uint8_t *syn, int syn_is_log,
                                  const uint8_t *pos8, const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt,
                                  uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const dim3 grid(persistent_grid(count, COR_WG, num_cu));
    if (pos32)
        hipLaunchKernelGGL(rs_correct_k<uint32_t>, grid, dim3(COR_WG), 0, stream, tab, *prm, data, dstride, parity,
                           pstride, count, syn, syn_is_log, pos32, pos_stride, cnt, ok, corrected);
    else
        hipLaunchKernelGGL(rs_correct_k<uint8_t>, grid, dim3(COR_WG), 0, stream, tab, *prm, data, dstride, parity,
                           pstride, count, syn, syn_is_log, pos8, pos_stride, cnt, ok, corrected);
    return hipGetLastError();
}
