/*
 * rs_correct.hip -- RS(n, n-32) error/erasure correction on CDNA4 (gfx950).
 *
 * rs_correct_k: syndromes in, corrected codewords out; one codeword per lane,
 * 1024-thread persistent workgroups (one per CU).  Follows src/decode.c:17-230
 * of the reference step by step (erasure locator, Berlekamp-Massey in Karn's
 * form, Chien search, Omega, Forney, re-syndrome check, apply), with the same
 * integer semantics, so results (bytes, bool, corrected_num) are bit-exact.
 *
 * LDS (163,840 B, all of it):
 *   lsyn 32 KB   each lane's 32 log-syndromes, [row][lane] (conflict-free).
 *   lgf  64 KB   GF(256) {exp2[x], log[x & 255]} dwords, replicated 32x so
 *                lane l's ds_read_u8 always hits bank l & 31: every random
 *                table lookup is conflict-free.
 *   lch  64 KB   Chien chunk rows: term j (1..16) at 16 consecutive points for
 *                a coefficient of log e (e = 255: zero row), ds_read_b128.
 *
 * Control flow is wave-uniform: loops run to the wave's maximum degree (a
 * readfirstlane'd DPP/shuffle max) and every lane's arithmetic inside is
 * branch-free (zero coefficients contribute zero), so the LDS lookups of a
 * group of terms issue back to back instead of serialising behind per-lane
 * branches.  Roots are walked in ascending order by a divergence-free
 * "first set bit of a 256-bit map" iterator.
 *
 * The re-syndrome check (src/decode.c:193-209) is run whenever it can fail:
 * when the locator degree is below the BM length L, or when the reference's
 * int16 exponent there can overflow (large fcr*prim).  If deg(Lambda) = L and
 * Lambda has deg distinct roots, Lambda generates S_1..S_32 with distinct
 * characteristic roots, so S_k = sum_j Y_j X_j^k for every k and Forney's Y_j
 * reproduce every syndrome: the check passes by construction.
 * (RsCorrParams.force_verify runs it always; tests compare both modes.)
 */
#include <hip/hip_runtime.h>

#include "rs_device.h"

#define COR_WG 1024
#define GF_REPL 32
#define A0 RS_A0

struct Gf {
    const uint8_t *p; /* table base + (lane & 31) * 4 */
    __device__ __forceinline__ uint32_t exp(uint32_t x) const { return p[x * (GF_REPL * 4)]; }     /* x < 512 */
    __device__ __forceinline__ uint32_t log(uint32_t v) const { return p[v * (GF_REPL * 4) + 1]; } /* v < 256 */
};

/* gf_mod of src/internal/common.h:102-110 on the uint16 truncation of v */
__device__ __forceinline__ uint32_t mod255(uint32_t v) { return (v & 0xffffu) % 255u; }
/* x < 510 -> x mod 255 */
__device__ __forceinline__ uint32_t red(uint32_t x) { return x >= 255u ? x - 255u : x; }

/* Maximum of v (< 64) over the ACTIVE lanes of the wave, bit by bit from
 * ballots.  (A shuffle butterfly is wrong here: lanes that have left the
 * codeword's control flow do not forward partial maxima.) */
__device__ __forceinline__ uint32_t wave_max(uint32_t v)
{
    uint32_t m = 0;
#pragma unroll
    for (int b = 5; b >= 0; --b) {
        const uint32_t c = m | (1u << b);
        if (__ballot(v >= c) != 0ull)
            m = c;
    }
    return m;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) { return 63u - wave_max(63u - v); }

/* byte-wise zero test of 16 bytes -> 16-bit mask (bit b: byte b is zero) */
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

/* data[0] ^= v (v < 256).  COR_ATOMIC_APPLY (experiment, measured slower:
 * L2 atomic throughput): a device-scope atomic XOR of the aligned dword that
 * holds the byte, with no return value, so the wave does not wait for it. */
#ifndef COR_ATOMIC_APPLY
#define COR_ATOMIC_APPLY 0
#endif
__device__ __forceinline__ void xor_byte(uint8_t *p, uint32_t v)
{
#if COR_ATOMIC_APPLY
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    __hip_atomic_fetch_xor(reinterpret_cast<uint32_t *>(a & ~uintptr_t(3)), v << (8u * (uint32_t)(a & 3u)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
    *p ^= (uint8_t)v;
#endif
}

/* Walks a 256-bit root map over i' = i mod 255 in the reference's order:
 * i = 1..254 ascending, then i = 255 (bit 0).  No per-lane loops. */
struct RootIter {
    uint32_t w[9]; /* w[0..7]: bits of i' (bit 0 of w[0] removed), w[8]: the i = 255 bit */
    __device__ __forceinline__ void init(const uint32_t (&rb)[8])
    {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            w[k] = rb[k];
        w[8] = rb[0] & 1u;
        w[0] &= ~1u;
    }
    __device__ __forceinline__ uint32_t next()
    {
        uint32_t sel = 8, bits = w[8];
#pragma unroll
        for (int k = 7; k >= 0; --k) {
            const bool nz = w[k] != 0u;
            sel = nz ? (uint32_t)k : sel;
            bits = nz ? w[k] : bits;
        }
        const uint32_t b = __builtin_ctz(bits | 0x80000000u);
        const uint32_t clr = bits & (bits - 1u);
#pragma unroll
        for (int k = 0; k < 9; ++k)
            w[k] = (sel == (uint32_t)k) ? clr : w[k];
        return sel < 8u ? 32u * sel + b : 255u;
    }
};

template <typename PosT>
__device__ __forceinline__ bool correct_one(const Gf &gf, const uint4 *__restrict__ chien, const uint8_t *srow,
                                            const RsCorrParams &P, uint8_t *data, uint8_t *parity, uint32_t ne,
                                            const PosT *pos, uint32_t &corrected)
{
    const int32_t pad = P.pad;
    const uint32_t size = P.size;
#define SLOG(k) ((uint32_t)srow[(31u - (k)) * COR_WG]) /* log S_k */

    /* ---- erasure locator prod(1 + X_l x), src/decode.c:31-47 ---- */
    uint32_t lam[RS_NR + 1];
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i)
        lam[i] = 0;
    lam[0] = 1;
    const uint32_t nemax = wave_max(ne);
    if (nemax > 0) {
        if (ne > 0)
            lam[1] = gf.exp(mod255(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[0] + (uint32_t)pad))));
        for (uint32_t i = 1; i < nemax; ++i) { /* uniform loop; lane active while i < ne */
            const bool act = i < ne;
            const uint32_t xl =
                act ? mod255(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[i] + (uint32_t)pad))) : 0u;
#pragma unroll
            for (int g = RS_NR; g >= 1; g -= 8) {
                if ((uint32_t)(g - 7) <= i + 1) { /* uniform */
#pragma unroll
                    for (int j = g; j > g - 8; --j) {
                        const uint32_t lg = gf.log(lam[j - 1]);
                        const uint32_t t = gf.exp(xl + lg);
                        lam[j] ^= (act && (uint32_t)j <= i + 1 && lg != A0) ? t : 0u;
                    }
                }
            }
        }
    }

    /* ---- Berlekamp-Massey, src/decode.c:49-96 ----
     * dl, db: upper bounds of the nonzero indices of lam and of B (log form,
     * A0 = zero); they only bound the work, exactness comes from the
     * per-coefficient zero tests. */
    uint32_t B[RS_NR + 1];
    uint32_t dl = ne, db = ne, L = ne;
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i)
        B[i] = ((uint32_t)i <= dl) ? gf.log(lam[i]) : A0;
    for (uint32_t r = wave_min(ne) + 1u; r <= RS_NR; ++r) {
        const bool act = r > ne;
        const uint32_t ub = wave_max(act ? dl : 0u); /* <= r - 1 */
        const uint8_t *sr = srow + (RS_NR - r) * COR_WG; /* sr[i*COR_WG] = log S_(r-1-i) */
        uint32_t disc = 0;
#pragma unroll
        for (int g = 0; g < RS_NR; g += 8) {
            if ((uint32_t)g <= ub) {
#pragma unroll
                for (int i = g; i < g + 8; ++i) {
                    /* i >= r happens only inside the last group, where
                     * lam[i] == 0 for every active lane: the read (a row past
                     * this lane's 32, still inside the LDS block) is masked
                     * below, and being unconditional it issues back to back
                     * with the group's other reads */
                    const uint32_t li = lam[i];
                    const uint32_t s = (uint32_t)sr[i * COR_WG];
                    const uint32_t t = gf.exp(gf.log(li) + s);
                    disc ^= (li != 0u && s != A0) ? t : 0u;
                }
            }
        }
        disc = gf.log(disc);
        const bool upd = act && disc != A0;
        const bool lengthen = upd && (2u * L <= r + ne - 1u);
        const bool shift = act && !lengthen;
        const uint32_t up = min((uint32_t)RS_NR, max(dl, db + 1u));
        const uint32_t ub2 = wave_max(act ? up : 0u);
#pragma unroll
        for (int g = RS_NR; g >= 1; g -= 8) {
            if ((uint32_t)(g - 7) <= ub2) {
#pragma unroll
                for (int i = g; i > g - 8; --i) {
                    const uint32_t bim1 = B[i - 1], li = lam[i];
                    const uint32_t t = gf.exp(disc + bim1);
                    const uint32_t nb = li ? red(gf.log(li) + RS_NN - disc) : A0;
                    B[i] = lengthen ? nb : (shift ? bim1 : B[i]);
                    lam[i] = li ^ ((upd && bim1 != A0) ? t : 0u);
                }
            }
        }
        B[0] = lengthen ? red(RS_NN - disc) : (shift ? A0 : B[0]); /* lam[0] == 1 */
        if (act) {
            db = lengthen ? dl : min(db + 1u, (uint32_t)RS_NR);
            if (upd)
                dl = up;
            if (lengthen)
                L = r + ne - L;
        }
    }

    if (P.stop_at == 2u)
        return dl > 40u; /* profiling ablation */

    /* ---- log form and degree, src/decode.c:98-110 ---- */
    uint32_t ll[RS_NR + 1];
    uint32_t deg = 0;
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i) {
        ll[i] = ((uint32_t)i <= dl) ? gf.log(lam[i]) : A0;
        deg = (ll[i] != A0) ? (uint32_t)i : deg;
    }
    if (deg == 0)
        return false;
    const uint32_t degmax = wave_max(deg);

    /* ---- Chien search: root map over the 255 points ----
     * With num_roots erasures BM does not run (src/decode.c:55) and Lambda is
     * exactly prod(1 + X_l x): its roots are the points alpha^i with
     * i = -log X_l, so the map is built from the positions (a repeated X_l is
     * a double root that the search counts once: cnt < deg fails below, as in
     * the reference).  Other lanes search. */
    const bool direct = ne == RS_NR;
    const uint32_t degsearch = wave_max(direct ? 0u : deg);
    uint32_t rb[8];
    if (degsearch <= 16) {
        /* chunk a: points i' = 16a + b: Lambda = 1 + sum_j T_j[e_j], e_j = log(Lambda_j) + 16aj */
        uint32_t ej[17];
#pragma unroll
        for (int j = 1; j <= 16; ++j)
            ej[j] = ll[j];
#pragma unroll
        for (int a = 0; a < 16; ++a) {
            uint32_t acc[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
#pragma unroll
            for (int j = 1; j <= 16; ++j) {
                if ((uint32_t)j <= degsearch) {
                    const uint4 row = chien[(j - 1) * 256 + ej[j]];
                    acc[0] ^= row.x;
                    acc[1] ^= row.y;
                    acc[2] ^= row.z;
                    acc[3] ^= row.w;
                    ej[j] = (ej[j] == A0) ? A0 : red(ej[j] + (16u * j) % 255u);
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
                    const uint32_t rj = red(reg[j] + j);
                    const bool nz = reg[j] != A0;
                    reg[j] = nz ? rj : A0;
                    acc ^= nz ? gf.exp(rj) : 0u;
                }
                bits |= (acc == 0 ? 1u : 0u) << b;
            }
            rb[w] = bits;
        }
        uint32_t acc = 1; /* point i = 255 (alpha^0) */
#pragma unroll
        for (int j = 1; j <= RS_NR; ++j)
            acc ^= (reg[j] != A0) ? gf.exp(red(reg[j] + j)) : 0u;
        rb[0] |= (acc == 0 ? 1u : 0u);
    }
    if (wave_max(direct ? 1u : 0u)) {
        uint32_t dm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (direct) {
            for (uint32_t l = 0; l < RS_NR; ++l) {
                const uint32_t xl = mod255(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[l] + (uint32_t)pad)));
                const uint32_t ip = xl ? RS_NN - xl : 0u; /* i' = -log X_l mod 255 */
#pragma unroll
                for (int w = 0; w < 8; ++w)
                    dm[w] |= ((ip >> 5) == (uint32_t)w) ? (1u << (ip & 31u)) : 0u;
            }
        }
#pragma unroll
        for (int w = 0; w < 8; ++w)
            rb[w] = direct ? dm[w] : rb[w];
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int w = 0; w < 8; ++w)
        cnt += __popc(rb[w]);
    if (cnt != deg)
        return false; /* src/decode.c:143-145 */
    if (P.stop_at == 3u)
        return false; /* profiling ablation */

    /* locations k = (i*iprim - 1) mod 255 below pad fail, src/decode.c:132-134 */
    if (pad > 0) {
        RootIter it;
        it.init(rb);
        bool low = false;
        for (uint32_t n = 0; n < cnt; ++n) {
            const uint32_t i = it.next();
            low |= (int32_t)((i * P.iprim + 254u) % 255u) < pad;
        }
        if (low)
            return false;
    }

    /* ---- Omega = S * Lambda mod x^deg (log form), src/decode.c:147-158 ---- */
    uint32_t om[RS_NR];
#pragma unroll
    for (int m = 0; m < RS_NR; ++m) {
        om[m] = A0;
        if ((uint32_t)m < degmax) {
            uint32_t acc = 0;
#pragma unroll
            for (int j = 0; j <= m; ++j) {
                const uint32_t s = SLOG((uint32_t)(m - j)), l = ll[j];
                const uint32_t t = gf.exp(s + l);
                acc ^= (s != A0 && l != A0) ? t : 0u;
            }
            om[m] = ((uint32_t)m < deg) ? gf.log(acc) : A0;
        }
    }
    if (P.stop_at == 4u)
        return (om[0] ^ om[1]) > 300u; /* profiling ablation */
    const uint32_t dtop = (deg < RS_NR - 1 ? deg : RS_NR - 1) & ~1u;
    const uint32_t dtopmax = wave_max(dtop);
    const uint32_t cntmax = wave_max(cnt);
    /* the check can fail only if deg < L, or where the reference's int16
     * exponent (src/decode.c:201-202) overflows (then it is not the math) */
    const bool verify = P.force_verify || deg != L || !P.vfast;

    /* ---- Forney per root, src/decode.c:159-191; pass 0 = re-syndrome check
     * (only where it can fail), pass 1 = apply (src/decode.c:211-227) ---- */
    bool good = true;
    const uint32_t vwave = wave_max(verify ? 1u : 0u);
    for (uint32_t pass = vwave ? 0u : 1u; pass < 2u; ++pass) {
        const bool run = pass == 1u || verify; /* this lane does this pass */
        uint32_t V[RS_NR / 4];
#pragma unroll
        for (int q = 0; q < RS_NR / 4; ++q)
            V[q] = 0;
        RootIter it;
        it.init(rb);
        for (uint32_t n = 0; n < cntmax; ++n) {
            const bool act = run && n < cnt;
            const uint32_t i = it.next(); /* root, ascending as in the reference */
            uint32_t num = 0, ir = 0;
#pragma unroll
            for (int m = 0; m < RS_NR; ++m) {
                if ((uint32_t)m < degmax) {
                    const uint32_t t = gf.exp(om[m] + ir);
                    num ^= (om[m] != A0) ? t : 0u;
                    ir = red(ir + i);
                }
            }
            const uint32_t ln2 = mod255((uint32_t)((int32_t)i * ((int32_t)P.fcr - 1) + (int32_t)RS_NN));
            const uint32_t i2 = red(i + i);
            uint32_t den = 0;
            ir = 0;
#pragma unroll
            for (int m = 0; m < RS_NR; m += 2) {
                if ((uint32_t)m <= dtopmax) {
                    const uint32_t l = ((uint32_t)m <= dtop) ? ll[m + 1] : A0;
                    const uint32_t t = gf.exp(l + ir);
                    den ^= (l != A0) ? t : 0u;
                    ir = red(ir + i2);
                }
            }
            const uint32_t lmag = (gf.log(num) + ln2 + RS_NN - gf.log(den)) % 255u;
            const uint32_t mag = gf.exp(lmag);
            const bool nz = act && num != 0u; /* zero numerator: no correction, not counted */
            if (nz && (verify ? pass == 0u : pass == 1u)) /* counted once, before the check */
                ++corrected;
            const uint32_t k = (i * P.iprim + 254u) % 255u;
            if (pass == 1u) {
                if (nz) {
                    const uint32_t p = pos ? (uint32_t)pos[n] /* quirk Q1/Q2: slot by root ordinal */
                                           : (uint32_t)((int32_t)k - pad);
                    if (p < size)
                        xor_byte(data + p, mag);
                    else if (p < size + RS_NR)
                        xor_byte(parity + p - size, mag);
                }
            } else if (nz) {
                /* re-syndrome contribution mag * alpha^((fcr+q)*prim*(254-k)) */
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
                        const int32_t kk =
                            (int16_t)((int32_t)(P.fcr + q) * (int32_t)P.prim * (int32_t)(254u - k));
                        V[q >> 2] ^= gf.exp(mod255((uint32_t)((int32_t)lmag + kk))) << (8 * (q & 3));
                    }
                }
            }
        }
        if (pass == 0u) {
#pragma unroll
            for (int q = 0; q < RS_NR; ++q) {
                const uint32_t s = SLOG((uint32_t)q);
                V[q >> 2] ^= (s == A0 ? 0u : gf.exp(s)) << (8 * (q & 3));
            }
            bool same = true;
#pragma unroll
            for (int q = 0; q < RS_NR / 4; ++q)
                same = same && V[q] == 0u;
            if (verify && !same) {
                good = false;
                break; /* src/decode.c:206-208: nothing applied */
            }
        }
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
    /* one block, carved by hand so that the layout is known: the BM
     * discrepancy reads up to 31 rows past lsyn (masked terms), which land in
     * lgf */
    __shared__ uint4 lds[(RS_NR * COR_WG + 512 * GF_REPL * 4 + 16 * 256 * 16) / 16];
    uint8_t *lsyn = reinterpret_cast<uint8_t *>(lds);                           /* 32 KB */
    uint32_t *lgf = reinterpret_cast<uint32_t *>(lds + RS_NR * COR_WG / 16);     /* 64 KB */
    uint4 *lch = lds + (RS_NR * COR_WG + 512 * GF_REPL * 4) / 16;              /* 64 KB */
    for (uint32_t t = threadIdx.x; t < 512u * GF_REPL; t += COR_WG) {
        const uint32_t x = t / GF_REPL;
        lgf[t] = (uint32_t)T->exp2[x] | ((uint32_t)T->log[x & 255u] << 8);
    }
    for (uint32_t t = threadIdx.x; t < 16u * 256u; t += COR_WG)
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
        else if (any && P.stop_at != 1u)
            good = correct_one<PosT>(gf, lch, srow, P, data + cw * dstride, parity + cw * pstride, ne,
                                     pos ? pos + cw * pos_stride : nullptr, fixed);
        ok[cw] = good ? 1 : 0;
        if (corrected)
            corrected[cw] = (uint8_t)fixed;
    }
}

static int persistent_grid(size_t count, int wg, int num_cu)
{
    size_t need = (count + wg - 1) / wg;
    size_t g = (size_t)(num_cu > 0 ? num_cu : 256);
    return (int)(need < g ? (need ? need : 1) : g);
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
