/*
 * rs_correct.hip -- RS(n, n-32) error/erasure correction on CDNA4 (gfx950).
 *
 * rs_correct_k: syndromes in, corrected codewords out; one codeword per lane,
 * 1024-thread persistent workgroups (one per CU).  Follows src/decode.c:17-230
 * of the reference step by step (erasure locator, Berlekamp-Massey in Karn's
 * form, Omega, Chien search, Forney, re-syndrome check, apply), with the same
 * integer semantics, so results (bytes, bool, corrected_num) are bit-exact.
 *
 * LDS (163,840 B, all of it; the order matters):
 *   lsyn [0, 32K)     each lane's 32 log-syndromes (byte, 255 = zero),
 *                     [row][lane]: conflict-free.
 *   lch  [32K, 96K)   Chien chunk rows: term j (1..16) at 16 consecutive
 *                     points for a coefficient of log e (e = 255: zero row),
 *                     ds_read_b128.
 *   lgf  [96K, 160K)  GF(256) dwords {exp2[x] (byte 0), log16[x & 255]
 *                     (bytes 2-3)}, x < 512, replicated 32x so that lane l's
 *                     reads always hit bank l & 31 (conflict-free).
 *
 * Zero sentinel.  In registers the log of zero is ZL = 1024 (or 511, as
 * returned by the log table), and every valid log is reduced (< 255).  A
 * product is exp(a + b): with both logs valid a + b <= 508 indexes lgf; with
 * either one a zero the index is >= 511, where exp2[511] = 0 or the address
 * lies past the end of the workgroup's LDS allocation, where gfx950 returns 0
 * (probed: tools/probes/lds_oob.hip, profiles/r01_lds_oob_probe.log).  So GF
 * multiply-accumulate needs no zero tests.
 *
 * Scaled logs.  The log table holds 128 log v (0xFFFF for zero): 128 is the
 * stride of the replicated table, so exp(a + b) of scaled logs is the byte at
 * p + a + b (one v_add3).  Berlekamp-Massey keeps its logs in "address form"
 * a = 128 log + p (p = this lane's exp byte of entry 0): exp(a) is one
 * ds_read_u8 at a, exp(a + s) one add; the zero 0xFFFF + p lies past the
 * allocation end because lgf starts at 96K + 1.
 *
 * Control flow is wave-uniform: loops run to the wave's maximum degree (a
 * ballot-based max over the active lanes) in groups of 4 terms; inside a
 * group every lane's arithmetic is branch-free, so a group's LDS lookups
 * issue back to back.  Roots are walked in ascending order by a
 * divergence-free "first set bit of a 256-bit map" iterator.
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

#include <algorithm>
#include <type_traits>

#include "rs_device.h"
#include "rs_lane.h"

#define COR_WG 1024
#define GF_REPL 32
#define A0 RS_A0
#define BM_DISC_G 8 /* BM discrepancy terms per branch-free group */
#define FORNEY_R 4  /* Forney/apply: roots per step (their sums and byte loads overlap) */
#define ZL 1024u         /* log of zero (registers): exp(ZL + anything) reads past the LDS block -> 0 */
#define BIG 0x10000000u  /* log of zero in the Chien index walk (survives 255 reductions, clamped to 255) */

#define LDS_SYN 0u
#define LDS_CH (RS_NR * COR_WG)
#define LDS_GF (LDS_CH + 16u * 256u * 16u)
#define LDS_END (LDS_GF + 512u * GF_REPL * 4u)
static_assert(LDS_END == 163840u, "lgf must end exactly at the end of the 160 KiB LDS allocation");

struct Gf {
    uint32_t pa; /* LDS byte address of this lane's copy of the exp byte of entry 0: lgf + (lane & 31) * 4 + 1 */
    /* alpha^x for x < 511; 0 for x >= 511 (exp2[511] = 0, past it the allocation ends) -- x < 2^24 */
    __device__ __forceinline__ uint32_t exp(uint32_t x) const { return lds8(pa + x * (GF_REPL * 4)); }
    /* scaled log of v < 256: 128 log v, 0xFFFF for v = 0 */
    __device__ __forceinline__ uint32_t logs(uint32_t v) const { return lds16(pa + v * (GF_REPL * 4) + 1); }
    /* log of v < 256; 511 for v = 0 (exp of 511 + anything is 0) */
    __device__ __forceinline__ uint32_t log(uint32_t v) const { return logs(v) >> 7; }
    /* "address-form" logs (BM): a = 128 log v + pa, zero = 0xFFFF + pa: the
     * exp byte of a plus a scaled log s is at LDS byte a + s */
    __device__ __forceinline__ uint32_t expa(uint32_t a) const { return lds8(a); }
    /* the base of address-form logs */
    __device__ __forceinline__ uint32_t pofs() const { return pa; }
};

template <typename PosT, bool ERA, bool REC>
__device__ __forceinline__ bool correct_one(const Gf &gf, const uint4 *__restrict__ chien, const uint8_t *srow,
                                            const RsCorrParams &P, uint8_t *data, uint8_t *parity, uint32_t ne,
                                            const PosT *pos, uint8_t *recp, uint32_t &corrected)
{
    const int32_t pad = P.pad;
    const uint32_t size = P.size;
#define SLOG(k) conv((uint32_t)srow[(31u - (k)) * COR_WG]) /* register log of S_k */

    /* ---- erasure locator prod(1 + X_l x), src/decode.c:31-47 ----
     * lam[j] ^= X_l * lam[j-1]: terms past the current degree multiply a
     * zero (log ZL), lanes past their erasure count use X_l = zero. */
    uint32_t lam[RS_NR + 1];
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i)
        lam[i] = 0;
    lam[0] = 1;
    const uint32_t nemax = ERA ? wave_max_full(ne) : 0u; /* error mode: no erasure locator */
    for (uint32_t i = 0; i < nemax; ++i) { /* uniform */
        const uint32_t xl = i < ne ? mod255(P.prim * (uint32_t)(RS_NN - 1u - ((uint32_t)pos[i] + (uint32_t)pad))) : ZL;
#pragma unroll
        for (int g = RS_NR; g >= 1; g -= 4) {
            if ((uint32_t)(g - 3) <= i + 1) { /* uniform */
#pragma unroll
                for (int j = g; j > g - 4; --j)
                    lam[j] ^= gf.exp(xl + gf.log(lam[j - 1]));
            }
        }
    }

    /* ---- Berlekamp-Massey, src/decode.c:49-96 ----
     * Massey's form of the reference's (Karn's) iteration: B is kept
     * unnormalised (a copy of an earlier Lambda, shifted) together with the
     * discrepancy b it was taken at, and the update multiplies by disc / b:
     *   Lambda += (disc / b) x B,   B <- Lambda (b <- disc) or x B.
     * Karn's normalised B is B / b, so every product -- and every result --
     * is the same field element as the reference's.  Lambda lives only in
     * address-form logs al[] (its coefficients are re-read from exp), B in
     * bl[] (same form), so the whole state is 2 x 33 VGPRs:
     *   coefficient update  exp(dq + b_(i-1)) ^ exp(al_i) -> log   (3 lookups)
     *   discrepancy term    exp(al_i + s_(r-1-i))                  (1 lookup)
     * dl, db: upper bounds of the nonzero indices of Lambda and of B; they
     * only bound the work (zero coefficients contribute zero). */
    const uint32_t pofs = gf.pofs(); /* LDS byte address of this lane's exp(0) */
    const uint32_t AZ = pofs + 0xFFFFu;                /* address-form zero */
    uint32_t al[RS_NR + 1], bl[RS_NR + 1];
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i) {
        al[i] = (uint32_t)i <= nemax ? gf.logs(lam[i]) + pofs : AZ;
        bl[i] = al[i];
    }
    uint32_t dl = ne, db = ne, L = ne;
    uint32_t lb = 0; /* scaled log of b (b = 1) */
    /* syndrome window: W entry i (u16 halves: entry 2k low, 2k+1 high) =
     * scaled log of S_(r-1-i), 0xFFFF (zero) where r-1-i < 0; one entry
     * shifts in per iteration, so the discrepancy terms read registers */
    uint32_t W[RS_NR / 2];
#pragma unroll
    for (int k = 0; k < RS_NR / 2; ++k)
        W[k] = 0xFFFFFFFFu;
    const uint32_t r0 = (ERA ? 63u - wave_max_full(63u - ne) : 0u) + 1u;
    uint32_t ubp = 0;
    /* window for step r: S_(r-1) shifted in at the end of step r-1, after
     * the update (at the head of a step it would compete with the first
     * discrepancy group for registers and serialise its lookups) */
    auto shift_in = [&](uint32_t r) __attribute__((always_inline)) {
#pragma unroll
        for (int k = RS_NR / 2 - 1; k > 0; --k)
            W[k] = __builtin_amdgcn_alignbyte(W[k], W[k - 1], 2);
        const uint32_t s8 = srow[(RS_NR - r) * COR_WG]; /* S_(r-1), byte log (255 = zero) */
        W[0] = (W[0] << 16) | (s8 == 255u ? 0xFFFFu : s8 << 7);
    };
    shift_in(1);
    for (uint32_t r = 1; r <= RS_NR; ++r) {
        if (r < r0) { /* uniform: before the first codeword's BM step (erasure mode) */
            if (r < RS_NR)
                shift_in(r + 1);
            continue;
        }
        const bool act = r > ne;
        /* error mode: every lane is active from r = 1, and dl only grows to
         * the previous step's `up`, so the previous step's bound serves */
        const uint32_t ub = (ERA || r == r0) ? wave_max_full(act ? dl : 0u) : ubp; /* <= r - 1 */
        uint32_t disc = 0;
#pragma unroll
        for (int g = 0; g < RS_NR; g += BM_DISC_G) {
            if ((uint32_t)g <= ub) {
#pragma unroll
                for (int i = g; i < g + BM_DISC_G; ++i)
                    disc ^= gf.expa(al[i] + half(W, i)); /* i >= r: window zero */
            }
        }
        const uint32_t ld = gf.logs(disc);
        const bool upd = act && disc != 0u;
        const bool lengthen = upd && (2u * L <= r + ne - 1u);
        /* scaled log of disc / b; past the allocation where nothing is updated */
        const int32_t dd = (int32_t)ld - (int32_t)lb;
        const uint32_t dq = upd ? (uint32_t)(dd < 0 ? dd + 255 * 128 : dd) : (ZL << 7);
        const uint32_t up = min((uint32_t)RS_NR, max(dl, db + 1u));
        const uint32_t ub2 = wave_max_full(act ? up : 0u);
        ubp = ub2;
        /* coefficients top down (index i reads the old bl[i-1] before it is
         * rewritten); groups of 4 share a uniform bound test */
#pragma unroll
        for (int g = RS_NR; g >= 0; g -= 4) {
            if ((uint32_t)max(g - 3, 0) <= ub2) {
#pragma unroll
                for (int i = g; i > g - 4 && i >= 0; --i) {
                    const uint32_t old = al[i];
                    if (i > 0) {
                        const uint32_t v = gf.expa(old) ^ gf.expa(dq + bl[i - 1]);
                        al[i] = gf.logs(v) + pofs;
                        bl[i] = lengthen ? old : (ERA ? (act ? bl[i - 1] : bl[i]) : bl[i - 1]);
                    } else {
                        bl[0] = lengthen ? old : (ERA ? (act ? AZ : bl[0]) : AZ);
                    }
                }
            }
        }
        if (act) {
            db = lengthen ? dl : min(db + 1u, (uint32_t)RS_NR);
            if (upd)
                dl = up;
            if (lengthen) {
                L = r + ne - L;
                lb = ld;
            }
        }
        if (r < RS_NR)
            shift_in(r + 1);
    }
    uint32_t ll[RS_NR + 1];
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i) {
        const uint32_t l = (al[i] - pofs) >> 7;
        ll[i] = l < 255u ? l : ZL;
    }

    /* ---- degree, src/decode.c:98-110 ---- */
    uint32_t deg = 0;
#pragma unroll
    for (int i = 0; i <= RS_NR; ++i)
        deg = ll[i] < ZL ? (uint32_t)i : deg;
    if (deg == 0)
        return false;
    const uint32_t degmax = wave_max(deg);

    /* ---- Omega = S * Lambda mod x^deg (log form), src/decode.c:147-158 ----
     * (computed before the Chien search: it needs only Lambda and S); logs
     * packed two per register like BM's */
    uint32_t omp[RS_NR / 2];
    /* DM > 0: the wave's maximum degree is DM (compile time: the syndromes
     * are read once and the products of all terms interleave, no guards) */
    auto omega = [&](auto dmc) __attribute__((always_inline)) {
        constexpr int DM = decltype(dmc)::value;
        uint32_t sl[DM > 0 ? DM : 1];
        if constexpr (DM > 0) {
#pragma unroll
            for (int k = 0; k < DM; ++k)
                sl[k] = SLOG((uint32_t)k);
        }
#pragma unroll
        for (int m = 0; m < RS_NR; ++m) {
            uint32_t o = ZL;
            if (DM ? m < DM : (uint32_t)m < degmax) {
                uint32_t acc = 0;
#pragma unroll
                for (int j = 0; j <= m; ++j)
                    acc ^= gf.exp((DM ? sl[DM ? m - j : 0] : SLOG((uint32_t)(m - j))) + ll[j]);
                o = (uint32_t)m < deg ? gf.log(acc) : ZL;
            }
            if (m & 1)
                omp[m >> 1] |= o << 16;
            else
                omp[m >> 1] = o;
        }
    };
    if (degmax == 16u)
        omega(std::integral_constant<int, 16>{});
    else
        omega(std::integral_constant<int, 0>{});
#define OMLOG(m) (((m) & 1) ? (omp[(m) >> 1] >> 16) : (omp[(m) >> 1] & 0xffffu))
    /* derivative terms (Forney, below): Lambda_(2h+1) for 2h <= min(deg, 31) (src/decode.c:176-180);
     * those with 2h + 1 > deg are zero, so the terms stop at 2h <= deg - 1
     * (16 errors: 8 terms, and Forney's powers stop at m < 16, not 17) */
    const uint32_t dtop = (deg - 1u < RS_NR - 1 ? deg - 1u : RS_NR - 1) & ~1u;
    const uint32_t dtopmax = wave_max(dtop);
    uint32_t loddp[RS_NR / 4]; /* packed like omp: h = 2q (low), 2q+1 (high) */
#pragma unroll
    for (int q = 0; q < RS_NR / 4; ++q) {
        const uint32_t lo = (uint32_t)(4 * q) <= dtop ? ll[4 * q + 1] : ZL;
        const uint32_t hi = (uint32_t)(4 * q + 2) <= dtop ? ll[4 * q + 3] : ZL;
        loddp[q] = lo | (hi << 16);
    }
#define LODD(h) (((h) & 1) ? (loddp[(h) >> 1] >> 16) : (loddp[(h) >> 1] & 0xffffu))
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
        /* chunk a: points i' = 16a + b: Lambda = 1 + sum_j T_j[e_j], e_j = log(Lambda_j) + 16aj.
         * A rolled loop over chunk pairs (a = 2w, 2w+1): its body stays small
         * (instruction cache, registers); the 32-bit map words come out in
         * order and shift through rb. */
        uint32_t ej[17];
#pragma unroll
        for (int j = 1; j <= 16; ++j)
            ej[j] = ll[j] < ZL ? ll[j] : BIG;
        /* DS > 0: every lane's degree bound is DS (compile time, no guards;
         * the 16-error case: 0.462 -> 0.433 ms) */
        auto chunks = [&](auto dsc) __attribute__((always_inline)) {
        constexpr int DS = decltype(dsc)::value;
#pragma unroll 1
        for (int w = 0; w < 8; ++w) {
            uint32_t word = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t acc[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
#pragma unroll
                for (int j = 1; j <= 16; j += 2) {
                    if (DS ? j <= DS : (uint32_t)j <= degsearch) {
                        const uint4 r1 = chien[(j - 1) * 256 + min(ej[j], A0)];
                        ej[j] = red(ej[j] + (16u * j) % 255u);
                        if (DS ? j + 1 <= DS : (uint32_t)j + 1u <= degsearch) {
                            const uint4 r2 = chien[j * 256 + min(ej[j + 1], A0)];
                            ej[j + 1] = red(ej[j + 1] + (16u * (j + 1)) % 255u);
                            acc[0] = xor3(acc[0], r1.x, r2.x);
                            acc[1] = xor3(acc[1], r1.y, r2.y);
                            acc[2] = xor3(acc[2], r1.z, r2.z);
                            acc[3] = xor3(acc[3], r1.w, r2.w);
                        } else {
                            acc[0] ^= r1.x;
                            acc[1] ^= r1.y;
                            acc[2] ^= r1.z;
                            acc[3] ^= r1.w;
                        }
                    }
                }
                word |= zero_bytes16(acc) << (16 * h);
            }
#pragma unroll
            for (int q = 0; q < 7; ++q)
                rb[q] = rb[q + 1];
            rb[7] = word;
        }
        };
        if (degsearch == 16u)
            chunks(std::integral_constant<int, 16>{});
        else
            chunks(std::integral_constant<int, 0>{});
        rb[7] &= 0x7FFFFFFFu; /* i' = 255 repeats i' = 0 */
    } else {
        /* Karn's register form, src/decode.c:117-141 (beyond-capacity locators) */
        uint32_t reg[RS_NR + 1];
#pragma unroll
        for (int j = 1; j <= RS_NR; ++j)
            reg[j] = ll[j] < ZL ? ll[j] : BIG;
#pragma unroll
        for (int w = 0; w < 8; ++w) {
            uint32_t bits = 0;
            for (uint32_t b = (w == 0 ? 1u : 0u); b < 32u; ++b) {
                if (w == 7 && b == 31u)
                    break;
                uint32_t acc = 1;
#pragma unroll
                for (int j = 1; j <= RS_NR; ++j) {
                    reg[j] = red(reg[j] + j);
                    acc ^= gf.exp(min(reg[j], 511u)); /* exp2[511] = 0 */
                }
                bits |= (acc == 0 ? 1u : 0u) << b;
            }
            rb[w] = bits;
        }
        uint32_t acc = 1; /* point i = 255 (alpha^0) */
#pragma unroll
        for (int j = 1; j <= RS_NR; ++j)
            acc ^= gf.exp(min(red(reg[j] + j), 511u));
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

    const uint32_t nir = max(degmax, dtopmax + 1u); /* powers i*m needed: m < nir */
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
        /* Forney sums of root i: num = sum_m Omega_m a^(i m), den = sum_h
         * Lambda_(2h+1) a^(2h i), a^(i m) as two interleaved chains of logs
         * (even / odd m); returns num, sets lmag = log of the magnitude */
        auto forney = [&](uint32_t i, uint32_t &lmag) __attribute__((always_inline)) {
            const uint32_t i1 = i == 255u ? 0u : i;
            const uint32_t i2 = red(i1 + i1);
            uint32_t ie = 0, io = i1, num = 0, den = 0;
#pragma unroll
            for (int m0 = 0; m0 < RS_NR; m0 += 4) {
                /* groups of 4 powers (one basic block: 6 lookups together);
                 * terms past deg / dtop have log ZL and add 0 */
                if ((uint32_t)m0 < nir) {
#pragma unroll
                    for (int m = m0; m < m0 + 4; m += 2) {
                        num ^= gf.exp(OMLOG(m) + ie);
                        den ^= gf.exp(LODD(m >> 1) + ie);
                        num ^= gf.exp(OMLOG(m + 1) + io);
                        ie = red(ie + i2);
                        io = red(io + i2);
                    }
                }
            }
            const uint32_t ln2 = mod255((uint32_t)((int32_t)i * ((int32_t)P.fcr - 1) + (int32_t)RS_NN));
            const uint32_t lden = min(gf.log(den), A0); /* log 0 = A0 in the reference: no den = 0 guard */
            lmag = (min(gf.log(num), A0) + ln2 + RS_NN - lden) % 255u;
            return num;
        };
        /* the same for FORNEY_R roots at once, group-major: one bound test
         * per group of powers for all the roots, whose lookups share the block */
        auto forney_r = [&](const uint32_t (&ir)[FORNEY_R], uint32_t (&lm)[FORNEY_R], uint32_t (&nm)[FORNEY_R])
                            __attribute__((always_inline)) {
            uint32_t i2[FORNEY_R], ie[FORNEY_R], io[FORNEY_R], den[FORNEY_R];
#pragma unroll
            for (int t = 0; t < FORNEY_R; ++t) {
                const uint32_t i1 = ir[t] == 255u ? 0u : ir[t];
                i2[t] = red(i1 + i1);
                ie[t] = 0;
                io[t] = i1;
                nm[t] = 0;
                den[t] = 0;
            }
#pragma unroll
            for (int m0 = 0; m0 < RS_NR; m0 += 4) {
                if ((uint32_t)m0 < nir) {
#pragma unroll
                    for (int m = m0; m < m0 + 4; m += 2) {
#pragma unroll
                        for (int t = 0; t < FORNEY_R; ++t) {
                            nm[t] ^= gf.exp(OMLOG(m) + ie[t]);
                            den[t] ^= gf.exp(LODD(m >> 1) + ie[t]);
                            nm[t] ^= gf.exp(OMLOG(m + 1) + io[t]);
                            ie[t] = red(ie[t] + i2[t]);
                            io[t] = red(io[t] + i2[t]);
                        }
                    }
                }
            }
#pragma unroll
            for (int t = 0; t < FORNEY_R; ++t) {
                const uint32_t ln2 = mod255((uint32_t)((int32_t)ir[t] * ((int32_t)P.fcr - 1) + (int32_t)RS_NN));
                const uint32_t lden = min(gf.log(den[t]), A0);
                lm[t] = (min(gf.log(nm[t]), A0) + ln2 + RS_NN - lden) % 255u;
            }
        };
        auto target = [&](uint32_t p) __attribute__((always_inline)) {
            return p < size ? data + p : (p < size + RS_NR ? parity + (p - size) : data);
        };
        if (pass == 1u && REC) {
            if constexpr (ERA && REC) {
                /* record mode (the split erasure decode): the magnitudes go to
                 * this codeword's 64-byte record -- 32 slot positions (clamped
                 * to 255), 32 magnitudes (0: nothing to apply) -- and rs_apply_k
                 * XORs them in (a zero numerator corrects nothing and is not
                 * counted; repeated slots accumulate as in the reference) */
                static_assert(FORNEY_R == 4, "record words hold four magnitudes");
                uint32_t pk[RS_NR / 4], M[RS_NR / 4];
#pragma unroll
                for (int q = 0; q < RS_NR / 4; ++q) {
                    pk[q] = 0;
                    M[q] = 0;
                }
#pragma unroll
                for (int n = 0; n < RS_NR; ++n) {
                    const uint32_t p = (uint32_t)n < cnt ? min((uint32_t)pos[n], 255u) : 255u;
                    pk[n >> 2] |= p << (8 * (n & 3));
                }
                uint32_t steps = 0;
                for (uint32_t n = 0; n < cntmax; n += FORNEY_R) {
                    uint32_t cur = 0;
#pragma unroll
                    for (int t = 0; t < FORNEY_R; ++t) {
                        uint32_t lm;
                        const uint32_t num = forney(it.next(), lm);
                        const bool z = n + t < cnt && num != 0u;
                        if (!verify)
                            corrected += z ? 1u : 0u;
                        cur |= (z ? gf.exp(lm) : 0u) << (8 * t);
                    }
#pragma unroll
                    for (int q = 0; q < RS_NR / 4 - 1; ++q)
                        M[q] = M[q + 1];
                    M[RS_NR / 4 - 1] = cur;
                    ++steps;
                }
                for (; steps < RS_NR / 4; ++steps) { /* uniform: words into place */
#pragma unroll
                    for (int q = 0; q < RS_NR / 4 - 1; ++q)
                        M[q] = M[q + 1];
                    M[RS_NR / 4 - 1] = 0;
                }
                uint4 *r = reinterpret_cast<uint4 *>(recp);
                r[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
                r[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
                r[2] = make_uint4(M[0], M[1], M[2], M[3]);
                r[3] = make_uint4(M[4], M[5], M[6], M[7]);
            }
        } else if (pass == 1u) {
            /* apply (src/decode.c:211-227), FORNEY_R roots per step: their
             * sums are independent (the lookups of a step issue together),
             * and the bytes they correct are loaded one step ahead, so the
             * HBM latency of the loads hides behind the previous step's
             * sums.  Error mode: the root's location; erasure mode: list
             * slot n (quirk Q1/Q2: slot by root ordinal). */
            /* erasure mode: the slot positions, clamped to 255 (bytes
             * >= size + 32 are never written), packed 4 per dword.  If the
             * slots that are applied are not strictly ascending, two roots
             * may correct the same byte: then (seq) every byte is loaded
             * right before its store, in root order, as in the reference. */
            uint32_t pk[RS_NR / 4];
            bool seq = false;
            if (ERA) {
                bool asc = true;
                uint32_t prev = 0, have = 0;
#pragma unroll
                for (int n = 0; n < RS_NR; ++n) {
                    if ((n & 3) == 0)
                        pk[n >> 2] = 0;
                    if ((uint32_t)n < cntmax) { /* uniform */
                        const uint32_t p = (uint32_t)n < cnt ? min((uint32_t)pos[n], 255u) : 255u;
                        pk[n >> 2] |= p << (8 * (n & 3));
                        const bool app = (uint32_t)n < cnt && p < size + RS_NR;
                        asc = asc && !(app && have && p <= prev);
                        prev = app ? p : prev;
                        have |= app ? 1u : 0u;
                    }
                }
                seq = wave_max(asc ? 0u : 1u) != 0u;
            }
            auto tpos = [&](uint32_t n, uint32_t i) __attribute__((always_inline)) {
                if (ERA) {
                    uint32_t w = pk[0];
#pragma unroll
                    for (int q = 1; q < RS_NR / 4; ++q)
                        w = (n >> 2) == (uint32_t)q ? pk[q] : w;
                    return (w >> (8u * (n & 3u))) & 0xffu;
                }
                return (uint32_t)((int32_t)((i * P.iprim + 254u) % 255u) - pad);
            };
            /* erasure mode loads the next step's bytes during this step's
             * sums (measured: 1.03 -> 0.90 ms at 32 erasures); error mode
             * loads a step's bytes at its start (the extra registers of the
             * look-ahead spill there: 0.475 -> 0.491 ms) */
            constexpr bool AHEAD = ERA;
            uint32_t ir[FORNEY_R], ov[FORNEY_R];
            if (AHEAD) {
#pragma unroll
                for (int t = 0; t < FORNEY_R; ++t) {
                    ir[t] = it.next(); /* 255 past the last root */
                    ov[t] = seq ? 0u : *target(tpos((uint32_t)t, ir[t]));
                }
            }
            for (uint32_t n = 0; n < cntmax; n += FORNEY_R) {
                uint32_t irn[FORNEY_R], ovn[FORNEY_R], lm[FORNEY_R], nm[FORNEY_R];
                const bool more = AHEAD && n + FORNEY_R < cntmax; /* uniform */
                if (!AHEAD) {
#pragma unroll
                    for (int t = 0; t < FORNEY_R; ++t) {
                        ir[t] = it.next();
                        ov[t] = *target(tpos(n + (uint32_t)t, ir[t]));
                    }
                } else if (more) {
#pragma unroll
                    for (int t = 0; t < FORNEY_R; ++t) {
                        irn[t] = it.next();
                        ovn[t] = seq ? 0u : *target(tpos(n + FORNEY_R + (uint32_t)t, irn[t]));
                    }
                }
                if constexpr (!ERA) { /* group-major: 0.418 -> 0.414 ms; erasure mode root-major (0.89 vs 0.91) */
                    forney_r(ir, lm, nm);
                } else {
#pragma unroll
                    for (int t = 0; t < FORNEY_R; ++t)
                        nm[t] = forney(ir[t], lm[t]);
                }
#pragma unroll
                for (int t = 0; t < FORNEY_R; ++t) {
                    const bool z = n + t < cnt && nm[t] != 0u; /* zero numerator: no correction, not counted */
                    if (!verify) /* else counted in the check pass */
                        corrected += z ? 1u : 0u;
                    const uint32_t p = tpos(n + (uint32_t)t, ir[t]);
                    if (z && p < size + RS_NR) {
                        uint8_t *d = target(p);
                        *d = (uint8_t)((seq ? (uint32_t)*d : ov[t]) ^ gf.exp(lm[t]));
                    }
                }
                if (more) {
#pragma unroll
                    for (int t = 0; t < FORNEY_R; ++t) {
                        ir[t] = irn[t];
                        ov[t] = ovn[t];
                    }
                }
            }
        } else {
            /* re-syndrome check (src/decode.c:193-209), per root */
            for (uint32_t n = 0; n < cntmax; ++n) {
                const uint32_t i = it.next(); /* root, ascending as in the reference */
                const uint32_t k = (i * P.iprim + 254u) % 255u;
                uint32_t lmag;
                const uint32_t num = forney(i, lmag);
                const bool nz = run && n < cnt && num != 0u;
                if (nz) {
                    ++corrected; /* counted once, before the check */
                    /* contribution mag * alpha^((fcr+q)*prim*(254-k)) */
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
        }
        if (pass == 0u) {
#pragma unroll
            for (int q = 0; q < RS_NR; ++q)
                V[q >> 2] ^= gf.exp(SLOG((uint32_t)q)) << (8 * (q & 3)); /* zero S: ZL -> 0 */
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
#undef OMLOG
#undef LODD
    return good;
}

/* REC (erasure mode): corrections go to 64-byte records (rec) for rs_apply_k,
 * meta[cw] = RS_ST_FAST where a record was written, RS_ST_DONE elsewhere */
template <typename PosT, bool ERA, bool REC = false>
__global__ __launch_bounds__(COR_WG) void rs_correct_k(const RsDevTables *__restrict__ T, RsCorrParams P,
                                                       uint8_t *data, size_t dstride, uint8_t *parity, size_t pstride,
                                                       size_t count, const uint8_t *__restrict__ syn,
                                                       const uint16_t *__restrict__ syn16, size_t syn16_stride,
                                                       const PosT *__restrict__ pos, size_t pos_stride,
                                                       const uint8_t *__restrict__ cnt, uint8_t *__restrict__ ok,
                                                       uint8_t *__restrict__ corrected,
                                                       const uint32_t *__restrict__ list,
                                                       const uint32_t *__restrict__ list_n,
                                                       uint8_t *__restrict__ rec = nullptr,
                                                       uint8_t *__restrict__ meta = nullptr)
{
    /* list mode (the split decode's fallback, rs_fast.hip): the codewords
     * list[0 .. *list_n); otherwise 0 .. count - 1.  The codewords are dealt
     * to the waves in runs of 64, run c to workgroup c mod G, so that a short
     * list (or a small batch) spreads over every CU instead of filling the
     * first few workgroups: each wave is one lane-serial decode chain, and
     * the time of a short list is the latency of the busiest SIMD's waves
     * (74k beyond-capacity codewords of 2^20 on 73 of 256 CUs took 0.36 ms).
     * Blocks with no work leave before filling the tables. */
    const size_t n = list ? (size_t)*list_n : count;
    if ((size_t)blockIdx.x * 64u >= n)
        return;
    /* one block, carved by hand: the layout (and lgf ending exactly at the
     * allocation's end) is part of the arithmetic, see the header */
    __shared__ uint4 lds[LDS_END / 16];
    uint8_t *lsyn = reinterpret_cast<uint8_t *>(lds) + LDS_SYN;
    uint4 *lch = lds + LDS_CH / 16;
    uint32_t *lgf = reinterpret_cast<uint32_t *>(reinterpret_cast<uint8_t *>(lds) + LDS_GF);
    {
        /* byte 1: exp2[x]; bytes 2-3: scaled log of x & 255 (0xFFFF for 0):
         * the host-built image RsDevTables::gfc, and the Chien rows -- every
         * load issued before the first store (a rolled loop waits for each) */
        static_assert(GF_REPL == 32, "gfc is built for 32 replicas");
        constexpr int KG = 512 * GF_REPL / 4 / COR_WG, KC = 16 * 256 / COR_WG;
        uint4 g[KG], c[KC];
#pragma unroll
        for (int k = 0; k < KG; ++k)
            g[k] = T->gfc[threadIdx.x + k * COR_WG];
#pragma unroll
        for (int k = 0; k < KC; ++k)
            c[k] = T->chien[threadIdx.x + k * COR_WG];
#pragma unroll
        for (int k = 0; k < KG; ++k)
            reinterpret_cast<uint4 *>(lgf)[threadIdx.x + k * COR_WG] = g[k];
#pragma unroll
        for (int k = 0; k < KC; ++k)
            lch[threadIdx.x + k * COR_WG] = c[k];
    }
    __syncthreads();
    const Gf gf{lds_addr(lgf) + (threadIdx.x & (GF_REPL - 1)) * 4 + 1};
    uint8_t *srow = lsyn + threadIdx.x;

    /* Runs of 64 codewords are dealt per wave, so the trip count is uniform
     * per wave only -- waves of one workgroup may make different numbers of
     * passes, and no workgroup barrier may appear inside this loop.  The whole
     * wave enters the correction when any of its codewords needs it (the
     * rest, with zero syndromes, ride through BM as no-ops and leave at
     * deg = 0): the BM bounds are then full-wave DPP reductions. */
    const uint32_t wslot = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    for (size_t run = (size_t)wslot * gridDim.x + blockIdx.x; run * 64u < n; run += (size_t)(COR_WG / 64) * gridDim.x) {
        const size_t idx = run * 64u + lane; /* the wave's run of 64 codewords: the trip count is wave-uniform */
        const bool valid = idx < n;
        const size_t cw = list ? (valid ? (size_t)list[idx] : 0) : idx;
        uint32_t sw[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        bool ext_bad = false; /* external syndrome > 255: out-of-table in the reference, refused */
        if (valid && syn16) {
            /* external log-form syndromes (u16, the reference's type) */
            const uint16_t *e = syn16 + cw * syn16_stride;
#pragma unroll
            for (int q = 0; q < RS_NR; ++q) {
                const uint32_t v = e[q];
                ext_bad |= v > 255u;
                sw[q >> 2] |= (v & 0xffu) << (8 * (q & 3));
            }
        } else if (valid) {
            const uint4 *s4 = reinterpret_cast<const uint4 *>(syn + cw * RS_NR);
            const uint4 sa = s4[0], sb = s4[1];
            sw[0] = sa.x, sw[1] = sa.y, sw[2] = sa.z, sw[3] = sa.w;
            sw[4] = sb.x, sw[5] = sb.y, sw[6] = sb.z, sw[7] = sb.w;
        }
        const uint32_t ne0 = (ERA && valid) ? cnt[cw] : 0u;
        /* a clean codeword succeeds whatever its erasure count (src/decode.c:468:
         * the syndrome test comes first); a dirty one with more erasures than
         * roots overflows the reference's locator (quirk Q5): refused, as
         * rs_era_bp_k does */
        bool dirty = false;
#pragma unroll
        for (int q = 0; q < RS_NR / 4; ++q)
            dirty |= syn16 ? sw[q] != 0xFFFFFFFFu : sw[q] != 0u;
        const bool refuse = (ne0 > RS_NR && dirty) || ext_bad;
        bool any = false;
#pragma unroll
        for (uint32_t q = 0; q < RS_NR; ++q) {
            const uint32_t v = (sw[q >> 2] >> (8u * (q & 3u))) & 0xffu;
            const uint32_t lv = (valid && !refuse) ? (syn16 ? v : min(gf.log(v), A0)) : A0;
            any |= lv != A0;
            srow[(31u - q) * COR_WG] = (uint8_t)lv;
        }
        const bool need = any;
        const size_t cs = valid ? cw : 0; /* rows of lanes past the batch: a mapped row, never written */
        uint32_t fixed = 0;
        bool good = !refuse;
        if (__ballot(need) != 0ull) { /* uniform: the whole wave enters */
            const bool r = correct_one<PosT, ERA, REC>(gf, lch, srow, P, data + cs * dstride, parity + cs * pstride,
                                                       need ? ne0 : 0u, ERA ? pos + cs * pos_stride : nullptr,
                                                       REC ? rec + cs * 64u : nullptr, fixed);
            good = need ? r : good;
        }
        if (valid) {
            ok[cw] = good ? 1 : 0;
            if (corrected)
                corrected[cw] = (uint8_t)fixed;
            if constexpr (REC)
                meta[cw] = (uint8_t)(((need && good) ? RS_ST_FAST : RS_ST_DONE) << 5);
        }
    }
}

/* one workgroup per CU at most, and no more than there are runs of 64
 * codewords to deal (a small batch still spreads over the CUs) */
static int persistent_grid(size_t count, int wg, int num_cu)
{
    (void)wg;
    size_t need = (count + 63) / 64;
    size_t g = (size_t)(num_cu > 0 ? num_cu : 256);
    return (int)(need < g ? (need ? need : 1) : g);
}

extern "C" hipError_t rsk_correct(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride,
                                  uint8_t *parity, size_t pstride, size_t count, const uint8_t *syn,
                                  const uint16_t *syn16, size_t syn16_stride,
                                  const uint8_t *pos8, const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt,
                                  uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const dim3 grid(persistent_grid(count, COR_WG, num_cu));
    if (pos32)
        RS_LAUNCH((rs_correct_k<uint32_t, true>), grid, dim3(COR_WG), 0, stream, tab, *prm, data, dstride,
                           parity, pstride, count, syn, syn16, syn16_stride, pos32, pos_stride, cnt, ok, corrected, nullptr, nullptr, nullptr,
                  nullptr);
    else if (pos8)
        RS_LAUNCH((rs_correct_k<uint8_t, true>), grid, dim3(COR_WG), 0, stream, tab, *prm, data, dstride,
                           parity, pstride, count, syn, syn16, syn16_stride, pos8, pos_stride, cnt, ok, corrected, nullptr, nullptr, nullptr,
                  nullptr);
    else /* error mode */
        RS_LAUNCH((rs_correct_k<uint8_t, false>), grid, dim3(COR_WG), 0, stream, tab, *prm, data, dstride,
                           parity, pstride, count, syn, syn16, syn16_stride, pos8, pos_stride, cnt, ok, corrected, nullptr, nullptr, nullptr,
                  nullptr);
    return hipGetLastError();
}

/* error-mode correction of the codewords list[0 .. *list_n) (the count is read
 * on the device: the split decode's fallback, rs_fast.hip) */
extern "C" hipError_t rsk_correct_list(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride,
                                       uint8_t *parity, size_t pstride, size_t count, const uint8_t *syn,
                                       const uint32_t *list, const uint32_t *list_n, uint8_t *ok,
                                       uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    /* full persistent grid: the list is empty for codewords with at most 16
     * errors, and blocks past its length leave before filling their tables */
    const dim3 grid(persistent_grid(count, COR_WG, num_cu));
    RS_LAUNCH((rs_correct_k<uint8_t, false>), grid, dim3(COR_WG), 0, stream, tab, *prm, data, dstride,
                       parity, pstride, count, syn, nullptr, 0, nullptr, 0, nullptr, ok, corrected, list, list_n, nullptr, nullptr);
    return hipGetLastError();
}

/* erasure mode with the corrections as records (the split erasure decode,
 * then rsk_apply_era): rec 64 B and meta 1 B per codeword */
extern "C" hipError_t rsk_correct_era_rec(const RsDevTables *tab, const RsCorrParams *prm, size_t count,
                                          const uint8_t *syn, const uint8_t *pos8, const uint32_t *pos32,
                                          size_t pos_stride, const uint8_t *cnt, uint8_t *ok, uint8_t *corrected,
                                          uint8_t *rec, uint8_t *meta, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const dim3 grid(persistent_grid(count, COR_WG, num_cu));
    if (pos32)
        RS_LAUNCH((rs_correct_k<uint32_t, true, true>), grid, dim3(COR_WG), 0, stream, tab, *prm, nullptr,
                           0, nullptr, 0, count, syn, nullptr, 0, pos32, pos_stride, cnt, ok, corrected, nullptr,
                           nullptr, rec, meta);
    else
        RS_LAUNCH((rs_correct_k<uint8_t, true, true>), grid, dim3(COR_WG), 0, stream, tab, *prm, nullptr, 0,
                           nullptr, 0, count, syn, nullptr, 0, pos8, pos_stride, cnt, ok, corrected, nullptr, nullptr,
                           rec, meta);
    return hipGetLastError();
}

/* the same over the codewords list[0 .. *list_n) that rs_era_bp_k hands on */
extern "C" hipError_t rsk_correct_era_list(const RsDevTables *tab, const RsCorrParams *prm, size_t count,
                                           const uint8_t *syn, const uint8_t *pos8, size_t pos_stride,
                                           const uint8_t *cnt, uint8_t *ok, uint8_t *corrected, uint8_t *rec,
                                           uint8_t *meta, const uint32_t *list, const uint32_t *list_n, int num_cu,
                                           hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    /* full persistent grid: blocks past the list's length leave at once */
    const dim3 grid(persistent_grid(count, COR_WG, num_cu));
    RS_LAUNCH((rs_correct_k<uint8_t, true, true>), grid, dim3(COR_WG), 0, stream, tab, *prm, nullptr, 0,
                       nullptr, 0, count, syn, nullptr, 0, pos8, pos_stride, cnt, ok, corrected, list, list_n, rec,
                       meta);
    return hipGetLastError();
}
