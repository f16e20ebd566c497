/*
 * rs_single.hip -- one codeword per launch: the reference's calling pattern
 * (include/poporon.h:90-91, one poporon_encode / poporon_decode per 223-byte
 * message), on one 256-thread workgroup.
 *
 *   rs_enc1_k   parity of one message (src/encode.c:120-143) as the sum of
 *               host-built rows of the GF-linear LFSR (RsDevTables::encq)
 *   rs_dec1_k   the whole of rs_decode (src/decode.c:431-487) for one
 *               codeword in one launch: syndromes (:375-415) or external
 *               syndromes (:446-464), erasure locator (:31-47),
 *               Berlekamp-Massey (:49-96), degree (:98-110), Chien (:112-145),
 *               Omega (:147-158), Forney (:159-191), re-syndrome check
 *               (:193-209), apply (:211-227)
 *
 * The batch kernels put one codeword on one lane, which makes one codeword
 * a serial chain of ~10^4 dependent steps on one lane.  Here the codeword is
 * spread over the workgroup instead: each syndrome over 8 lanes, Berlekamp-
 * Massey with coefficient i of Lambda and B on lane i of one wave (the
 * discrepancy is a wave XOR reduction), Chien with one point per lane,
 * Omega and Forney with one coefficient / root per lane, the re-syndrome
 * check with one syndrome per lane, the corrections XORed into an LDS copy
 * of the codeword.  Every step keeps the reference's integer semantics
 * (uint16 gf_mod truncations, the int16 exponent of the check), so results
 * -- bytes, the bool and corrected_num -- are bit-exact for every branch.
 *
 * The codeword and the results may live in coherent host memory (the
 * single-call API hands over its caller's bytes that way): with `flag` set
 * the kernel writes `seq` there after everything else, with a system-scope
 * release, and the host polls it instead of synchronising the stream.
 *
 * GF arithmetic: logs in registers with ZL = 1024 for zero; ex[x] = alpha^(x
 * mod 255) for x <= 508 and 0 from 509 to EXN, so a product of two logs is
 * one LDS byte read and a zero operand (any sum with ZL) needs no test.
 */
#include <hip/hip_runtime.h>

#include "rs_device.h"

#define S1_WG 256
#define ZL 1024u    /* log of zero: any sum with it indexes the zero part of ex */
#define EXN 3072    /* ex[x] = alpha^(x mod 255) for x <= 508, 0 for 509 <= x < EXN */

namespace {

__device__ __forceinline__ uint32_t m255(uint32_t x) { return x % 255u; }
/* x mod 255 for x < 510; x >= 1024 stays >= 769 (a zero operand stays zero) */
__device__ __forceinline__ uint32_t red(uint32_t x) { return min(x, x - 255u); }

/* XOR over the 64 lanes of a wave, in every lane (DPP row reduction, then
 * the four row totals through SGPRs) */
__device__ __forceinline__ uint32_t wave_xor(uint32_t v)
{
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  /* quad_perm [1,0,3,2] */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  /* quad_perm [2,3,0,1] */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false); /* row_ror:4 */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false); /* row_ror:8 */
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 16) ^
           (uint32_t)__builtin_amdgcn_readlane((int)v, 32) ^ (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

/* XOR over each group of eight consecutive lanes, in every lane of the group */
__device__ __forceinline__ uint32_t oct_xor(uint32_t v)
{
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  /* quad_perm [1,0,3,2] */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  /* quad_perm [2,3,0,1] */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false); /* row_half_mirror */
    return v;
}

/* XOR over the 64 lanes of a wave, in every lane: the two halves and the
 * two rows of each half meet by gfx950's permlane swaps, the 16 lanes of a
 * row by DPP (six VALU ops, no scalar round trip) */
__device__ __forceinline__ uint32_t wave_xor_v(uint32_t v)
{
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    v = a[0] ^ a[1];
    const auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = b[0] ^ b[1];
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false); /* row_ror:8 */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false); /* row_ror:4 */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  /* quad_perm [2,3,0,1] */
    v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  /* quad_perm [1,0,3,2] */
    return v;
}

/* v of lane - 1 across the whole wave (DPP wave_shr:1); lane 0 keeps `old` */
__device__ __forceinline__ uint32_t wave_up_old(uint32_t v, uint32_t old)
{
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)v, 0x138, 0xf, 0xf, false);
}

/* v of lane - 1 across the whole wave (DPP wave_shr:1); lane 0 gets `first` */
__device__ __forceinline__ uint32_t wave_up(uint32_t v, uint32_t lane, uint32_t first)
{
    const uint32_t u = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, true);
    return lane ? u : first;
}

struct Tabs {
    uint8_t ex[EXN];
    uint16_t lg[256];
};

/* ex / lg from the handle's tables (exp2: alpha^(x mod 255) for x < 511) */
__device__ __forceinline__ void fill_tabs(Tabs &s, const RsDevTables *__restrict__ T, uint32_t t)
{
    const uint32_t a = T->exp2[t], b = T->exp2[t + 256u];
    s.ex[t] = (uint8_t)a;
    s.ex[t + 256u] = t + 256u <= 508u ? (uint8_t)b : 0;
#pragma unroll
    for (uint32_t k = 2; k < EXN / S1_WG; ++k)
        s.ex[t + k * S1_WG] = 0;
    s.lg[t] = t ? T->log[t] : ZL;
}

} // namespace

/* ------------------------------------------------------------------------ */
/* encode                                                                    */
/* ------------------------------------------------------------------------ */

/* parity = sum_j data_j Q[size-1-j], Q[d] = the parity of a one-byte message
 * 1 followed by d zeros (RsDevTables::encq, log form, built on the host by
 * running the reference's LFSR).  Thread j: message byte j times its 32-byte
 * row (two 16-byte loads, issued with the message and table loads: one
 * memory round trip); the products are XOR-reduced over each wave (DPP),
 * then over the four waves in LDS. */
/* the encode of one message by the whole workgroup; the tables in s are
 * filled (or being filled: the first barrier below orders them) */
__device__ __forceinline__ void enc1_body(Tabs &s, uint32_t (*wred)[8], const RsDevTables *__restrict__ T,
                                          const uint8_t *data, uint8_t *parity, uint32_t size, uint32_t npar = RS_NR)
{
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    uint32_t w = 0;
    uint4 q0 = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu), q1 = q0;
    if (t < size) {
        w = data[t]; /* may be host memory: one round trip, with the table loads */
        const uint4 *q = reinterpret_cast<const uint4 *>(T->encq + (size - 1u - t) * RS_NR);
        q0 = q[0];
        q1 = q[1];
    }
    __syncthreads();
    const uint32_t lm = s.lg[w];
    const uint32_t qw[8] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w};
    uint32_t P[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        uint32_t v = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const uint32_t qb = (qw[k] >> (8 * b)) & 0xffu;
            v |= (uint32_t)s.ex[lm + (qb == 255u ? ZL : qb)] << (8 * b);
        }
        P[k] = v;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
        P[k] = wave_xor(P[k]);
    if (lane < 8) {
        uint32_t v = P[0];
#pragma unroll
        for (int k = 1; k < 8; ++k)
            v = lane == (uint32_t)k ? P[k] : v;
        wred[wave][lane] = v;
    }
    __syncthreads();
    if (t < npar) { /* npar < 32: a code with fewer roots (its encq rows are zero past npar) */
        const uint32_t d = wred[0][t >> 2] ^ wred[1][t >> 2] ^ wred[2][t >> 2] ^ wred[3][t >> 2];
        parity[t] = (uint8_t)(d >> (8u * (t & 3u)));
    }
}

__global__ __launch_bounds__(S1_WG) void rs_enc1_k(const RsDevTables *__restrict__ T, const uint8_t *data,
                                                   uint8_t *parity, uint32_t size, uint32_t *flag, uint32_t seq,
                                                   uint32_t npar)
{
    __shared__ Tabs s;
    __shared__ uint32_t wred[4][8];
    const uint32_t t = threadIdx.x;
    fill_tabs(s, T, t);
    enc1_body(s, wred, T, data, parity, size, npar);
    if (flag) {
        /* every wave's parity stores acknowledged, then lane 0's system-scope
         * release and the flag (rs_serve_k) */
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (t == 0)
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* ------------------------------------------------------------------------ */
/* decode                                                                    */
/* ------------------------------------------------------------------------ */

struct Dec1Smem {
    Tabs g;
    uint8_t cw[256];     /* the codeword, corrected in place */
    uint16_t lw[256];    /* log of each codeword byte (ZL: zero) */
    uint32_t part[S1_WG];
    uint32_t slog[64];   /* log S_i (ZL: zero), i < 32; ZL at 32..63 */
    uint32_t spoly[32];  /* S_i as field elements (the check compares against these) */
    uint32_t llam[33];   /* log Lambda_j (ZL: zero) after BM */
    uint32_t lom[32];    /* log Omega_m (ZL: zero) */
    uint32_t roots[32], locs[32], mags[32];
    uint32_t pos[32];    /* erasure slots (erasure mode) */
    uint32_t wcnt[4];    /* roots per wave (Chien) */
    uint32_t flags;
    uint32_t low;        /* Chien: a root below the padding (its own word: a wave still
                          * testing `flags` after the BM barrier must not see it) */
    uint32_t deg, nfix;
};

#define F_ANY 1u
#define F_FAIL 2u

/* mode: 0 plain, 1 erasure (pos8 or pos32 slots, *cnt erasures), 2 external
 * log-form syndromes (ext, 32 x u16).  ok / cor: one byte each (written
 * always, as rs_decode writes corrected_num also on failure). */
/* rs_decode of one codeword by the whole workgroup (the tables in s.g
 * filled, or being filled: the first barrier orders them); ok / corrected
 * stored, the caller signals completion */
__device__ void dec1_body(Dec1Smem &s, const RsCorrParams &P, uint32_t mode, uint8_t *data, uint8_t *parity,
                          const uint8_t *pos8, const uint32_t *pos32, const void *cnt, uint32_t cnt_bytes,
                          const uint16_t *ext, uint8_t *okp, uint8_t *corp)
{
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    const uint32_t nr = P.nr; /* 32, or fewer (a code with fewer roots: syndromes, BM, check over nr) */
    const uint32_t size = P.size, L = size + nr;
    const int32_t pad = P.pad;
    uint32_t ok = 0, fixed = 0;
    /* STAMP 0 */

    /* ---- inputs: the codeword (one byte per thread), slots: all loads
     * issued together (the codeword may be host memory) ---- */
    uint32_t w = 0;
    if (t < L)
        w = t < size ? data[t] : parity[t - size];
    uint32_t ne = 0, xs = 0;
    if (mode == 1u) {
        ne = cnt_bytes == 4u ? *(const uint32_t *)cnt : *(const uint8_t *)cnt;
        if (t < nr)
            s.pos[t] = pos32 ? pos32[t] : pos8[t];
    } else if (mode == 2u && t < nr) {
        xs = ext[t];
    }
    s.cw[t] = (uint8_t)w;
    if (t == 0) {
        s.flags = 0;
        s.low = 0;
    }
    if (t >= nr && t < 64u)
        s.slog[t] = ZL;
    __syncthreads();
    /* STAMP 1 */

    /* ---- syndromes, log form (src/decode.c:375-415; external: :446-454) ---- */
    bool refuse = false;
    if (mode == 2u) {
        if (t < nr) {
            refuse = xs > 255u; /* out-of-table in the reference: refused */
            s.slog[t] = xs >= 255u ? ZL : xs;
            s.spoly[t] = xs >= 255u ? 0u : s.g.ex[xs];
            if (xs != 255u)
                atomicOr(&s.flags, F_ANY);
        }
    } else {
        s.lw[t] = s.g.lg[w]; /* ZL past the codeword (w = 0) */
        __syncthreads();
        /* S_i = sum_j w_j beta_i^(L-1-j), beta_i = alpha^(prim (fcr+i)) (the
         * reference's Horner steps, exact for the fast parameters): thread t
         * sums syndrome i = t & 31 over j = t >> 5 + 8k -- 32 independent
         * lookups */
        const uint32_t i = t & 31u, g0 = t >> 5;
        const uint32_t b = m255(P.prim * (P.fcr + i));
        const uint32_t d8 = m255(8u * b);
        uint32_t e = m255(b * (L - 1u - g0)), acc = 0;
#pragma unroll
        for (uint32_t k = 0; k < 32; ++k) {
            acc ^= s.g.ex[s.lw[g0 + 8u * k] + e]; /* j = g0 + 8k <= 255: ZL past the codeword */
            e = e >= d8 ? e - d8 : e + 255u - d8;
        }
        s.part[t] = acc;
        __syncthreads();
        if (t < nr) {
            uint32_t v = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k)
                v ^= s.part[t + 32u * k];
            s.spoly[t] = v;
            s.slog[t] = s.g.lg[v];
            if (v)
                atomicOr(&s.flags, F_ANY);
        }
    }
    if (__syncthreads_or(refuse)) /* uniform */
        goto finish;
    /* STAMP 2 */
    {
        const bool any = (s.flags & F_ANY) != 0u;
        /* a clean codeword succeeds whatever its erasure count (src/decode.c:468);
         * a dirty one with more erasures than roots overflows the reference's
         * locator (quirk Q5): refused, as the batch kernels do */
        if (!any || (mode == 1u && ne > nr)) {
            ok = any ? 0u : 1u;
            goto finish;
        }
    }

    /* ---- erasure locator and Berlekamp-Massey on wave 0: lane i holds
     * Lambda_i (poly and log) and B_i (log), i <= 32 ---- */
    if (wave == 0) {
        const bool co = lane <= nr; /* a coefficient lane */
        uint32_t lam = lane == 0 ? 1u : 0u;
        /* Lambda = prod (1 + X_l x), X_l = alpha^(prim (254 - (pos_l + pad))) with the
         * reference's uint32 arithmetic and uint16 gf_mod (src/decode.c:34-47) */
        for (uint32_t l = 0; l < ne; ++l) {
            const uint32_t xl = ((P.prim * (uint32_t)(RS_NN - 1u - (s.pos[l] + (uint32_t)pad))) & 0xffffu) % 255u;
            const uint32_t prev = wave_up(lam, lane, 0u);
            lam ^= lane ? s.g.ex[xl + s.g.lg[prev]] : 0u;
        }
        uint32_t llam = s.g.lg[lam];
        uint32_t B = llam; /* coefficients[] of the reference (ZL for its 255) */
        uint32_t Lr = ne;
        /* Karn's iteration (src/decode.c:55-96), r = ne+1 .. 32, with Lambda in
         * poly and log form.  The critical path is disc -> log disc -> the next
         * discrepancy's terms, formed from the pre-update log, (Lambda_i +
         * q B_(i-1)) S = Lambda_i S + q B_(i-1) S; the updated coefficient
         * and its log follow off that path.  disc = 0 gives log disc = ZL:
         * no update.  Lanes past 32 only ever meet zero syndromes (ZL), so
         * whatever they hold never reaches a discrepancy. */
        uint32_t term = s.g.ex[llam + s.slog[lane <= ne ? ne - lane : 63u]]; /* Lambda_i S_(r-1-i), r = ne + 1 */
        /* S_(r-i) for the terms of the next iteration, read one iteration
         * ahead (slog[63] = ZL past them) */
        uint32_t s1 = s.slog[lane <= ne + 1u && ne + 1u < nr ? ne + 1u - lane : 63u];
        for (uint32_t r = ne + 1u; r <= nr; ++r) {
            const uint32_t disc = wave_xor_v(term); /* in every lane */
            const uint32_t bs = wave_up_old(B, ZL);  /* B_(i-1); lane 0: zero (Lambda_0 stays 1) */
            const uint32_t ld = s.g.lg[disc];
            const uint32_t dq = red(ld + bs);         /* log of disc B_(i-1); >= 255: zero */
            const uint32_t t1 = s.g.ex[llam + s1], t2 = s.g.ex[dq + s1], up = s.g.ex[dq];
            s1 = s.slog[lane <= r + 1u && r + 1u < nr ? r + 1u - lane : 63u];
            term = t1 ^ t2;
            const uint32_t ds = __builtin_amdgcn_readfirstlane(disc);
            const bool len = ds != 0u && 2u * Lr <= r + ne - 1u; /* uniform */
            const uint32_t bl = lam ? red(llam + 255u - ld) : ZL; /* B <- Lambda (old) / disc */
            B = len ? bl : bs;                                    /* or B <- x B */
            Lr = len ? r + ne - Lr : Lr;
            lam ^= up;
            llam = s.g.lg[lam];
        }
        /* degree, src/decode.c:98-110 (lane 0 holds Lambda_0 = 1) */
        const uint64_t nz = __ballot(co && lam != 0u);
        const uint32_t deg = 63u - (uint32_t)__builtin_clzll(nz);
        if (lane <= RS_NR) /* ZL past nr: Chien, Omega and Forney read up to Lambda_32 */
            s.llam[lane] = co ? llam : ZL;
        if (lane == 0) {
            s.deg = deg;
            s.nfix = 0;
            if (deg == 0u)
                s.flags |= F_FAIL;
        }
    }
    __syncthreads();
    /* STAMP 3 */
    if (s.flags & F_FAIL)
        goto finish;
    {
        const uint32_t deg = s.deg;
        /* ---- Chien: point i = t + 1 (1..255), Lambda(alpha^i) = 1 + sum_j
         * alpha^(log Lambda_j + i j); location k = (i iprim - 1) mod 255
         * (src/decode.c:117-141) ---- */
        {
            const uint32_t i = t + 1u, ii = i == 255u ? 0u : i;
            uint32_t ev = 1u, e = 0;
#pragma unroll
            for (uint32_t jb = 0; jb < RS_NR; jb += 8) {
                if (jb < deg) { /* uniform: eight terms at a time up to the degree */
#pragma unroll
                    for (uint32_t j = jb + 1u; j <= jb + 8u; ++j) {
                        e = red(e + ii);
                        ev ^= s.g.ex[s.llam[j] + e]; /* ZL past the degree */
                    }
                }
            }
            const bool root = t < 255u && ev == 0u;
            const uint32_t k = (i * P.iprim + 254u) % 255u;
            const uint64_t rb = __ballot(root);
            if (lane == 0)
                s.wcnt[wave] = (uint32_t)__builtin_popcountll(rb);
            if (root && (int32_t)k < pad) /* src/decode.c:132-134 */
                atomicOr(&s.low, 1u);
            __syncthreads();
            uint32_t before = 0, total = 0;
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) {
                before += q < wave ? s.wcnt[q] : 0u;
                total += s.wcnt[q];
            }
            if (root) {
                const uint32_t idx = before + (uint32_t)__builtin_popcountll(rb & ((1ull << lane) - 1ull));
                if (idx < RS_NR) {
                    s.roots[idx] = i;
                    s.locs[idx] = k;
                }
            }
            if ((total != deg || s.low) && t == 0) /* src/decode.c:143-145 */
                atomicOr(&s.flags, F_FAIL);
            __syncthreads();
            if (s.flags & F_FAIL)
                goto finish;
        }
        /* STAMP 4 */

        /* ---- Omega_m = sum_(j <= m) S_(m-j) Lambda_j, m < deg (src/decode.c:147-158):
         * thread t sums coefficient m = t & 31 over j = 4 (t >> 5) .. + 3 ---- */
        {
            const uint32_t m = t & 31u, j0 = (t >> 5) * 4u;
            uint32_t acc = 0;
#pragma unroll
            for (uint32_t j = j0; j < j0 + 4u; ++j) /* j > m reads slog[32..63] = ZL; llam is ZL past the degree */
                acc ^= s.g.ex[s.slog[(m - j) & 63u] + s.llam[j]];
            s.part[t] = acc;
            __syncthreads();
            if (t < RS_NR) {
                uint32_t v = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    v ^= s.part[t + 32u * k];
                s.lom[t] = t < deg ? (uint32_t)s.g.lg[v] : ZL;
            }
        }
        __syncthreads();
        /* STAMP 5 */

        /* ---- Forney, src/decode.c:159-191: root q = t >> 3 on eight lanes, lane
         * u = t & 7 summing the numerator terms m = u + 8k and the denominator
         * terms h = 2u, 2u + 16; the eight partial sums meet by DPP ---- */
        {
            const uint32_t q = t >> 3, u = t & 7u;
            const uint32_t rt = q < deg ? s.roots[q] : 0u;
            const uint32_t rm = rt % 255u;
            uint32_t num = 0, den = 0;
#pragma unroll
            for (uint32_t k = 0; k < 4; ++k) { /* alpha^(Omega_m + m root); Omega is ZL past deg - 1 */
                const uint32_t m = u + 8u * k;
                num ^= s.g.ex[s.lom[m] + (m * rm) % 255u];
            }
#pragma unroll
            for (uint32_t k = 0; k < 2; ++k) { /* alpha^(Lambda_(h+1) + h root), even h <= 30: Lambda is ZL
                                                * past the degree (the reference's bound min(deg, 31) & ~1) */
                const uint32_t h = 2u * u + 16u * k;
                den ^= s.g.ex[s.llam[h + 1u] + (h * rm) % 255u];
            }
            num = oct_xor(num);
            den = oct_xor(den);
            if (u == 0u) {
                uint32_t mag = 0;
                if (q < deg && num) {
                    const uint32_t l2 =
                        ((uint32_t)((int32_t)rt * ((int32_t)P.fcr - 1) + (int32_t)RS_NN) & 0xffffu) % 255u;
                    const uint32_t lden = den ? s.g.lg[den] : 255u; /* no den = 0 guard: log 0 = 255 */
                    mag = s.g.ex[(s.g.lg[num] + l2 + RS_NN - lden) % 255u];
                    atomicAdd(&s.nfix, 1u);
                }
                s.mags[q] = mag;
                if (q >= deg)
                    s.locs[q] = 0;
            }
        }
        __syncthreads();
        /* STAMP 6 */
        fixed = s.nfix; /* Q6: corrected_num counts the nonzero numerators, also on failure */

        /* ---- re-syndrome check, src/decode.c:193-209, with the reference's
         * int16 exponent and uint16 gf_mod ---- */
        {
            /* thread t: syndrome i = t & 31 over roots q = 4 (t >> 5) .. + 3;
             * the eight partial sums meet in LDS (mags is 0 past the root count) */
            const uint32_t i = t & 31u, q0 = (t >> 5) * 4u;
            const int32_t ci = (int32_t)(P.fcr + i) * (int32_t)P.prim;
            uint32_t acc = 0;
#pragma unroll
            for (uint32_t q = q0; q < q0 + 4u; ++q) {
                const uint32_t mg = s.mags[q];
                const int16_t k16 = (int16_t)(ci * (int32_t)(RS_NN - 1u - s.locs[q]));
                const uint32_t x = ((uint32_t)((int32_t)s.g.lg[mg] + (int32_t)k16) & 0xffffu) % 255u;
                acc ^= mg ? (uint32_t)s.g.ex[x] : 0u;
            }
            s.part[t] = acc;
            __syncthreads();
            if (t < nr) {
                uint32_t v = 0;
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    v ^= s.part[t + 32u * k];
                if (v != s.spoly[t])
                    atomicOr(&s.flags, F_FAIL);
            }
        }
        __syncthreads();
        /* STAMP 7 */
        if (s.flags & F_FAIL)
            goto finish;

        /* ---- apply, src/decode.c:211-227 ---- */
        bool bad = false;
        if (t < deg) {
            const uint32_t mg = s.mags[t];
            uint32_t p;
            if (mode == 1u) {
                /* magnitude q (ascending location) into slot q (quirks Q1/Q2);
                 * slots past the codeword: parity when < size + nr (Q4), else dropped */
                p = s.pos[t];
            } else {
                p = (uint32_t)((int32_t)s.locs[t] - pad);
                bad = (int32_t)s.locs[t] - pad < 0 || p >= L;
            }
            if (mg && p < L && !bad)
                atomicXor(reinterpret_cast<uint32_t *>(s.cw) + (p >> 2), mg << (8u * (p & 3u)));
        }
        /* error mode: the corrections before the first bad location stay
         * applied and the call fails (src/decode.c:223-225) -- unreachable for
         * Chien locations (pad <= loc <= 254), kept for the rule's sake */
        if (__syncthreads_count(bad)) {
            __shared__ uint32_t first_bad;
            if (t == 0)
                first_bad = RS_NR;
            __syncthreads();
            if (bad)
                atomicMin(&first_bad, t);
            __syncthreads();
            if (t < deg && t > first_bad) { /* undo the corrections after the first bad one */
                const uint32_t p = (uint32_t)((int32_t)s.locs[t] - pad);
                const uint32_t mg = s.mags[t];
                if (mg && p < L)
                    atomicXor(reinterpret_cast<uint32_t *>(s.cw) + (p >> 2), mg << (8u * (p & 3u)));
            }
        } else {
            ok = 1;
        }
        __syncthreads();
        if (t < L) {
            const uint8_t v = s.cw[t];
            if (v != (uint8_t)w) {
                if (t < size)
                    data[t] = v;
                else
                    parity[t - size] = v;
            }
        }
    }
finish:
    /* STAMP 8 */
    if (t == 0) {
        *okp = (uint8_t)ok;
        if (corp) /* the batch API's d_corrected may be NULL */
            *corp = (uint8_t)fixed;
    }
}

__global__ __launch_bounds__(S1_WG) void rs_dec1_k(const RsDevTables *__restrict__ T, RsCorrParams P, uint32_t mode,
                                                   uint8_t *data, uint8_t *parity, const uint8_t *pos8,
                                                   const uint32_t *pos32, const void *cnt, uint32_t cnt_bytes,
                                                   const uint16_t *ext, uint8_t *okp, uint8_t *corp,
                                                   uint32_t *flag, uint32_t seq)
{
    __shared__ Dec1Smem s;
    const uint32_t t = threadIdx.x;
    fill_tabs(s.g, T, t);
    dec1_body(s, P, mode, data, parity, pos8, pos32, cnt, cnt_bytes, ext, okp, corp);
    if (flag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); /* as rs_enc1_k */
        __syncthreads();
        if (t == 0)
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* ------------------------------------------------------------------------ */
/* launchers                                                                 */
/* ------------------------------------------------------------------------ */

extern "C" hipError_t rsk_encode1(const RsDevTables *tab, const uint8_t *data, uint8_t *parity, uint32_t size,
                                  uint32_t *flag, uint32_t seq, hipStream_t stream)
{
    RS_LAUNCH(rs_enc1_k, dim3(1), dim3(S1_WG), 0, stream, tab, data, parity, size, flag, seq, (uint32_t)RS_NR);
    return hipGetLastError();
}

extern "C" hipError_t rsk_encode1_nr(const RsDevTables *tab, const uint8_t *data, uint8_t *parity, uint32_t size,
                                     uint32_t npar, uint32_t *flag, uint32_t seq, hipStream_t stream)
{
    RS_LAUNCH(rs_enc1_k, dim3(1), dim3(S1_WG), 0, stream, tab, data, parity, size, flag, seq, npar);
    return hipGetLastError();
}

extern "C" hipError_t rsk_decode1(const RsDevTables *tab, const RsCorrParams *prm, uint32_t mode, uint8_t *data,
                                  uint8_t *parity, const uint8_t *pos8, const uint32_t *pos32, const void *cnt,
                                  uint32_t cnt_bytes, const uint16_t *ext, uint8_t *ok, uint8_t *corrected,
                                  uint32_t *flag, uint32_t seq, hipStream_t stream)
{
    RS_LAUNCH(rs_dec1_k, dim3(1), dim3(S1_WG), 0, stream, tab, *prm, mode, data, parity, pos8, pos32, cnt,
                       cnt_bytes, ext, ok, corrected, flag, seq);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* single-call server                                                        */
/* ------------------------------------------------------------------------ */

/*
 * rs_serve_k: one workgroup that stays resident between single-codeword calls
 * and serves them from the handle's coherent host buffer (ZC_* layout,
 * rs_device.h), so that a poporon_encode / poporon_decode call costs no kernel
 * launch: the host writes the codeword and a request header there and bumps
 * ZC_REQ; lane 0 polls ZC_REQ (system-scope acquire loads over PCIe), the
 * workgroup runs enc1_body / dec1_body on the buffer and stores the request's
 * sequence number to ZC_FLAG with a system-scope release after every result.
 * The tables are filled once per launch.
 *
 * Every launch ends on its own: after idle_ticks of s_memrealtime (100 MHz)
 * without a request, after max_ticks in all, at an RS_SRV_STOP request
 * (poporon_destroy, or a batch call on the same handle), or, with no request
 * pending, when ZC_YIELD (read in the same 8-byte load as the request word)
 * differs from the value it was launched with (a batch call of another
 * handle on the device, api.cpp yield_servers).  It then stores its launch id to ZC_EXITED and serves
 * nothing more; a request the host posted meanwhile is seen unserved there
 * and the host launches a new server for it (api.cpp srv_call), on the same
 * stream, so two servers never run at once.
 */
#ifndef SRV_FULL_FENCE
#define SRV_FULL_FENCE 0 /* 1: a system-scope release fence in every wave (measured ~1.4 us more per call) */
#endif
__global__ __launch_bounds__(S1_WG) void rs_serve_k(const RsDevTables *__restrict__ T, RsCorrParams P, uint8_t *zc,
                                                    uint32_t last, uint32_t id, uint32_t yv,
                                                    uint64_t idle_ticks, uint64_t max_ticks)
{
    __shared__ Dec1Smem s;
    __shared__ uint32_t cmd[4]; /* seq, op (0: leave), size, mode */
    const uint32_t t = threadIdx.x;
    fill_tabs(s.g, T, t);
    uint64_t *req = reinterpret_cast<uint64_t *>(zc + ZC_REQ); /* ZC_REQ, ZC_YIELD */
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t idle0 = t0;
    for (;;) {
        if (t == 0) {
            /* the whole request is one word: one PCIe round trip per poll */
            uint32_t r = last, op = 0;
            for (;;) {
                /* the request word and ZC_YIELD in one 8-byte load */
                const uint64_t w = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                r = (uint32_t)w;
                if (r != last) {
                    op = ZC_REQ_OP(r); /* RS_SRV_STOP: leave */
                    cmd[2] = ZC_REQ_SIZE(r);
                    cmd[3] = ZC_REQ_MODE(r);
                    break;
                }
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                if (now - idle0 > idle_ticks || now - t0 > max_ticks || (uint32_t)(w >> 32) != yv)
                    break; /* op = 0: leave */
                __builtin_amdgcn_s_sleep(1);
            }
            cmd[0] = r;
            cmd[1] = op;
        }
        __syncthreads();
        const uint32_t seq = cmd[0], op = cmd[1], size = cmd[2], mode = cmd[3];
        if ((op != RS_SRV_ENCODE && op != RS_SRV_DECODE) || size == 0u || size > RS_NN - P.nr)
            break; /* uniform: idle, lifetime, RS_SRV_STOP; a malformed request also ends the
                    * launch (the host sees it unserved) */
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); /* this wave's loads of the payload: after the request */
        if (op == RS_SRV_ENCODE) {
            enc1_body(s.g, reinterpret_cast<uint32_t(*)[8]>(s.part), T, zc + ZC_DATA, zc + ZC_PAR, size, P.nr);
        } else {
            RsCorrParams Q = P;
            Q.size = size;
            Q.pad = (int32_t)(RS_NN - P.nr - size);
            dec1_body(s, Q, mode, zc + ZC_DATA, zc + ZC_PAR, nullptr, reinterpret_cast<const uint32_t *>(zc + ZC_POS),
                      zc + ZC_CNT, 4u, reinterpret_cast<const uint16_t *>(zc + ZC_EXT), zc + ZC_OK, zc + ZC_COR);
        }
        /* every wave's result stores (bytes, ok, count: several waves write
         * them) acknowledged before the barrier -- __syncthreads() alone is a
         * bare s_barrier here -- then lane 0's system-scope release (L2
         * write-back + wait) and the completion word */
#if SRV_FULL_FENCE
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
#else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        __syncthreads();
        if (t == 0)
            __hip_atomic_store(reinterpret_cast<uint32_t *>(zc + ZC_FLAG), seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        last = seq;
        idle0 = __builtin_amdgcn_s_memrealtime();
    }
    if (t == 0)
        __hip_atomic_store(reinterpret_cast<uint32_t *>(zc + ZC_EXITED), id, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" hipError_t rsk_serve(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *zc_dev, uint32_t last,
                                uint32_t id, uint32_t yv, uint64_t idle_ticks, uint64_t max_ticks,
                                hipStream_t stream)
{
    hipLaunchKernelGGL(rs_serve_k, dim3(1), dim3(S1_WG), 0, stream, tab, *prm, zc_dev, last, id, yv, idle_ticks,
                       max_ticks);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* one codeword per wave: small batches and the split decode's lists         */
/* ------------------------------------------------------------------------ */

/*
 * rs_wave_k: rs_decode (src/decode.c:431-487) for one codeword per WAVE with
 * dec1_body's steps and integer semantics: syndromes (:375-415; each of the
 * 32 over the two half-waves), or the split decode's poly syndromes, or
 * external log-form syndromes (:446-464); erasure locator (:31-47) and
 * Berlekamp-Massey (:49-96) with coefficient i on lane i; degree (:98-110);
 * Chien (:112-145) with four points per lane; Omega (:147-158), Forney
 * (:159-191) and the re-syndrome check (:193-209) over the two half-waves;
 * the apply (:211-227) in place: error mode straight into the codeword
 * (distinct locations), erasure mode through an LDS copy of the codeword
 * (slot n gets root n's magnitude, repeated slots accumulate: quirks Q1-Q4).
 *
 * It serves what one codeword per lane serves badly: few codewords.  The
 * lane-per-codeword kernels are a ~10^4-step serial chain per lane, so a
 * batch of a few thousand codewords (a few waves per SIMD) or the split
 * decode's list (the beyond-capacity codewords of a batch: 74k of 2^20 on a
 * binomial channel with mean 11.5 errors took 0.36 ms there) costs the
 * latency of that chain; here a codeword's work is spread over 64 lanes and
 * 32 waves per CU run side by side.
 *
 * Four waves per workgroup share the GF tables (no workgroup barrier after
 * their fill); each wave loops over its codewords: index e -> codeword
 * list[e] (list mode, length read on the device) or e.
 *
 * Modes: syn == NULL && syn16 == NULL: syndromes from the codeword; syn: the
 * split decode's poly syndromes (32 B per codeword); syn16: external log-form
 * u16 syndromes (> 255 refused).  pos8 / pos32 (at most one): erasure mode,
 * u8 counts in cnt.
 */
#define W_WG 256

struct WaveState {
    uint32_t slog[64];  /* log S_i (ZL: zero), i < 32; ZL at 32..63 */
    uint32_t spoly[32];
    uint32_t llam[64];  /* log Lambda_j (ZL: zero), j <= 32; ZL past */
    uint32_t lom[32];
    uint32_t roots[32], locs[32], mags[32], pos[32];
    uint16_t lw[256];   /* log of each codeword byte (ZL: zero or past the codeword) */
    uint32_t cw[64];    /* the codeword (erasure-mode apply) */
};

struct WaveSmem {
    Tabs g;
    WaveState w[W_WG / 64];
};

/* lane order within a wave: LDS writes by some lanes, then reads by others */
__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* v of lane l ^ 32 (the other half of the wave): the swap's first result
 * holds, in every lane, the low half's value, the second the high half's */
__device__ __forceinline__ uint32_t other_half(uint32_t v, uint32_t lane)
{
    const auto a = __builtin_amdgcn_permlane32_swap(v, v, false, false);
    return lane < 32u ? a[1] : a[0];
}

template <typename PosT>
__global__ __launch_bounds__(W_WG) void rs_wave_k(const RsDevTables *__restrict__ T, RsCorrParams P, uint8_t *data,
                                                  size_t dstride, uint8_t *parity, size_t pstride, size_t count,
                                                  const uint32_t *__restrict__ list, const uint32_t *__restrict__ list_n,
                                                  const uint8_t *__restrict__ syn, const uint16_t *__restrict__ syn16,
                                                  size_t syn16_stride, const PosT *__restrict__ pos, size_t pos_stride,
                                                  const uint8_t *__restrict__ cnt, uint8_t *__restrict__ okp,
                                                  uint8_t *__restrict__ corp)
{
    const size_t n = list ? (size_t)*list_n : count;
    if ((size_t)blockIdx.x * (W_WG / 64) >= n)
        return;
    __shared__ WaveSmem sm;
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    fill_tabs(sm.g, T, t);
    __syncthreads();
    const Tabs &g = sm.g;
    WaveState &s = sm.w[wave];
    const uint32_t size = P.size, L = size + RS_NR;
    const int32_t pad = P.pad;
    const bool co = lane <= RS_NR;
    const bool era = pos != nullptr;
    for (size_t e = (size_t)blockIdx.x * (W_WG / 64) + wave; e < n; e += (size_t)gridDim.x * (W_WG / 64)) {
        const size_t c = list ? (size_t)list[e] : e;
        uint8_t *cdata = data + c * dstride, *cpar = parity + c * pstride;
        /* ---- inputs: the codeword where the syndromes or the erasure apply
         * need it (lane j, j + 64, ...: coalesced), the slots ---- */
        uint32_t w4[4] = {0, 0, 0, 0};
        const bool own_syn = syn == nullptr && syn16 == nullptr;
        if (own_syn || era) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = lane + 64u * k;
                w4[k] = j < size ? cdata[j] : j < L ? cpar[j - size] : 0u;
            }
        }
        uint32_t ne = 0;
        if (era) {
            ne = cnt[c];
            if (lane < RS_NR)
                s.pos[lane] = (uint32_t)pos[c * pos_stride + lane];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t j = lane + 64u * k;
                reinterpret_cast<uint8_t *>(s.cw)[j] = (uint8_t)w4[k];
            }
        }
        /* ---- syndromes, log form ---- */
        bool refuse = false;
        uint32_t sv = 0; /* S_i as a field element, lanes < 32 */
        if (own_syn) {
#pragma unroll
            for (int k = 0; k < 4; ++k)
                s.lw[lane + 64u * k] = (uint16_t)g.lg[w4[k]]; /* ZL past the codeword (w = 0) */
            wave_sync();
            /* S_i = sum_j w_j beta_i^(L-1-j), beta_i = alpha^(prim (fcr+i)) (the
             * reference's Horner steps, exact for these parameters): lane l
             * sums syndrome i = l & 31 over j = (l >> 5) + 2k */
            const uint32_t i = lane & 31u, g0 = lane >> 5;
            const uint32_t b = m255(P.prim * (P.fcr + i));
            const uint32_t d2 = m255(2u * b);
            uint32_t ex = m255(b * (L - 1u - g0)), acc = 0;
#pragma unroll 8
            for (uint32_t k = 0; k < 128u; ++k) {
                acc ^= g.ex[s.lw[g0 + 2u * k] + ex]; /* j <= 255: ZL past the codeword */
                ex = ex >= d2 ? ex - d2 : ex + 255u - d2;
            }
            sv = acc ^ other_half(acc, lane);
        } else if (syn) {
            sv = lane < RS_NR ? syn[c * RS_NR + lane] : 0u;
        }
        if (syn16) {
            const uint32_t xs = lane < RS_NR ? syn16[c * syn16_stride + lane] : 255u;
            refuse = __ballot(xs > 255u) != 0ull; /* out-of-table in the reference: refused */
            if (lane < RS_NR) {
                s.slog[lane] = xs >= 255u ? ZL : xs;
                s.spoly[lane] = xs >= 255u ? 0u : g.ex[xs];
            } else {
                s.slog[lane] = ZL;
            }
        } else {
            if (lane < RS_NR)
                s.spoly[lane] = sv;
            s.slog[lane] = lane < RS_NR ? (uint32_t)g.lg[sv] : ZL;
        }
        const bool any = __ballot(lane < RS_NR && s.slog[lane] != ZL) != 0ull;
        wave_sync();
        uint32_t ok = 0, fixed = 0;
        /* a clean codeword succeeds whatever its erasure count (src/decode.c:468);
         * a dirty one with more erasures than roots overflows the reference's
         * locator (quirk Q5): refused, as every other kernel */
        bool fail = refuse || !any || (era && ne > RS_NR);
        if (!refuse && !any)
            ok = 1;

        uint32_t deg = 0;
        if (!fail) {
            /* ---- erasure locator and Berlekamp-Massey (dec1_body's wave-0
             * loop): lane i holds Lambda_i (poly and log) and B_i (log) ---- */
            uint32_t lam = lane == 0 ? 1u : 0u;
            for (uint32_t l = 0; l < ne; ++l) {
                const uint32_t xl =
                    ((P.prim * (uint32_t)(RS_NN - 1u - (s.pos[l] + (uint32_t)pad))) & 0xffffu) % 255u;
                const uint32_t prev = wave_up(lam, lane, 0u);
                lam ^= lane ? g.ex[xl + g.lg[prev]] : 0u;
            }
            uint32_t llam = g.lg[lam];
            uint32_t B = llam, Lr = ne;
            uint32_t term = g.ex[llam + s.slog[lane <= ne ? ne - lane : 63u]];
            uint32_t s1 = s.slog[lane <= ne + 1u && ne + 1u < RS_NR ? ne + 1u - lane : 63u];
            for (uint32_t r = ne + 1u; r <= RS_NR; ++r) {
                const uint32_t disc = wave_xor_v(term);
                const uint32_t bs = wave_up_old(B, ZL);
                const uint32_t ld = g.lg[disc];
                const uint32_t dq = red(ld + bs);
                const uint32_t t1 = g.ex[llam + s1], t2 = g.ex[dq + s1], up = g.ex[dq];
                s1 = s.slog[lane <= r + 1u && r + 1u < RS_NR ? r + 1u - lane : 63u];
                term = t1 ^ t2;
                const uint32_t ds = __builtin_amdgcn_readfirstlane(disc);
                const bool len = ds != 0u && 2u * Lr <= r + ne - 1u; /* uniform */
                const uint32_t bl = lam ? red(llam + 255u - ld) : ZL;
                B = len ? bl : bs;
                Lr = len ? r + ne - Lr : Lr;
                lam ^= up;
                llam = g.lg[lam];
            }
            const uint64_t nz = __ballot(co && lam != 0u);
            deg = 63u - (uint32_t)__builtin_clzll(nz); /* lane 0 holds Lambda_0 = 1 */
            s.llam[lane] = co ? llam : ZL;
            wave_sync();
            fail = deg == 0u; /* src/decode.c:108-110 */
        }

        /* ---- Chien, src/decode.c:117-145: points i = 64 k + lane + 1 ---- */
        if (!fail) {
            uint32_t total = 0;
#pragma unroll 1
            for (uint32_t k = 0; k < 4; ++k) {
                const uint32_t i = 64u * k + lane + 1u, ii = i == 255u ? 0u : i;
                uint32_t ev = 1u, ee = 0;
#pragma unroll 8
                for (uint32_t j = 1; j <= deg; ++j) {
                    ee = red(ee + ii);
                    ev ^= g.ex[s.llam[j] + ee];
                }
                const bool root = i <= 255u && ev == 0u;
                const uint64_t rb = __ballot(root);
                const uint32_t loc = (i * P.iprim + 254u) % 255u;
                if (root) {
                    const uint32_t idx = total + (uint32_t)__builtin_popcountll(rb & ((1ull << lane) - 1ull));
                    if (idx < RS_NR) {
                        s.roots[idx] = i;
                        s.locs[idx] = loc;
                    }
                }
                fail |= __ballot(root && (int32_t)loc < pad) != 0ull; /* :132-134 */
                total += (uint32_t)__builtin_popcountll(rb);
            }
            fail |= total != deg; /* src/decode.c:143-145 */
            wave_sync();
        }

        if (!fail) {
            /* ---- Omega_m = sum_(j <= m) S_(m-j) Lambda_j, m < deg: lane m
             * and lane m + 32 each take half of the terms ---- */
            const uint32_t m = lane & 31u, j0 = (lane >> 5) * 16u;
            uint32_t acc = 0;
#pragma unroll
            for (uint32_t j = j0; j < j0 + 16u; ++j) /* j > m reads slog[32..63] = ZL */
                acc ^= g.ex[s.slog[(m - j) & 63u] + s.llam[j]];
            acc ^= other_half(acc, lane);
            if (lane < RS_NR)
                s.lom[lane] = lane < deg ? (uint32_t)g.lg[acc] : ZL;
            wave_sync();

            /* ---- Forney, src/decode.c:159-191: root q = lane & 31; the low
             * half sums the numerator, the high half the denominator ---- */
            const uint32_t q = lane & 31u;
            const uint32_t rt = q < deg ? s.roots[q] : 0u, rm = rt % 255u;
            uint32_t part = 0;
            if (lane < 32u) {
#pragma unroll 8
                for (uint32_t mm = 0; mm < RS_NR; ++mm) /* Omega is ZL past deg - 1 */
                    part ^= g.ex[s.lom[mm] + (mm * rm) % 255u];
            } else {
#pragma unroll 8
                for (uint32_t h = 0; h <= 30u; h += 2u) /* Lambda is ZL past the degree */
                    part ^= g.ex[s.llam[h + 1u] + (h * rm) % 255u];
            }
            const uint32_t oth = other_half(part, lane);
            const uint32_t num = lane < 32u ? part : oth, den = lane < 32u ? oth : part;
            uint32_t mag = 0;
            if (q < deg && num) {
                const uint32_t l2 = ((uint32_t)((int32_t)rt * ((int32_t)P.fcr - 1) + (int32_t)RS_NN) & 0xffffu) % 255u;
                const uint32_t lden = den ? (uint32_t)g.lg[den] : 255u; /* no den = 0 guard */
                mag = g.ex[(g.lg[num] + l2 + RS_NN - lden) % 255u];
            }
            fixed = (uint32_t)__builtin_popcountll(__ballot(lane < 32u && q < deg && num != 0u)); /* Q6 */
            if (lane < 32u) {
                s.mags[q] = mag;
                if (q >= deg)
                    s.locs[q] = 0;
            }
            wave_sync();

            /* ---- re-syndrome check, src/decode.c:193-209 (int16 exponent,
             * uint16 gf_mod): syndrome i = lane & 31, roots split over the
             * halves ---- */
            const uint32_t i = lane & 31u, q0 = (lane >> 5) * 16u;
            const int32_t ci = (int32_t)(P.fcr + i) * (int32_t)P.prim;
            uint32_t chk = 0;
#pragma unroll 4
            for (uint32_t qq = q0; qq < q0 + 16u; ++qq) {
                const uint32_t mg = s.mags[qq];
                const int16_t k16 = (int16_t)(ci * (int32_t)(RS_NN - 1u - s.locs[qq]));
                const uint32_t x = ((uint32_t)((int32_t)g.lg[mg] + (int32_t)k16) & 0xffffu) % 255u;
                chk ^= mg ? (uint32_t)g.ex[x] : 0u;
            }
            chk ^= other_half(chk, lane);
            fail |= __ballot(lane < 32u && chk != s.spoly[i]) != 0ull;

            /* ---- apply, src/decode.c:211-227 ---- */
            if (!fail) {
                ok = 1;
                if (!era) { /* error mode: Chien locations lie in [pad, 254]: none out of range */
                    if (lane < deg) {
                        const uint32_t p = (uint32_t)((int32_t)s.locs[lane] - pad);
                        if (mag && p < L) {
                            uint8_t *d = p < size ? cdata + p : cpar + (p - size);
                            *d = (uint8_t)(*d ^ mag);
                        }
                    }
                } else {
                    /* erasure mode: magnitude q (ascending location) into slot q
                     * (Q1/Q2); slots past the codeword: parity when < size + 32
                     * (Q4), else dropped; repeated slots accumulate */
                    if (lane < deg) {
                        const uint32_t p = s.pos[lane];
                        if (mag && p < L)
                            atomicXor(&s.cw[p >> 2], mag << (8u * (p & 3u)));
                    }
                    wave_sync();
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        const uint32_t j = lane + 64u * k;
                        const uint32_t v = reinterpret_cast<const uint8_t *>(s.cw)[j];
                        if (j < L && v != w4[k]) {
                            if (j < size)
                                cdata[j] = (uint8_t)v;
                            else
                                cpar[j - size] = (uint8_t)v;
                        }
                    }
                }
            }
        }
        if (lane == 0) {
            okp[c] = (uint8_t)ok;
            if (corp)
                corp[c] = (uint8_t)fixed;
        }
        wave_sync(); /* this codeword's LDS reads before the next one's writes */
    }
}

/* the grid: eight 4-wave workgroups per CU (32 waves), fewer for a small
 * batch; workgroups past a list's length (read on the device) leave at once */
static dim3 wave_grid(size_t count, int num_cu)
{
    const size_t cap = 8u * (size_t)(num_cu > 0 ? num_cu : 256), need = (count + 3) / 4;
    return dim3((uint32_t)(need < cap ? (need ? need : 1) : cap));
}

extern "C" hipError_t rsk_wave(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride,
                               uint8_t *parity, size_t pstride, size_t count, const uint32_t *list,
                               const uint32_t *list_n, const uint8_t *syn, const uint16_t *syn16,
                               size_t syn16_stride, const uint8_t *pos8, const uint32_t *pos32, size_t pos_stride,
                               const uint8_t *cnt, uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    if (pos32)
        RS_LAUNCH(rs_wave_k<uint32_t>, wave_grid(count, num_cu), dim3(W_WG), 0, stream, tab, *prm, data, dstride,
                  parity, pstride, count, list, list_n, syn, syn16, syn16_stride, pos32, pos_stride, cnt, ok,
                  corrected);
    else
        RS_LAUNCH(rs_wave_k<uint8_t>, wave_grid(count, num_cu), dim3(W_WG), 0, stream, tab, *prm, data, dstride,
                  parity, pstride, count, list, list_n, syn, syn16, syn16_stride, pos8, pos_stride, cnt, ok,
                  corrected);
    return hipGetLastError();
}
