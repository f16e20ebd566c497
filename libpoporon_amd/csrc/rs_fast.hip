/*
 * rs_fast.hip -- RS(255,223) error-mode decode split into small kernels,
 * each small enough in LDS (<= 64 KiB) for two workgroups per CU: Chien at 8
 * waves per SIMD (<= 64 VGPRs), Forney at 6 and Berlekamp-Massey at 4 with
 * fewer instructions per term -- against the single correction kernel (rs_correct.hip,
 * 160 KiB + 128 VGPRs), whose time was half waiting on LDS results.  One
 * codeword per lane.
 *
 *   rs_bm_k      syndromes -> Berlekamp-Massey (src/decode.c:49-96) -> Lambda,
 *                degree (:98-110), Omega (:147-158)
 *   rs_chien_k   Lambda -> root map over the 255 points (:112-145)
 *   rs_forney_k  roots, Omega, Lambda -> Forney magnitudes (:159-191), apply
 *                (:215-226)
 *
 * Fast path = the codewords the reference corrects without its re-syndrome
 * check being able to fail: deg(Lambda) = L <= 16 (then Lambda has deg
 * distinct roots or the root count check fails, and Forney's magnitudes
 * reproduce every syndrome -- rs_correct.hip header).  Everything else --
 * L > 16, a locator that would grow past x^16, deg != L, deg = 0 -- is put
 * on a list that the general kernel (rs_correct_k, list mode) decodes with
 * the reference's full-length arrays and checks.  Results are bit-exact
 * either way; the list is empty for codewords with at most 16 errors.
 *
 * GF table of rs_bm_k / rs_forney_k (64 KiB; dword x * 32 + r, x < 512,
 * replica r = lane & 31 so every lane's byte reads hit bank lane & 31):
 *   byte 0     0
 *   byte 1     exp2[x]
 *   bytes 2-3  for x < 256: the "address-form" log of x, 128 log x + 4r + 1
 *              (the LDS address of this replica's exp byte of log x), and
 *              for x = 0 the zero AZ = 128 Z0 + 4r (a byte 0); 0 for x >= 256
 * exp of an address-form log a plus a plain scaled log s = 128 log is the
 * byte at a + s.  Zeros never leave the table: the plain scaled zero is
 * SZ = 128 Z0 - 1 (= log of 0 as returned by the table minus 4r + 1), and
 * with Z0 = 200 every sum with a zero operand lands on a byte 0 (AZ + s,
 * a + SZ) or on a high log byte of an entry >= 256 (AZ + SZ), all zero.
 * (Past a 64 KiB allocation a read is not reliably 0: the first bytes after
 * it return another workgroup's LDS, tools/probes/lds_oob64.hip.)  Valid
 * address-form logs are odd, zeros even.
 *
 * Chien table of rs_chien_k (65,280 B, the whole allocation): the 16-byte
 * row of term j (1..16) at 16 consecutive points, alpha^(e + j b) for
 * b = 0..15, stored at e * 256 + (j - 1) * 16.  Lane l visits the terms in
 * the order j = ((k + l) mod 16) + 1, k = 0..15, so the 16 lanes of every
 * ds_read_b128 lane group read 16 different bank slots: conflict-free
 * whatever the coefficients (the single kernel's data-dependent rows cost
 * 32 M conflict cycles per 2^20 codewords, profiles/r01_pmc_stages_v10.txt).
 */
#include <hip/hip_runtime.h>

#include <type_traits>

#include "rs_device.h"
#include "rs_gfa.h"
#include "rs_lane.h"

#define FWG 1024       /* threads per workgroup; two workgroups per CU */
#define NL 17          /* Lambda_0..16 and B_0..16: t = 16 */
#define BWG 512 /* rs_bm_k: 4 waves/SIMD, two workgroups per CU (profiles/r03_bm_value.log) */
#define BM_WAVES 4

/* Grids of up to 8 resident rounds: at 2^20 codewords every workgroup takes
 * one batch.  A persistent grid (one round, each workgroup looping) measured
 * 3-6 % slower for rs_bm_k / rs_chien_k / rs_forney_k
 * (profiles/r03_grid_rounds.log): the oldest waves win the issue arbitration,
 * finish first, and the last batches run at low occupancy. */
#define FAST_ROUNDS 8
static int fast_grid(size_t count, int num_cu)
{
    const size_t need = (count + FWG - 1) / FWG;
    const size_t g = FAST_ROUNDS * 2u * (size_t)(num_cu > 0 ? num_cu : 256);
    return (int)(need < g ? (need ? need : 1) : g);
}

/* ------------------------------------------------------------------------ */
/* rs_bm_k: Berlekamp-Massey + Omega                                         */
/* ------------------------------------------------------------------------ */

/*
 * BM in Massey's unnormalised form over address-form logs, as rs_correct.hip
 * (which shows every product equal to the reference's Karn form), with the
 * arrays cut to 17 coefficients.  The cut is exact while L <= 16 and
 * B_16..B_32 play no part: an update with B_16 != 0 (or with B's part past
 * x^16 nonzero, `bo`) would give Lambda a term past x^16, and lengthening
 * to L > 16 ends with deg != L -- all of these go to the list.
 *
 * Syndromes enter a window of 20 entries, four per block of four
 * iterations: at block q the entry e holds 128 log S_(4q+3-e), so term i of
 * iteration r = 4q+1+s reads entry 3 - s + i at a compile-time place (the
 * four iterations are unrolled; blocks are a rolled loop).  Lambda is kept
 * as the addresses of its log entries (below): 0.147 -> 0.137 ms against the
 * 4-lookup log form at 8 waves/SIMD; the same at 8, 6 or 5 waves spilled
 * (profiles/r03_bm_value.log).
 */
/* NRG: a byte-symbol code of npar < 32 roots (syndromes S_0..S_(npar-1),
 * zeros behind them): npar iterations, and the fast path needs 2L <= npar
 * besides -- the bound under which the locator's roots and Forney's
 * magnitudes reproduce every syndrome -- the rest goes to the list */
template <bool NRG>
__global__ __launch_bounds__(BWG, BM_WAVES) void rs_bm_k(const RsDevTables *__restrict__ T, const uint8_t *__restrict__ syn,
                                                   size_t count, uint8_t *__restrict__ lamo, uint8_t *__restrict__ omo,
                                                   uint8_t *__restrict__ meta, uint32_t *__restrict__ list,
                                                   uint32_t *__restrict__ nlist, uint8_t *__restrict__ ok,
                                                   uint8_t *__restrict__ corrected, uint32_t npar)
{
    __shared__ uint32_t lgf[512 * 32];
    fill_gfa<BWG>(lgf, T);
    __syncthreads();
    const GfA gf{lds_addr(lgf) + 4u * (threadIdx.x & 31u) + 1u};
    const uint32_t pofs = gf.pofs;
    const uint32_t AZ = gf.az();         /* address-form zero */
    constexpr uint32_t DQZ = SZ;         /* "no update": dq + B's logs read zeros */

    for (size_t base = (size_t)blockIdx.x * BWG; base < count; base += (size_t)gridDim.x * BWG) {
        const size_t cw = base + threadIdx.x;
        const bool valid = cw < count;
        const uint32_t *sp = reinterpret_cast<const uint32_t *>(syn + (valid ? cw : 0) * RS_NR);
        uint4 sa = make_uint4(0, 0, 0, 0), sb = sa;
        if (valid) {
            sa = reinterpret_cast<const uint4 *>(sp)[0];
            sb = reinterpret_cast<const uint4 *>(sp)[1];
        }
        const bool any = (sa.x | sa.y | sa.z | sa.w | sb.x | sb.y | sb.z | sb.w) != 0u;
        if (__ballot(any) == 0ull) { /* uniform: every codeword of the wave is clean */
            if (valid) {
                ok[cw] = 1;
                if (corrected)
                    corrected[cw] = 0;
                meta[cw] = (uint8_t)(RS_ST_DONE << 5);
            }
            continue;
        }

        /* ---- Berlekamp-Massey, src/decode.c:49-96 (error mode: r = 1..32) ---- */
        /* ---- Berlekamp-Massey, src/decode.c:49-96 (error mode: r = 1..32) ----
         * hl: Lambda_0..16 as the LDS addresses of their log entries,
         * pofs + 1 + 128 Lambda_i (bits 7..14 hold the value, the replica
         * offset sits below), so an update Lambda_i += q B_(i-1) is
         * hl ^= exp << 7 (one lookup) and Lambda's logs are one ds_read_u16
         * each, taken once per iteration for the discrepancy and B's copy: 3
         * lookups per term instead of 4.  B (address-form logs) and the
         * syndrome window one register per entry: no half-word extractions
         * (103 VGPRs, 4 waves/SIMD) */
        const uint32_t HZ = pofs + 1u; /* hl of a zero coefficient */
        uint32_t hl[NL], B[NL + 1];
        hl[0] = HZ + 128u;
#pragma unroll
        for (int i = 1; i < NL; ++i)
            hl[i] = HZ;
        B[0] = pofs;
#pragma unroll
        for (int k = 1; k <= NL; ++k)
            B[k] = AZ;
        uint32_t dl = 0, db = 0, L = 0, lb = 0, ubp = 0;
        uint32_t over = 0, bo = 0; /* 0 / 1 */
        uint32_t WL[20];
#pragma unroll
        for (int k = 0; k < 20; ++k)
            WL[k] = SZ;
        uint32_t snext = any ? sa.x : 0u; /* S_0..S_3 */

        auto step = [&](auto sc, uint32_t r) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const uint32_t ub = ubp;
            uint32_t la[NL];
            uint32_t disc = 0;
            la[0] = pofs;
#pragma unroll
            for (int g = 0; g < NL; g += 4) {
#pragma unroll
                for (int i = g; i < g + 4 && i < NL; ++i)
                    if (i > 0)
                        la[i] = AZ;
                if ((uint32_t)g <= ub) {
#pragma unroll
                    for (int i = g; i < g + 4 && i < NL; ++i) {
                        if (i > 0)
                            la[i] = lds16(hl[i]);
                        disc ^= gf.expa(la[i] + WL[3 - s + i]); /* S_(r-1-i), zero where r-1-i < 0 */
                    }
                }
            }
            const uint32_t ld = gf.logs(disc);
            const bool upd = disc != 0u;
            const bool lengthen = upd && (2u * L <= r - 1u);
            const int32_t dd = (int32_t)ld - (int32_t)lb;
            const uint32_t dq = upd ? (uint32_t)(dd < 0 ? dd + 255 * 128 : dd) : DQZ;
            const uint32_t b16 = B[NL - 1] != AZ;
            over |= upd ? (bo | b16) : 0u;
            bo = lengthen ? 0u : (bo | b16);
            /* (formed before the discrepancy instead, to overlap its lookups:
             * unchanged, profiles/r04_bm_hoist_ab.log) */
            const uint32_t up = min((uint32_t)(NL - 1), max(dl, db + 1u));
            const uint32_t ub2 = wave_max_full(up);
            ubp = ub2;
            const uint64_t lmask = __ballot(lengthen);
            static_for<0, (NL - 1) / 4 + 1, 1>([&](auto mc) __attribute__((always_inline)) {
                constexpr int m = (NL - 1) / 4 - decltype(mc)::value; /* top down */
                if ((uint32_t)(4 * m) <= ub2) {
#pragma unroll
                    for (int i = 4 * m + 3; i >= 4 * m; --i)
                        if (i > 0 && i < NL)
                            hl[i] ^= shl7(gf.expa(dq + B[i - 1]));
                    /* B_i <- lengthen ? log Lambda_i (old) : B_(i-1), top down,
                     * as VOP2 selects on VCC (the compiler's e64 selects on an
                     * SGPR mask issue at half rate; 2 %, profiles/r03_bm_vccsel.log) */
                    if constexpr (4 * m + 3 < NL) {
                        const uint32_t b0 = m > 0 ? B[m > 0 ? 4 * m - 1 : 0] : AZ;
                        asm("s_mov_b64 vcc, %8\n\t"
                            "v_cndmask_b32_e32 %3, %2, %7, vcc\n\t"
                            "v_cndmask_b32_e32 %2, %1, %6, vcc\n\t"
                            "v_cndmask_b32_e32 %1, %0, %5, vcc\n\t"
                            "v_cndmask_b32_e32 %0, %9, %4, vcc"
                            : "+v"(B[4 * m]), "+v"(B[4 * m + 1]), "+v"(B[4 * m + 2]), "+v"(B[4 * m + 3])
                            : "v"(la[4 * m]), "v"(la[4 * m + 1]), "v"(la[4 * m + 2]), "v"(la[4 * m + 3]),
                              "s"(lmask), "v"(b0)
                            : "vcc");
                    } else {
                        B[4 * m] = lengthen ? la[4 * m] : B[4 * m - 1]; /* B_16; B_17 plays no part */
                    }
                }
            });
            db = lengthen ? dl : min(db + 1u, (uint32_t)(NL - 1));
            if (upd)
                dl = up;
            if (lengthen) {
                L = r - L;
                lb = ld;
            }
        };
        const uint32_t nq = NRG ? (npar + 3u) >> 2 : RS_NR / 4;
#pragma unroll 1
        for (uint32_t q = 0; q < nq; ++q) {
            const uint32_t sd = snext;
            if (q + 1u < nq) /* uniform */
                snext = any ? sp[q + 1u] : 0u;
            /* shift the window by four entries, S_(4q+3) .. S_(4q) in front */
            const uint32_t s0 = gf.logs(sd & 0xffu), s1 = gf.logs((sd >> 8) & 0xffu);
            const uint32_t s2 = gf.logs((sd >> 16) & 0xffu), s3 = gf.logs(sd >> 24);
#pragma unroll
            for (int k = 19; k >= 4; --k)
                WL[k] = WL[k - 4];
            WL[0] = s3, WL[1] = s2, WL[2] = s1, WL[3] = s0;
            step(std::integral_constant<int, 0>{}, 4u * q + 1u);
            if (!NRG || 4u * q + 2u <= npar) /* uniform */
                step(std::integral_constant<int, 1>{}, 4u * q + 2u);
            if (!NRG || 4u * q + 3u <= npar)
                step(std::integral_constant<int, 2>{}, 4u * q + 3u);
            if (!NRG || 4u * q + 4u <= npar)
                step(std::integral_constant<int, 3>{}, 4u * q + 4u);
        }

        uint32_t al[NL]; /* address-form logs of the final Lambda */
        al[0] = pofs;
#pragma unroll
        for (int i = 1; i < NL; ++i)
            al[i] = (uint32_t)i <= ubp ? lds16(hl[i]) : AZ;
        /* ---- degree, src/decode.c:98-110 ---- */
        uint32_t deg = 0;
#pragma unroll
        for (int i = 0; i < NL; ++i)
            deg = (al[i] & 1u) ? (uint32_t)i : deg;
        const bool fast = any && !over && deg == L && deg != 0u && (!NRG || 2u * L <= npar);

        /* ---- Omega = S * Lambda mod x^deg (log form), src/decode.c:147-158 ---- */
        uint32_t ob[4] = {0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu};
        const uint32_t degmax = wave_max(fast ? deg : 0u);
        if (degmax) {
            /* S_0..S_15 again (L2): keeping them live through BM costs registers */
            const uint4 s4 = any ? reinterpret_cast<const uint4 *>(sp)[0] : make_uint4(0, 0, 0, 0);
            const uint32_t sw[4] = {s4.x, s4.y, s4.z, s4.w};
            auto omega = [&](auto dmc) __attribute__((always_inline)) {
                constexpr int DM = decltype(dmc)::value; /* > 0: every lane's bound is DM (no guards) */
                uint32_t sl[16]; /* plain scaled logs of S_0..S_15, one register each */
#pragma unroll
                for (int k = 0; k < 16; ++k)
                    sl[k] = gf.logs((sw[k >> 2] >> (8 * (k & 3))) & 0xffu);
#pragma unroll
                for (int m = 0; m < 16; ++m) {
                    if (DM ? m < DM : (uint32_t)m < degmax) {
                        uint32_t acc = 0;
#pragma unroll
                        for (int j = 0; j <= m; ++j)
                            acc ^= gf.expa(al[j] + sl[m - j]);
                        const uint32_t o = (uint32_t)m < deg ? gf.plog(gf.loga(acc)) : 255u;
                        ob[m >> 2] ^= (o ^ 0xffu) << (8 * (m & 3));
                    }
                    __builtin_amdgcn_sched_barrier(0); /* one coefficient's lookups at a time: registers */
                }
            };
            if (degmax == 16u)
                omega(std::integral_constant<int, 16>{});
            else
                omega(std::integral_constant<int, 0>{});
        }

        if (valid) {
            if (!any) {
                ok[cw] = 1;
                if (corrected)
                    corrected[cw] = 0;
                meta[cw] = (uint8_t)(RS_ST_DONE << 5);
            } else if (!fast) {
                meta[cw] = (uint8_t)(RS_ST_LIST << 5);
                list[atomicAdd(nlist, 1u)] = (uint32_t)cw;
            } else {
                uint32_t lb4[4] = {0, 0, 0, 0};
#pragma unroll
                for (int j = 1; j < NL; ++j)
                    lb4[(j - 1) >> 2] |= gf.plog(al[j]) << (8 * ((j - 1) & 3));
                reinterpret_cast<uint4 *>(lamo)[cw] = make_uint4(lb4[0], lb4[1], lb4[2], lb4[3]);
                reinterpret_cast<uint4 *>(omo)[cw] = make_uint4(ob[0], ob[1], ob[2], ob[3]);
                meta[cw] = (uint8_t)((RS_ST_FAST << 5) | deg);
            }
        }
    }
}



/* ------------------------------------------------------------------------ */
/* rs_chien_k: root map                                                      */
/* ------------------------------------------------------------------------ */

/*
 * Lambda(alpha^i'), i' = 16a + b, is 1 + sum_j row_j[e_j(a)]_b with
 * e_j(a) = (log Lambda_j + 16 a j) mod 255: 16 ds_read_b128 per 16 points.
 * Slot k of lane l holds term j_k = ((k + l) mod 16) + 1 as the LDS address
 * of its row, e * 256 + (j_k - 1) * 16, stepped by (16 j_k mod 255) * 256
 * per chunk and reduced below 255 * 256 by min(t, t - 255 * 256); a zero
 * coefficient points at the all-zero rows e = 255 and steps by 255 * 256,
 * which the reduction maps back onto itself (no read leaves the table).
 */
/* Chien point i' of flag bit b of word w (list entry 32 w + b): the flags
 * of points 16h + 4d + b' sit at bit 8b' + 7 - d - 4h, so i' = 32 w + 28 -
 * 4 (b & 7) + (b >> 3); entry 248 (bit 24 of word 7, masked as the repeat
 * of i' = 0) stands for i = 255 */
__device__ __forceinline__ uint32_t root_point(uint32_t e)
{
    return (e & 0xE0u) + 28u + ((e >> 3) & 3u) - 4u * (e & 7u);
}

__global__ __launch_bounds__(FWG, 8) void rs_chien_k(const RsDevTables *__restrict__ T, RsCorrParams P, size_t count,
                                                      const uint8_t *__restrict__ lam, uint8_t *__restrict__ meta,
                                                      uint8_t *__restrict__ roots, uint8_t *__restrict__ ok,
                                                      uint8_t *__restrict__ corrected)
{
    __shared__ uint4 lch[256 * 16];
    __shared__ uint4 lroot[FWG]; /* each lane's root list (64 + 16 KiB: two workgroups fill the 160 KiB) */
    {
        constexpr int K = 256 * 16 / FWG; /* every load first, then the stores */
        uint4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const uint32_t t = threadIdx.x + k * FWG;
            v[k] = T->chien[(t & 15u) * 256u + (t >> 4)];
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            lch[threadIdx.x + k * FWG] = v[k];
    }
    __syncthreads();
    const uint32_t cb = lds_addr(lch);
    const uint32_t lr0 = threadIdx.x & 15u;
    constexpr uint32_t WRAP = 255u * 256u;

    for (size_t base = (size_t)blockIdx.x * FWG; base < count; base += (size_t)gridDim.x * FWG) {
        const size_t cw = base + threadIdx.x;
        const bool valid = cw < count;
        const uint32_t st = valid ? meta[cw] : 0u;
        const bool fast = (st >> 5) == RS_ST_FAST;
        if (__ballot(fast) == 0ull)
            continue;
        const uint32_t deg = fast ? (st & 31u) : 0u;
        uint4 l4 = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu);
        if (fast)
            l4 = reinterpret_cast<const uint4 *>(lam)[cw];
        /* rotate the 16 log bytes by lr: byte k of R = log Lambda_(j_k) (lr
         * made opaque per codeword: hoisted, its 32 derived constants spill) */
        uint32_t lr = lr0;
        asm volatile("" : "+v"(lr));
        uint32_t D[4] = {l4.x, l4.y, l4.z, l4.w};
        uint32_t E[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            E[k] = (lr & 4u) ? D[(k + 1) & 3] : D[k];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            D[k] = (lr & 8u) ? E[(k + 2) & 3] : E[k];
        uint32_t R[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
            R[k] = __builtin_amdgcn_alignbyte(D[(k + 1) & 3], D[k], lr & 3u);
        uint32_t A[16], inc[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t jm = ((uint32_t)k + lr) & 15u; /* j_k - 1 */
            const uint32_t e = (R[k >> 2] >> (8 * (k & 3))) & 0xffu;
            A[k] = cb + (e << 8) + (jm << 4);
            inc[k] = e == 255u ? WRAP : (jm == 15u ? 256u : (jm + 1u) << 12);
        }
        /* the roots as a byte list in the lane's 16 LDS bytes, one ds_write_b8
         * per root (a register shift list cost ~30 % of the kernel's VALU in
         * the divergent loop); Forney reads them by compile-time index
         * instead of walking a bitmap (the walk cost rs_forney_k 38 of its
         * 97 us).  Entries are flag-bit indices 32 w + b (root_point()). */
        lroot[threadIdx.x] = make_uint4(0, 0, 0, 0);
        uint32_t lp = lds_addr(lroot) + 16u * threadIdx.x;
        uint32_t cnt = 0, z0 = 0;
        auto push = [&](uint32_t v) __attribute__((always_inline)) {
            lds_st8(lp, v);
            lp += 1u;
        };
#pragma unroll 1
        for (int w = 0; w < 8; ++w) {
            uint32_t word = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                uint32_t acc[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
#pragma unroll
                for (int k = 0; k < 16; k += 2) {
                    const lds_u32x4_t r1 = lds128(A[k]), r2 = lds128(A[k + 1]);
                    A[k] = chien_step<WRAP>(A[k], inc[k]);
                    A[k + 1] = chien_step<WRAP>(A[k + 1], inc[k + 1]);
                    acc[0] = xor3(acc[0], r1.x, r2.x);
                    acc[1] = xor3(acc[1], r1.y, r2.y);
                    acc[2] = xor3(acc[2], r1.z, r2.z);
                    acc[3] = xor3(acc[3], r1.w, r2.w);
                }
                /* zero bytes as flags: point 16h + 4d + b (byte b of dword d)
                 * at bit 8b + 7 - d - 4h -- shifts and 3-way ORs, no
                 * multiplies; error mode needs the roots in no order */
#pragma unroll
                for (int d = 0; d < 4; ++d)
                    word = __builtin_amdgcn_bitop3_b32(word, zero80(acc[d]) >> (d + 4 * h), 0u, 0xF0 | 0xCC);
            }
            if (w == 7)
                word &= ~(1u << 24); /* i' = 255 (point 31: bit 24) repeats i' = 0 */
            if (w == 0) {
                z0 = (word >> 7) & 1u; /* i' = 0 (bit 7) is the reference's last point, i = 255 */
                word &= ~0x80u;
            }
            cnt += __popc(word);
            const uint32_t wb = 32u * (uint32_t)w;
            while (word != 0u) { /* at most deg <= 16 pushes per lane in all */
                const uint32_t b = __builtin_ctz(word);
                word &= word - 1u;
                push(wb | b);
            }
        }
        if (z0)
            push(248u); /* flag bit 24 of word 7: root_point() = 255 */
        cnt += z0;
        const uint4 l4r = lroot[threadIdx.x];
        const uint32_t L[4] = {l4r.x, l4r.y, l4r.z, l4r.w};
        bool good = cnt == deg; /* src/decode.c:143-145 */
        if (P.pad > 0) {
            /* locations k = (i iprim - 1) mod 255 below pad fail, src/decode.c:132-134 */
            bool low = false;
#pragma unroll
            for (int n = 0; n < 16; ++n) {
                const uint32_t i = root_point((L[n >> 2] >> (8 * (n & 3))) & 0xffu);
                low |= (uint32_t)n < cnt && (int32_t)((i * P.iprim + 254u) % 255u) < P.pad;
            }
            good = good && !low;
        }
        if (fast)
            reinterpret_cast<uint4 *>(roots)[2 * cw] = make_uint4(L[0], L[1], L[2], L[3]);
        if (fast && !good) {
            {
                ok[cw] = 0;
                if (corrected)
                    corrected[cw] = 0;
                meta[cw] = (uint8_t)(RS_ST_DONE << 5);
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* rs_forney_k: magnitudes                                                   */
/* ------------------------------------------------------------------------ */

/*
 * Per root i (src/decode.c:136-138, any order: the roots are independent):
 * num = sum_m Omega_m alpha^(i m), den = sum_(2h <= dtop) Lambda_(2h+1)
 * alpha^(2h i), magnitude alpha^(log num + log alpha^(i (fcr-1)) + 255 -
 * log den) (no den = 0 guard, as the reference); a zero numerator corrects
 * nothing and is not counted.  The sums split at m = 8: one 8-step power
 * chain per root serves Omega_0..7 / Omega_8..15 and the derivative's lower
 * / upper four terms, merged by alpha^(8i) (0.062 -> 0.059 ms against the
 * even/odd chains, profiles/r03_forney_split8.log); FORNEY_R roots per step
 * (below), the logs unpacked.
 * The locations and magnitudes go out as a 32-byte record per codeword for
 * rs_apply_k.
 */
/* rs_forney_k: two roots per step at 62 VGPRs, 8 waves/SIMD in 1024-thread
 * groups: 0.0501-0.0508 vs 0.0519-0.0535 ms for four roots per step at 79
 * VGPRs, 6 waves in 768-thread groups (profiles/r05_forney_r2_ab.log; a
 * 640-thread group leaves SIMDs uneven: 0.084 ms) */
#ifndef F2WG
#define F2WG 1024
#endif
#ifndef F2_WAVES
#define F2_WAVES (F2WG / 128)
#endif
#ifndef FORNEY_R
#define FORNEY_R 2 /* roots per step */
#endif
template <bool P11>
__global__ __launch_bounds__(F2WG, F2_WAVES) void rs_forney_k(const RsDevTables *__restrict__ T, RsCorrParams P,
                                                      uint8_t *data, size_t dstride, uint8_t *parity, size_t pstride,
                                                      size_t count, const uint8_t *__restrict__ lam,
                                                      const uint8_t *__restrict__ om, uint8_t *__restrict__ roots,
                                                      const uint8_t *__restrict__ meta, uint8_t *__restrict__ ok,
                                                      uint8_t *__restrict__ corrected)
{
    __shared__ uint32_t lgf[512 * 32];
    fill_gfa<F2WG>(lgf, T);
    __syncthreads();
    const GfA gf{lds_addr(lgf) + 4u * (threadIdx.x & 31u) + 1u};
    const int32_t pad = P.pad;
    constexpr bool fcr1 = P11, iprim1 = P11;
    constexpr int R = FORNEY_R;
    const uint32_t mp = 255u * 128u + gf.pofs; /* alpha^(log a - log b) = expa(loga a - loga b + mp) */

    for (size_t base = (size_t)blockIdx.x * F2WG; base < count; base += (size_t)gridDim.x * F2WG) {
        const size_t cw = base + threadIdx.x;
        const bool valid = cw < count;
        const uint32_t st = valid ? meta[cw] : 0u;
        const bool fast = (st >> 5) == RS_ST_FAST;
        if (__ballot(fast) == 0ull)
            continue;
        const uint32_t deg = fast ? (st & 31u) : 0u;
        uint4 o4 = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0xFFFFFFFFu), l4 = o4;
        uint32_t rl[4] = {0, 0, 0, 0};
        if (fast) {
            o4 = reinterpret_cast<const uint4 *>(om)[cw];
            l4 = reinterpret_cast<const uint4 *>(lam)[cw];
            const uint4 ra = reinterpret_cast<const uint4 *>(roots)[2 * cw];
            rl[0] = ra.x, rl[1] = ra.y, rl[2] = ra.z, rl[3] = ra.w;
        }
        const uint32_t ow[4] = {o4.x, o4.y, o4.z, o4.w}, lw[4] = {l4.x, l4.y, l4.z, l4.w};
        const uint32_t dtop = deg ? (deg - 1u) & ~1u : 0u;
        uint32_t opu[16], lod[8]; /* address-form logs: Omega_m; Lambda_(2h+1) for 2h <= dtop */
#pragma unroll
        for (int m = 0; m < 16; ++m)
            opu[m] = gf.afrom((ow[m >> 2] >> (8 * (m & 3))) & 0xffu);
#pragma unroll
        for (int h = 0; h < 8; ++h)
            lod[h] = (uint32_t)(2 * h) <= dtop ? gf.afrom((lw[(2 * h) >> 2] >> (8 * ((2 * h) & 3))) & 0xffu) : gf.az();
        const uint32_t degmax = wave_max(deg);
        uint32_t posp[4] = {0, 0, 0, 0}, magp[4] = {0, 0, 0, 0};
        uint32_t fixed = 0;
#pragma unroll
        for (int n0 = 0; n0 < 16; n0 += R) {
            if ((uint32_t)n0 >= degmax) /* uniform */
                continue;
            uint32_t ir[R], si[R], s[R], num[R], den[R], nh[R], dh[R];
#pragma unroll
            for (int t = 0; t < R; ++t) {
                ir[t] = root_point((rl[(n0 + t) >> 2] >> (8 * ((n0 + t) & 3))) & 0xffu);
                si[t] = 128u * (ir[t] == 255u ? 0u : ir[t]);
                s[t] = num[t] = den[t] = nh[t] = dh[t] = 0;
            }
#pragma unroll
            for (int b = 0; b < 8; ++b) {
#pragma unroll
                for (int t = 0; t < R; ++t) {
                    num[t] ^= gf.expa(opu[b] + s[t]);
                    nh[t] ^= gf.expa(opu[b + 8] + s[t]);
                    if ((b & 1) == 0) {
                        den[t] ^= gf.expa(lod[b >> 1] + s[t]);
                        dh[t] ^= gf.expa(lod[(b >> 1) + 4] + s[t]);
                    }
                    s[t] = addmod7(s[t], si[t]);
                }
                if (b & 1) {
#pragma unroll
                    for (int t = 0; t < R; ++t)
                        asm volatile("" : "+v"(num[t]), "+v"(den[t]), "+v"(nh[t]), "+v"(dh[t]));
                    __builtin_amdgcn_sched_barrier(0); /* two powers at a time: registers */
                }
            }
#pragma unroll
            for (int t = 0; t < R; ++t) { /* s = 128 (8 i mod 255) */
                num[t] ^= gf.expa(gf.loga(nh[t]) + s[t]);
                den[t] ^= gf.expa(gf.loga(dh[t]) + s[t]);
                uint32_t mag;
                if constexpr (fcr1) {
                    /* alpha^(log num + 255 - log den) straight from the address
                     * forms: 128 (log num - log den + 255) + pofs is inside the
                     * exp table's two periods (den != 0 at the distinct roots of
                     * the fast path) */
                    mag = gf.expa(gf.loga(num[t]) - gf.loga(den[t]) + mp);
                } else {
                    const uint32_t ln2 = mod255((uint32_t)((int32_t)ir[t] * ((int32_t)P.fcr - 1) + (int32_t)RS_NN));
                    const uint32_t lden = gf.plog(gf.loga(den[t])); /* log 0 = 255 in the reference: no den = 0 guard */
                    mag = gf.exp(red(gf.plog(gf.loga(num[t])) + ln2 + RS_NN - lden));
                }
                const bool z = (uint32_t)(n0 + t) < deg && num[t] != 0u;
                fixed += z ? 1u : 0u;
                const uint32_t k = iprim1 ? ir[t] - 1u : (ir[t] * P.iprim + 254u) % 255u;
                const uint32_t p = (uint32_t)((int32_t)k - pad);
                posp[(n0 + t) >> 2] |= (p & 0xffu) << (8 * ((n0 + t) & 3));
                magp[(n0 + t) >> 2] |= (z ? mag : 0u) << (8 * ((n0 + t) & 3));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (fast) {
            uint4 *rec = reinterpret_cast<uint4 *>(roots + cw * 32u);
            rec[0] = make_uint4(posp[0], posp[1], posp[2], posp[3]);
            rec[1] = make_uint4(magp[0], magp[1], magp[2], magp[3]);
            ok[cw] = 1;
            if (corrected)
                corrected[cw] = (uint8_t)fixed;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* rs_era_bp_k: erasure decode at num_roots known positions (configs[3])    */
/* ------------------------------------------------------------------------ */

/*
 * Codewords with 32 erasures (= num_roots) in strictly ascending slots inside
 * the codeword, prim = 1.  Berlekamp-Massey does not run (src/decode.c:53-55:
 * r starts at the erasure count), so Lambda is the erasure locator
 * prod(1 + X_l x) of :31-47, X_l = alpha^(254 - L_l), L_l = slot + pad, of
 * degree 32 (every X_l nonzero).  Its roots are the Chien points (:117-141)
 * i_l = L_l + 1, found in ascending order = slot order, so magnitude l goes
 * to slot l (:211-214), and the count equals the degree.  Everything else --
 * other counts, unsorted or repeated slots, slots past the codeword -- is
 * left to the errata kernels (RS_ST_PEND) or goes to the list (rs_correct_k
 * in record mode).  Output: the 64-byte record of rs_apply_k<32> (slots,
 * magnitudes).  The round-3 kernel that ran the locator, Omega and Forney
 * here: profiles/experiments/rs_era_forney_k.hip.txt.
 */
/*
 * The magnitudes are solved directly.  With 32 erasures the 32 syndromes determine them: S_i =
 * sum_l z_l X_l^i (i < 32, z_l = Y_l X_l^fcr) is a square Vandermonde system
 * with distinct nodes, whatever the syndromes are, and the reference's
 * Forney step (src/decode.c:159-191) computes its unique solution (its
 * re-syndrome check passes by construction; for the parameters that reach
 * this kernel -- RsCorrParams.vfast, prim 1 -- its uint16 exponent of
 * alpha^(root (fcr-1)) does not wrap).  So any exact solver gives the
 * reference's bytes: here the Bjorck-Pereyra algorithm for the primal
 * Vandermonde system (Golub & Van Loan, Alg. 4.6.2), in GF(2^8):
 *
 *   for k = 0..30:     for i = 31 down to k+1:  b_i ^= X_k b_(i-1)
 *   for k = 30 .. 0:   for i = k+1 .. 31:       b_i /= X_i ^ X_(i-k-1)
 *                      for i = k .. 30:         b_i ^= b_(i+1)
 *
 * then Y_l = z_l X_l^-fcr = alpha^(log z_l + fcr (slot_l + pad + 1)).  Per
 * codeword 496 multiply-adds (2 lookups, 3 VALU) and 496 divisions (3
 * lookups, 6 VALU) + 496 XORs, against the locator (831 lookups), Omega (528)
 * and Forney (1,536) of the Forney route.  The b_i and X_l live as
 * "log-entry addresses" hz | v << 7 (GfA::hz): a log is one ds_read_u16 at
 * that address, an XOR of two values is one v_bitop3 ((A ^ B) | hz), and a
 * division b / D is alpha^(log b - log D) read at loga(b) - loga(D) + pofs +
 * 255 * 128 (a zero b lands on a byte 0 of the table, no test).
 * (Prototype against the oracle over fcr 0, 1, 2, 5, 97, sizes 223 and 100,
 * extra errors besides the erasures: bit-exact.)
 */
#ifndef BPWG
#define BPWG 1024 /* rs_era_bp_k: 4 waves/SIMD at 120 VGPRs; 5 or 6 (640- / 768-thread groups) spill 14 / 47 */
#endif
#ifndef BP_WAVES
#define BP_WAVES 4
#endif
__global__ __launch_bounds__(BPWG, BP_WAVES) void rs_era_bp_k(const RsDevTables *__restrict__ T, RsCorrParams P,
                                                            const uint8_t *__restrict__ syn,
                                                            const uint8_t *__restrict__ pos8, size_t pos_stride,
                                                            const uint8_t *__restrict__ cntp, size_t count,
                                                            uint8_t *__restrict__ rec, uint8_t *__restrict__ meta,
                                                            uint32_t *__restrict__ list, uint32_t *__restrict__ nlist,
                                                            uint8_t *__restrict__ ok, uint8_t *__restrict__ corrected,
                                                            uint32_t pend)
{
    __shared__ uint32_t lgf[512 * 32];
    fill_gfa<BPWG>(lgf, T);
    __syncthreads();
    const GfA gf{lds_addr(lgf) + 4u * (threadIdx.x & 31u) + 1u};
    const uint32_t pofs = gf.pofs, hz = gf.hz();
    const uint32_t lim = P.size + RS_NR, pad = (uint32_t)P.pad;

    uint32_t it = 0;
    for (size_t base = (size_t)blockIdx.x * BPWG; base < count; base += (size_t)gridDim.x * BPWG, ++it) {
        prio_by_progress(it);
        const size_t cw = base + threadIdx.x;
        const bool valid = cw < count;
        uint4 sa = make_uint4(0, 0, 0, 0), sb = sa, pa = sa, pb = sa;
        uint32_t ne = 0;
        const uint8_t *slots = pos8 + (valid ? cw : 0) * pos_stride;
        if (valid) {
            sa = reinterpret_cast<const uint4 *>(syn)[2 * cw];
            sb = reinterpret_cast<const uint4 *>(syn)[2 * cw + 1];
            pa = reinterpret_cast<const uint4 *>(slots)[0];
            pb = reinterpret_cast<const uint4 *>(slots)[1];
            ne = cntp[cw];
        }
        const bool any = (sa.x | sa.y | sa.z | sa.w | sb.x | sb.y | sb.z | sb.w) != 0u;
        uint32_t pk[RS_NR / 4] = {pa.x, pa.y, pa.z, pa.w, pb.x, pb.y, pb.z, pb.w};
        bool asc = true;
        uint32_t prev = pk[0] & 0xffu;
#pragma unroll
        for (int n = 1; n < RS_NR; ++n) {
            const uint32_t p = (pk[n >> 2] >> (8 * (n & 3))) & 0xffu;
            asc = asc && p > prev;
            prev = p;
        }
        const bool fast = valid && any && ne == RS_NR && asc && prev < lim;
        if (valid && !fast) {
            if (!any) {
                ok[cw] = 1;
                if (corrected)
                    corrected[cw] = 0;
                meta[cw] = (uint8_t)(RS_ST_DONE << 5);
            } else if (pend) { /* the errata kernels (rs_errata.hip) decode it */
                meta[cw] = (uint8_t)(RS_ST_PEND << 5);
            } else {
                meta[cw] = (uint8_t)(RS_ST_LIST << 5);
                list[atomicAdd(nlist, 1u)] = (uint32_t)cw;
            }
        }
        const uint64_t pw = __ballot(valid && any && !fast && pend);
        if (pw != 0ull && (threadIdx.x & 63u) == (uint32_t)__builtin_ctzll(pw))
            nlist[1] = 1u; /* the errata kernels run only if some codeword is pending: one store per wave */
        if (__ballot(fast) == 0ull) /* uniform */
            continue;
        uint32_t *recw = reinterpret_cast<uint32_t *>(rec + (valid ? cw : 0) * 64u);
        if (fast) { /* the record's slots */
            reinterpret_cast<uint4 *>(recw)[0] = pa;
            reinterpret_cast<uint4 *>(recw)[1] = pb;
        }
        if (!fast) { /* lanes along for the ride: distinct in-range nodes (no division by zero matters) */
#pragma unroll
            for (int k = 0; k < RS_NR / 4; ++k)
                pk[k] = 0x03020100u + 0x04040404u * (uint32_t)k;
        }
        auto slot = [&](int l) __attribute__((always_inline)) { return (pk[l >> 2] >> (8 * (l & 3))) & 0xffu; };

        /* b_i = S_i and X_l as log-entry addresses */
        uint32_t hb[RS_NR], hx[RS_NR];
        {
            const uint32_t sw[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
#pragma unroll
            for (int i = 0; i < RS_NR; ++i)
                hb[i] = hz | (((sw[i >> 2] >> (8 * (i & 3))) & 0xffu) << 7);
        }
#pragma unroll
        for (int l = 0; l < RS_NR; ++l)
            hx[l] = hz | shl7(gf.exp(RS_NN - 1u - (slot(l) + pad))); /* X_l = alpha^(254 - (slot + pad)) */

#pragma unroll
        for (int k = 0; k < RS_NR / 4; ++k)
            asm volatile("" : "+v"(pk[k]));
        /* stage 1: b_i ^= X_k b_(i-1), i descending (each log taken of the old b_(i-1)) */
        static_for<0, RS_NR - 1, 1>([&](auto kc) __attribute__((always_inline)) {
            constexpr int k = decltype(kc)::value;
            const uint32_t xs = 128u * (RS_NN - 1u - (slot(k) + pad)); /* plain scaled log X_k */
            static_for<0, RS_NR - 1 - k, 1>([&](auto jc) __attribute__((always_inline)) {
                constexpr int j = decltype(jc)::value, i = RS_NR - 1 - j;
                hb[i] ^= shl7(gf.expa(gf.logh(hb[i - 1]) + xs));
                if constexpr ((j & 7) == 7)
                    __builtin_amdgcn_sched_barrier(0); /* eight terms at a time: registers */
            });
            __builtin_amdgcn_sched_barrier(0); /* one pass at a time: registers */
        });
        /* stage 2: b_i /= X_i ^ X_(i-k-1) for i > k, then b_i ^= b_(i+1) ascending */
        static_for<0, RS_NR - 1, 1>([&](auto qc) __attribute__((always_inline)) {
            constexpr int k = RS_NR - 2 - decltype(qc)::value;
            static_for<k + 1, RS_NR, 1>([&](auto ic) __attribute__((always_inline)) {
                constexpr int i = decltype(ic)::value;
                const uint32_t hd = __builtin_amdgcn_bitop3_b32(hx[i], hx[i - k - 1], hz, 0xBE); /* (A ^ B) | C */
                const uint32_t e = gf.expa(gf.logh(hb[i]) - gf.logh(hd) + pofs + 255u * 128u);
                hb[i] = hz | shl7(e);
                if constexpr (((i - k) & 7) == 0)
                    __builtin_amdgcn_sched_barrier(0); /* eight divisions at a time: registers */
            });
            static_for<k, RS_NR - 1, 1>([&](auto ic) __attribute__((always_inline)) {
                constexpr int i = decltype(ic)::value;
                hb[i] = __builtin_amdgcn_bitop3_b32(hb[i], hb[i + 1], hz, 0xBE);
            });
            __builtin_amdgcn_sched_barrier(0);
        });

        /* Y_l = alpha^(log z_l + fcr (slot_l + pad + 1)); z_l = 0: no correction,
         * not counted.  The slots re-extracted here (opaque): kept from the
         * start, their 32 bytes spilled */
#pragma unroll
        for (int k = 0; k < RS_NR / 4; ++k)
            asm volatile("" : "+v"(pk[k]));
        uint32_t ncor = 0, mrec[RS_NR / 4];
        const uint32_t fcr = P.fcr; /* < 98 here (vfast): (slot + pad + 1) fcr < 2^16 */
#pragma unroll
        for (int l = 0; l < RS_NR; ++l) {
            const uint32_t x = (slot(l) + pad + 1u) * fcr; /* the Chien point 1..255, times fcr */
            const uint32_t ys = 128u * red((x & 0xffu) + (x >> 8)); /* 128 (x mod 255) */
            const uint32_t mag = gf.expa(gf.logh(hb[l]) + ys);
            ncor += hb[l] != hz ? 1u : 0u;
            if ((l & 3) == 0)
                mrec[l >> 2] = mag;
            else
                mrec[l >> 2] |= mag << (8 * (l & 3));
        }
        if (fast) {
            reinterpret_cast<uint4 *>(recw)[2] = make_uint4(mrec[0], mrec[1], mrec[2], mrec[3]);
            reinterpret_cast<uint4 *>(recw)[3] = make_uint4(mrec[4], mrec[5], mrec[6], mrec[7]);
            meta[cw] = (uint8_t)(RS_ST_FAST << 5);
            ok[cw] = 1;
            if (corrected)
                corrected[cw] = (uint8_t)ncor;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* rs_apply_k: the corrections, src/decode.c:215-226                         */
/* ------------------------------------------------------------------------ */

/*
 * One wave per 64 codewords.  Wire layout (255-byte rows back to back, data
 * 16-byte aligned), whole waves: the wave's 16,320-byte block is read into
 * LDS with coalesced 16-byte loads, each lane XORs its codeword's magnitudes
 * in (ds_xor_b32), and the block is written back the same way -- 2 x 16 memory
 * requests per wave-instruction row instead of one request per corrected
 * byte (scattered byte read-modify-writes measured 0.15 ms per 2^20
 * codewords with 16 errors, bound by the L2's request rate).  The block's
 * loads and stores are non-temporal: the codewords are not read again by
 * this decode, and the dirty lines written back here rather than evicted by
 * the next kernel's stream measured the following encode 0.100 vs 0.109 ms
 * and the round trip +2 % (profiles/r03_apply_nt_ab.log).  Other layouts
 * and a batch's last partial wave correct byte by byte.  Locations are
 * distinct (distinct roots), so the order of the corrections is immaterial.
 */
#define AWG 256                 /* 4 waves, 16,320 B of LDS each */
#define ABLK (64u * 255u / 16u) /* 16-byte chunks per wave block: 1020 */

template <int NC> /* corrections per record: 16 (error mode) or 32 (erasure mode) */
__global__ __launch_bounds__(AWG) void rs_apply_k(const uint8_t *__restrict__ meta, const uint8_t *__restrict__ rec,
                                                  uint8_t *data, size_t dstride, uint8_t *parity, size_t pstride,
                                                  uint32_t size, size_t count, uint32_t wire, uint32_t npar)
{
    constexpr int NW = NC / 4; /* record dwords of positions (then as many of magnitudes) */
    __shared__ uint4 img[AWG / 64][ABLK];
    const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    /* last blocks first: the codewords the syndrome pass read last may still sit in the MALL */
    const size_t base = ((size_t)(gridDim.x - 1u - blockIdx.x) * (AWG / 64) + w) * 64u;
    if (base >= count)
        return;
    const size_t cw = base + lane;
    const bool valid = cw < count;
    const bool fast = valid && (meta[cw] >> 5) == RS_ST_FAST;
    uint32_t pw[NW], mw[NW];
#pragma unroll
    for (int k = 0; k < NW; ++k)
        pw[k] = mw[k] = 0;
    if (fast) {
        const uint4 *r = reinterpret_cast<const uint4 *>(rec + cw * (2u * NC));
#pragma unroll
        for (int k = 0; k < NW / 4; ++k) {
            const uint4 a = r[k], b = r[NW / 4 + k];
            pw[4 * k] = a.x, pw[4 * k + 1] = a.y, pw[4 * k + 2] = a.z, pw[4 * k + 3] = a.w;
            mw[4 * k] = b.x, mw[4 * k + 1] = b.y, mw[4 * k + 2] = b.z, mw[4 * k + 3] = b.w;
        }
    }
    if (__ballot(fast) == 0ull)
        return;
    /* positions past the codeword (erasure slots, clamped to 255) are never written */
    const uint32_t lim = size + npar;
    if (wire && base + 64u <= count) { /* uniform */
        const uint4 *src = reinterpret_cast<const uint4 *>(data + base * 255u);
        uint4 *dst = reinterpret_cast<uint4 *>(data + base * 255u);
        uint4 *im = img[w];
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t c = lane + 64u * k;
            if (c < ABLK) {
                const lds_u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const lds_u32x4_t *>(src + c));
                im[c] = make_uint4(v.x, v.y, v.z, v.w);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t *imw = reinterpret_cast<uint32_t *>(im);
#pragma unroll
        for (int n = 0; n < NC; ++n) {
            const uint32_t mg = (mw[n >> 2] >> (8 * (n & 3))) & 0xffu;
            const uint32_t p = (pw[n >> 2] >> (8 * (n & 3))) & 0xffu;
            if (mg && p < lim) {
                const uint32_t b = lane * 255u + p;
                atomicXor(imw + (b >> 2), mg << (8u * (b & 3u)));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
        for (uint32_t k = 0; k < 16; ++k) {
            const uint32_t c = lane + 64u * k;
            if (c < ABLK) {
                const uint4 v = im[c];
                __builtin_nontemporal_store(lds_u32x4_t{v.x, v.y, v.z, v.w}, reinterpret_cast<lds_u32x4_t *>(dst + c));
            }
        }
    } else if (fast) {
        uint8_t *cdata = data + cw * dstride, *cpar = parity + cw * pstride;
#pragma unroll
        for (int n = 0; n < NC; ++n) {
            const uint32_t mg = (mw[n >> 2] >> (8 * (n & 3))) & 0xffu;
            const uint32_t p = (pw[n >> 2] >> (8 * (n & 3))) & 0xffu;
            if (mg && p < lim) {
                uint8_t *d = p < size ? cdata + p : cpar + (p - size);
                *d = (uint8_t)(*d ^ mg); /* in slot order: repeated slots accumulate */
            }
        }
    }
}

/* ------------------------------------------------------------------------ */
/* launchers                                                                 */
/* ------------------------------------------------------------------------ */

extern "C" hipError_t rsk_bm(const RsDevTables *tab, const RsSplitWs *ws, size_t count, uint8_t *ok,
                             uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const size_t need = (count + BWG - 1) / BWG,
                 res = FAST_ROUNDS * (size_t)(num_cu > 0 ? num_cu : 256) * (BM_WAVES * 256 / BWG);
    RS_LAUNCH(rs_bm_k<false>, dim3((uint32_t)(need < res ? need : res)), dim3(BWG), 0, stream, tab, ws->syn, count,
              ws->lam, ws->om, ws->meta, ws->list, ws->nlist, ok, corrected, (uint32_t)RS_NR);
    return hipGetLastError();
}

extern "C" hipError_t rsk_bm_nr(const RsDevTables *tab, const RsSplitWs *ws, size_t count, uint32_t npar, uint8_t *ok,
                                uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const size_t need = (count + BWG - 1) / BWG,
                 res = FAST_ROUNDS * (size_t)(num_cu > 0 ? num_cu : 256) * (BM_WAVES * 256 / BWG);
    RS_LAUNCH(rs_bm_k<true>, dim3((uint32_t)(need < res ? need : res)), dim3(BWG), 0, stream, tab, ws->syn, count,
              ws->lam, ws->om, ws->meta, ws->list, ws->nlist, ok, corrected, npar);
    return hipGetLastError();
}

extern "C" hipError_t rsk_chien(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, size_t count,
                                uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rs_chien_k, dim3(fast_grid(count, num_cu)), dim3(FWG), 0, stream, tab, *prm, count, ws->lam,
                       ws->meta, ws->roots, ok, corrected);
    return hipGetLastError();
}

extern "C" hipError_t rsk_forney(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, uint8_t *data,
                                 size_t dstride, uint8_t *parity, size_t pstride, size_t count, uint8_t *ok,
                                 uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const size_t need = (count + F2WG - 1) / F2WG, cap = FAST_ROUNDS * 2u * (size_t)(num_cu > 0 ? num_cu : 256);
    const dim3 grid((uint32_t)(need < cap ? need : cap));
    if (prm->fcr == 1u && prm->iprim == 1u)
        RS_LAUNCH(rs_forney_k<true>, grid, dim3(F2WG), 0, stream, tab, *prm, data, dstride, parity, pstride, count,
                  ws->lam, ws->om, ws->roots, ws->meta, ok, corrected);
    else
        RS_LAUNCH(rs_forney_k<false>, grid, dim3(F2WG), 0, stream, tab, *prm, data, dstride, parity, pstride, count,
                  ws->lam, ws->om, ws->roots, ws->meta, ok, corrected);
    return hipGetLastError();
}

/* wire: 255-byte rows back to back (size + npar = 255, parity right after
 * the data), 16-byte aligned */
template <int NC>
static hipError_t apply_launch(const RsCorrParams *prm, const uint8_t *meta, const uint8_t *rec, uint8_t *data,
                               size_t dstride, uint8_t *parity, size_t pstride, size_t count, hipStream_t stream,
                               uint32_t npar = RS_NR)
{
    if (count == 0)
        return hipSuccess;
    const uint32_t wire = prm->size + npar == 255u && dstride == 255u && pstride == 255u &&
                          parity == data + prm->size && (reinterpret_cast<uintptr_t>(data) & 15u) == 0u;
    const size_t waves = (count + 63) / 64;
    RS_LAUNCH(rs_apply_k<NC>, dim3((uint32_t)((waves + AWG / 64 - 1) / (AWG / 64))), dim3(AWG), 0, stream,
                       meta, rec, data, dstride, parity, pstride, prm->size, count, wire, npar);
    return hipGetLastError();
}

extern "C" hipError_t rsk_apply(const RsCorrParams *prm, const RsSplitWs *ws, uint8_t *data, size_t dstride,
                                uint8_t *parity, size_t pstride, size_t count, hipStream_t stream)
{
    return apply_launch<16>(prm, ws->meta, ws->roots, data, dstride, parity, pstride, count, stream);
}

extern "C" hipError_t rsk_apply_nr(const RsCorrParams *prm, const RsSplitWs *ws, uint8_t *data, size_t dstride,
                                   uint8_t *parity, size_t pstride, size_t count, uint32_t npar, hipStream_t stream)
{
    return apply_launch<16>(prm, ws->meta, ws->roots, data, dstride, parity, pstride, count, stream, npar);
}

extern "C" hipError_t rsk_apply_era_nr(const RsCorrParams *prm, const uint8_t *meta, const uint8_t *rec, uint8_t *data,
                                       size_t dstride, uint8_t *parity, size_t pstride, size_t count, uint32_t npar,
                                       hipStream_t stream)
{
    return apply_launch<32>(prm, meta, rec, data, dstride, parity, pstride, count, stream, npar);
}

extern "C" hipError_t rsk_apply_era(const RsCorrParams *prm, const uint8_t *meta, const uint8_t *rec, uint8_t *data,
                                    size_t dstride, uint8_t *parity, size_t pstride, size_t count, hipStream_t stream)
{
    return apply_launch<32>(prm, meta, rec, data, dstride, parity, pstride, count, stream);
}

extern "C" hipError_t rsk_era(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, const uint8_t *pos8,
                              size_t pos_stride, const uint8_t *cnt, size_t count, uint8_t *ok, uint8_t *corrected,
                              uint32_t pend, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const size_t need = (count + BPWG - 1) / BPWG, /* persistent (more rounds measured slower for rs_era_k) */
                 res = (size_t)(num_cu > 0 ? num_cu : 256) * (BP_WAVES * 256 / BPWG);
    RS_LAUNCH(rs_era_bp_k, dim3((uint32_t)(need < res ? need : res)), dim3(BPWG), 0, stream, tab, *prm, ws->syn,
              pos8, pos_stride, cnt, count, ws->ext, ws->meta, ws->list, ws->nlist, ok, corrected, pend);
    return hipGetLastError();
}
