/*
 * rs_errata.hip -- split errata decode of RS(255,223) on gfx950: erasure mode
 * with any erasure count and errors besides (src/decode.c:17-230 with
 * erasure_count > 0), one codeword per lane:
 *
 *   rs_ebm_k       erasure locator (src/decode.c:31-47), Berlekamp-Massey from
 *                  r = count + 1 (:49-96, the length rule 2L <= r + e - 1),
 *                  degree (:98-110), Omega = S Lambda mod x^deg (:147-158)
 *   rs_chien32_k   roots of Lambda, degree <= 32 (:112-145)
 *   rs_forney32_k  magnitudes (:159-191) as 64-byte records: root n (in the
 *                  reference's ascending order) with list slot n (:211-214)
 *
 * then rs_apply_k<32> (rs_fast.hip) XORs the records in.  rs_era_bp_k serves
 * the one case with its own closed form (32 sorted erasures, prim 1); this
 * path serves the rest: 1..31 erasures with or without errors, unsorted or
 * repeated slots, and the zero-count erasure mode (quirk Q3).
 *
 * Fast path = the codewords whose Berlekamp-Massey ends with deg(Lambda) =
 * L and whose Chien search finds deg roots: then BM has made every
 * discrepancy from r = L to 31 zero, Omega = S Lambda mod x^32 has degree <
 * deg, and the partial fractions of Omega / Lambda reproduce S_0..S_31 from
 * Forney's magnitudes, so the reference's re-syndrome check (:193-209)
 * passes (the rs_correct.hip header argues the error-mode case the same
 * way).  deg != L, more than 32 erasures, or a slot past the codeword go to
 * the general kernel's list (rsk_correct_era_list); a root count != deg is
 * the reference's failure (:143-145) and finishes here.  Results are
 * bit-exact either way.
 *
 * Arrays are full length (Lambda_0..32, B_0..32), so BM needs ~120 VGPRs:
 * 4 waves/SIMD, one 1024-thread workgroup per CU.  Ablations (round 3,
 * 16 erasures + 8 errors): BM ~60 % of rs_ebm_k, Omega ~13 %.
 */
#include <hip/hip_runtime.h>

#include "rs_device.h"
#include "rs_gfa.h"
#include "rs_lane.h"

#define XWG 1024 /* threads per workgroup, one workgroup per CU (4 waves/SIMD) */
#define XL 33    /* Lambda_0..32 */
#define XR 4     /* Forney roots per step */

static int errata_grid(size_t count, int num_cu)
{
    const size_t need = (count + XWG - 1) / XWG;
    const size_t g = (size_t)(num_cu > 0 ? num_cu : 256);
    return (int)(need < g ? (need ? need : 1) : g);
}

/* ------------------------------------------------------------------------ */
/* rs_ebm_k: erasure locator, Berlekamp-Massey, Omega                        */
/* ------------------------------------------------------------------------ */

/*
 * Address-form logs as rs_bm_k (rs_fast.hip header), Lambda kept as the
 * addresses of its log entries (GfA::hz): an update Lambda_j += q B_(j-1) is
 * one lookup (B is kept in logs) and the logs of Lambda are taken once per
 * iteration (one ds_read_u16 each), for the discrepancy and B's copy.  The erasure locator is built factor by factor, Lambda_j += X_l
 * Lambda_(j-1) top down (two lookups per coefficient); lanes past their
 * count multiply by zero.  BM
 * then runs from the wave's smallest count: a lane is active from r = its
 * count + 1 (before that its Lambda and B stay as they are).  Massey's
 * unnormalised form with B = the erasure locator and b = 1 at the start, as
 * rs_correct_k.  The syndrome window holds 36 u16 entries (18 VGPRs): at
 * block q entry e = 128 log S_(4q+3-e), so term i of iteration r = 4q+1+s
 * reads entry 3 - s + i.
 */
__global__ __launch_bounds__(XWG, 4) void rs_ebm_k(const RsDevTables *__restrict__ T, RsCorrParams P,
                                                  const uint8_t *__restrict__ syn, const uint8_t *__restrict__ pos8,
                                                  size_t pos_stride, const uint8_t *__restrict__ cntp, size_t count,
                                                  uint8_t *__restrict__ ext, uint8_t *__restrict__ meta,
                                                  uint32_t *__restrict__ list, uint32_t *__restrict__ nlist,
                                                  uint8_t *__restrict__ ok, uint8_t *__restrict__ corrected,
                                                  uint32_t only_pend, uint32_t npar)
{
    if (only_pend && nlist[1] == 0u) /* rs_era_bp_k decoded every codeword */
        return;
    __shared__ uint32_t lgf[512 * 32];
    fill_gfa<XWG>(lgf, T);
    __syncthreads();
    const GfA gf{lds_addr(lgf) + 4u * (threadIdx.x & 31u) + 1u};
    const uint32_t pofs = gf.pofs;
    const uint32_t AZ = gf.az();
    constexpr uint32_t DQZ = SZ; /* "no update": dq + B's logs read zeros */
    const uint32_t lim = P.size + npar, pad = (uint32_t)P.pad;

    uint32_t it = 0;
    for (size_t base = (size_t)blockIdx.x * XWG; base < count; base += (size_t)gridDim.x * XWG, ++it) {
        prio_by_progress(it);
        const size_t cw = base + threadIdx.x;
        const bool valid = cw < count && (!only_pend || (meta[cw] >> 5) == RS_ST_PEND);
        const uint32_t *sp = reinterpret_cast<const uint32_t *>(syn + (valid ? cw : 0) * RS_NR);
        uint4 sa = make_uint4(0, 0, 0, 0), sb = sa;
        uint32_t ne = 0;
        uint32_t pk[RS_NR / 4] = {0, 0, 0, 0, 0, 0, 0, 0}; /* slots 0..31, four per register */
        if (valid) {
            sa = reinterpret_cast<const uint4 *>(sp)[0];
            sb = reinterpret_cast<const uint4 *>(sp)[1];
            ne = cntp[cw];
            const uint32_t *pw = reinterpret_cast<const uint32_t *>(pos8 + cw * pos_stride);
#pragma unroll
            for (int k = 0; k < RS_NR / 4; ++k)
                if (4u * k < npar) /* uniform: the row holds npar slots (a code of npar < 32 roots) */
                    pk[k] = pw[k];
        }
        const bool any = (sa.x | sa.y | sa.z | sa.w | sb.x | sb.y | sb.z | sb.w) != 0u;
        bool inside = true; /* every erasure slot inside the codeword: L_l = slot + pad <= 254 */
#pragma unroll
        for (int n = 0; n < RS_NR; ++n)
            inside = inside && ((uint32_t)n >= ne || ((pk[n >> 2] >> (8 * (n & 3))) & 0xffu) < lim);
        const bool elig = valid && any && ne <= npar && inside;
        if (valid && !any) { /* zero syndromes: success whatever the list says (src/decode.c:468) */
            ok[cw] = 1;
            if (corrected)
                corrected[cw] = 0;
            meta[cw] = (uint8_t)(RS_ST_DONE << 5);
        } else if (valid && !elig) {
            meta[cw] = (uint8_t)(RS_ST_LIST << 5);
            list[atomicAdd(nlist, 1u)] = (uint32_t)cw;
        }
        if (__ballot(elig) == 0ull) /* uniform */
            continue;
        if (!elig)
            ne = 0;

        /* ---- erasure locator, src/decode.c:31-47 ---- */
        /* lv: Lambda_0..32 as log-entry addresses (GfA::hz; Lambda_0 = 1 is
         * never updated); a product term needs the log of the old
         * coefficient only, so an update is two lookups (log, exp) */
        const uint32_t HZ = gf.hz();
        uint32_t lv[XL];
        lv[0] = HZ + 128u;
#pragma unroll
        for (int i = 1; i < XL; ++i)
            lv[i] = HZ;
        const uint32_t nemax = wave_max_full(ne);
        {
            uint32_t q[RS_NR / 4]; /* slots shifted down one byte per factor */
#pragma unroll
            for (int k = 0; k < RS_NR / 4; ++k)
                q[k] = pk[k];
#pragma unroll 1
            for (uint32_t l = 0; l < nemax; ++l) { /* uniform */
                const uint32_t p = q[0] & 0xffu;
#pragma unroll
                for (int k = 0; k < RS_NR / 4 - 1; ++k)
                    q[k] = __builtin_amdgcn_alignbyte(q[k + 1], q[k], 1);
                q[RS_NR / 4 - 1] >>= 8;
                /* scaled log of X_l = alpha^(prim (254 - L_l)); zero past the count */
                const uint32_t xs = l < ne ? 128u * ((P.prim * (RS_NN - 1u - (p + pad))) % RS_NN) : SZ;
                /* Lambda_j += X_l Lambda_(j-1), j = l+1 .. 1 (top down: old Lambda_(j-1)) */
#pragma unroll
                for (int g = XL - 1; g >= 1; g -= 4) {
                    if ((uint32_t)(g - 3) <= l + 1u) { /* uniform */
#pragma unroll
                        for (int j = g; j > g - 4 && j >= 1; --j)
                            lv[j] ^= shl7(gf.expa((j == 1 ? pofs : gf.logh(lv[j - 1])) + xs));
                    }
                }
            }
        }

        /* ---- Berlekamp-Massey, src/decode.c:49-96 ---- */
        uint32_t BP[(XL + 1) / 2]; /* B_0..B_33 address-form, two per register (B_33 stays zero) */
        {
            uint32_t gl[XL];
            gl[0] = pofs;
#pragma unroll
            for (int i = 1; i < XL; ++i)
                gl[i] = (uint32_t)i <= nemax ? gf.logh(lv[i]) : AZ; /* Gamma has degree <= nemax */
#pragma unroll
            for (int k = 0; k < (XL + 1) / 2; ++k)
                BP[k] = gl[2 * k] | ((2 * k + 1 < XL ? gl[2 * k + 1] : AZ) << 16);
        }
        uint32_t dl = ne, db = ne, L = ne, lb = 0;
        const uint32_t nemin = 63u - wave_max_full(63u - (elig ? ne : 63u));
        uint32_t WL[18];
#pragma unroll
        for (int k = 0; k < 18; ++k)
            WL[k] = SZ | (SZ << 16);
        auto step = [&](auto sc, uint32_t r) __attribute__((always_inline)) {
            constexpr int s = decltype(sc)::value;
            const bool act = elig && r > ne && r <= npar;
            const uint32_t ub = wave_max_full(act ? dl : 0u);
            /* logs of the old coefficients: the discrepancy's terms and B's copy;
             * AZ above the wave's degree bound (those coefficients are zero) */
            uint32_t la[XL];
            la[0] = pofs;
#pragma unroll
            for (int g = 0; g < XL; g += 4) {
#pragma unroll
                for (int i = g; i < g + 4 && i < XL; ++i)
                    if (i > 0)
                        la[i] = AZ;
                if ((uint32_t)g <= ub) {
#pragma unroll
                    for (int i = g; i < g + 4 && i < XL; ++i)
                        if (i > 0)
                            la[i] = gf.logh(lv[i]);
                }
            }
            uint32_t disc = 0;
#pragma unroll
            for (int g = 0; g < XL; g += 4) {
                if ((uint32_t)g <= ub) {
#pragma unroll
                    for (int i = g; i < g + 4 && i < XL; ++i)
                        disc ^= gf.expa(la[i] + half(WL, 3 - s + i)); /* S_(r-1-i) */
                }
            }
            const uint32_t ld = gf.logs(disc);
            const bool upd = act && disc != 0u;
            const bool lengthen = upd && (2u * L <= r + ne - 1u);
            const int32_t dd = (int32_t)ld - (int32_t)lb;
            const uint32_t dq = upd ? (uint32_t)(dd < 0 ? dd + 255 * 128 : dd) : DQZ;
            const uint32_t up = min((uint32_t)(XL - 1), max(dl, db + 1u));
            const uint32_t ub2 = wave_max_full(act ? up : 0u);
#pragma unroll
            for (int m = (XL - 1) / 4; m >= 0; --m) {
                if ((uint32_t)(4 * m) <= ub2) {
#pragma unroll
                    for (int i = 4 * m + 3; i >= 4 * m; --i) {
                        if (i >= XL || i == 0)
                            continue;
                        lv[i] ^= shl7(gf.expa(dq + half(BP, i - 1)));
                    }
#pragma unroll
                    for (int k = 2 * m + 1; k >= 2 * m; --k) {
                        if (k >= (XL + 1) / 2)
                            continue;
                        const uint32_t lo = la[2 * k];
                        const uint32_t hi = 2 * k + 1 < XL ? la[2 * k + 1] : AZ;
                        const uint32_t sh = k > 0 ? __builtin_amdgcn_alignbyte(BP[k], BP[k - 1], 2)
                                                  : ((BP[0] << 16) | AZ);
                        BP[k] = lengthen ? (lo | (hi << 16)) : (act ? sh : BP[k]);
                    }
                }
            }
            if (act) {
                db = lengthen ? dl : min(db + 1u, (uint32_t)(XL - 1));
                if (upd)
                    dl = up;
                if (lengthen) {
                    L = r + ne - L;
                    lb = ld;
                }
            }
        };
        uint32_t snext = sp[0];
        const uint32_t nq = (npar + 3u) >> 2; /* iterations r <= npar (a step past npar changes nothing: act) */
#pragma unroll 1
        for (uint32_t q = 0; q < nq; ++q) {
            const uint32_t sd = snext;
            if (q + 1u < nq) /* uniform */
                snext = sp[q + 1u];
#pragma unroll
            for (int k = 17; k >= 2; --k)
                WL[k] = WL[k - 2];
            const uint32_t s0 = gf.logs(sd & 0xffu), s1 = gf.logs((sd >> 8) & 0xffu);
            const uint32_t s2 = gf.logs((sd >> 16) & 0xffu), s3 = gf.logs(sd >> 24);
            WL[0] = s3 | (s2 << 16);
            WL[1] = s1 | (s0 << 16);
            if (4u * q + 4u > nemin) { /* uniform: some lane is active in this block */
                step(std::integral_constant<int, 0>{}, 4u * q + 1u);
                step(std::integral_constant<int, 1>{}, 4u * q + 2u);
                step(std::integral_constant<int, 2>{}, 4u * q + 3u);
                step(std::integral_constant<int, 3>{}, 4u * q + 4u);
            }
        }

        /* ---- degree, src/decode.c:98-110 ---- */
        uint32_t deg = 0;
#pragma unroll
        for (int i = 0; i < XL; ++i)
            deg = lv[i] != HZ ? (uint32_t)i : deg;
        const bool fast = elig && deg == L && deg != 0u;
        if (elig && !fast) {
            meta[cw] = (uint8_t)(RS_ST_LIST << 5);
            list[atomicAdd(nlist, 1u)] = (uint32_t)cw;
        }
        const uint32_t dmx = wave_max_full(fast ? deg : 0u);
        uint32_t al[XL]; /* address-form logs of the final Lambda */
        al[0] = pofs;
#pragma unroll
        for (int i = 1; i < XL; ++i)
            al[i] = (uint32_t)i <= dmx ? gf.logh(lv[i]) : AZ;

        /* ---- Omega = S * Lambda mod x^deg (log form), src/decode.c:147-158 ---- */
        uint32_t ob[RS_NR / 4];
#pragma unroll
        for (int k = 0; k < RS_NR / 4; ++k)
            ob[k] = 0xFFFFFFFFu;
        const uint32_t degmax = wave_max_full(fast ? deg : 0u);
        if (degmax) {
            uint32_t sl[RS_NR]; /* plain scaled logs of S_0..S_31, one register each */
            {
                const uint4 s4a = reinterpret_cast<const uint4 *>(sp)[0], s4b = reinterpret_cast<const uint4 *>(sp)[1];
                const uint32_t sw[8] = {s4a.x, s4a.y, s4a.z, s4a.w, s4b.x, s4b.y, s4b.z, s4b.w};
#pragma unroll
                for (int k = 0; k < RS_NR; ++k)
                    sl[k] = gf.logs((sw[k >> 2] >> (8 * (k & 3))) & 0xffu);
            }
#pragma unroll
            for (int m = 0; m < RS_NR; ++m) {
                if ((uint32_t)m < degmax) { /* uniform */
                    uint32_t acc = 0;
#pragma unroll
                    for (int j = 0; j <= m; ++j)
                        acc ^= gf.expa(al[j] + sl[m - j]);
                    const uint32_t o = (uint32_t)m < deg ? gf.plog(gf.loga(acc)) : 255u;
                    ob[m >> 2] ^= (o ^ 0xffu) << (8 * (m & 3));
                }
                __builtin_amdgcn_sched_barrier(0); /* one coefficient's lookups at a time: registers */
            }
        }
        if (fast) {
            uint32_t lb8[RS_NR / 4];
#pragma unroll
            for (int k = 0; k < RS_NR / 4; ++k)
                lb8[k] = 0;
#pragma unroll
            for (int j = 1; j < XL; ++j)
                lb8[(j - 1) >> 2] |= gf.plog(al[j]) << (8 * ((j - 1) & 3));
            uint4 *e = reinterpret_cast<uint4 *>(ext + cw * 64u);
            e[0] = make_uint4(lb8[0], lb8[1], lb8[2], lb8[3]);
            e[1] = make_uint4(lb8[4], lb8[5], lb8[6], lb8[7]);
            e[2] = make_uint4(ob[0], ob[1], ob[2], ob[3]);
            e[3] = make_uint4(ob[4], ob[5], ob[6], ob[7]);
            meta[cw] = (uint8_t)((RS_ST_ERRATA << 5) | (deg & 31u));
        }
    }
}

/* ------------------------------------------------------------------------ */
/* rs_chien32_k: roots of a locator of degree <= 32                          */
/* ------------------------------------------------------------------------ */

/*
 * As rs_chien_k (rs_fast.hip) with 32 terms: Lambda(alpha^i'), i' = 16a + b,
 * is 1 + sum_j row_j[e_j(a)]_b, e_j(a) = (log Lambda_j + 16 a j) mod 255.
 * LDS: row (j, e) at e * 512 + (j - 1) * 16 (128 KiB).  Slot k of lane l
 * holds term ((k + l) mod NT) + 1, so the 16 lanes of a ds_read_b128 group
 * read 16 different bank slots; NT = 16 or 24 where the wave's degrees allow
 * (the upper rows' terms are zero).  Roots go into a 32-byte list, newest (largest
 * i) first.
 */
__global__ __launch_bounds__(XWG, 4) void rs_chien32_k(const RsDevTables *__restrict__ T, RsCorrParams P,
                                                      size_t count, const uint8_t *__restrict__ ext,
                                                      uint8_t *__restrict__ meta, uint8_t *__restrict__ roots,
                                                      uint8_t *__restrict__ ok, uint8_t *__restrict__ corrected,
                                                      const uint32_t *__restrict__ npend)
{
    if (npend && *npend == 0u) /* rs_era_bp_k decoded every codeword */
        return;
    __shared__ uint4 lch[256 * 32];
    for (uint32_t t = threadIdx.x; t < 256u * 32u; t += XWG)
        lch[t] = T->chien[(t & 31u) * 256u + (t >> 5)];
    __syncthreads();
    const uint32_t cb = lds_addr(lch);
    constexpr uint32_t RS = 512u;       /* LDS bytes per e */
    constexpr uint32_t WRAP = 255u * RS;

    uint32_t it = 0;
    for (size_t base = (size_t)blockIdx.x * XWG; base < count; base += (size_t)gridDim.x * XWG, ++it) {
        prio_by_progress(it);
        const size_t cw = base + threadIdx.x;
        const bool valid = cw < count;
        const uint32_t st = valid ? meta[cw] : 0u;
        const bool fast = (st >> 5) == RS_ST_ERRATA;
        if (__ballot(fast) == 0ull)
            continue;
        const uint32_t deg = fast ? ((st & 31u) ? (st & 31u) : 32u) : 0u;
        uint32_t lw[RS_NR / 4];
#pragma unroll
        for (int k = 0; k < RS_NR / 4; ++k)
            lw[k] = 0xFFFFFFFFu;
        if (fast) {
            const uint4 *e = reinterpret_cast<const uint4 *>(ext + cw * 64u);
            const uint4 a = e[0], b = e[1];
            lw[0] = a.x, lw[1] = a.y, lw[2] = a.z, lw[3] = a.w;
            lw[4] = b.x, lw[5] = b.y, lw[6] = b.z, lw[7] = b.w;
        }
        uint32_t R[RS_NR / 4] = {0, 0, 0, 0, 0, 0, 0, 0}; /* the root list, newest first */
        uint32_t cnt = 0;
        auto push = [&](uint32_t v) __attribute__((always_inline)) {
#pragma unroll
            for (int k = RS_NR / 4 - 1; k > 0; --k)
                R[k] = __builtin_amdgcn_alignbyte(R[k], R[k - 1], 3);
            R[0] = (R[0] << 8) | v;
        };
        /* the G log bytes of lw from byte b0 rotated by lr (G = 8, 16, 32):
         * byte k of Rl = log Lambda_(b0 + ((k + lr) mod G) + 1) */
        auto rotated = [&](auto gc, auto b0c, uint32_t lr, uint32_t *Rl) __attribute__((always_inline)) {
            constexpr int G = decltype(gc)::value, GD = G / 4, W0 = decltype(b0c)::value / 4;
            uint32_t D[GD];
#pragma unroll
            for (int k = 0; k < GD; ++k)
                D[k] = lw[W0 + k];
#pragma unroll
            for (int bit = 1; bit < GD; bit <<= 1) {
                const bool c = ((lr >> 2) & (uint32_t)bit) != 0u;
                uint32_t E[GD];
#pragma unroll
                for (int k = 0; k < GD; ++k)
                    E[k] = c ? D[(k + bit) % GD] : D[k];
#pragma unroll
                for (int k = 0; k < GD; ++k)
                    D[k] = E[k];
            }
#pragma unroll
            for (int k = 0; k < GD; ++k)
                Rl[k] = __builtin_amdgcn_alignbyte(D[(k + 1) % GD], D[k], lr & 3u);
        };
        /* NT slots: NT = 16 or 32 terms rotated by lane mod NT; NT = 24: terms
         * 1..16 rotated by lane mod 16, 17..24 by lane mod 8 (the last eight
         * slots read with 2-way bank conflicts: lanes l and l + 8 share a
         * slot) */
        auto search = [&](auto ntc) __attribute__((always_inline)) {
            constexpr int NT = decltype(ntc)::value;
            constexpr int G1 = NT == 32 ? 32 : 16, G2 = NT - G1;
            uint32_t lr = threadIdx.x & (G1 - 1);
            asm volatile("" : "+v"(lr));
            uint32_t Rl[NT / 4];
            rotated(std::integral_constant<int, G1>{}, std::integral_constant<int, 0>{}, lr, Rl);
            if constexpr (G2 > 0)
                rotated(std::integral_constant<int, G2>{}, std::integral_constant<int, G1>{}, lr & (G2 - 1u),
                        Rl + G1 / 4);
            uint32_t A[NT], inc[NT];
#pragma unroll
            for (int k = 0; k < NT; ++k) {
                const uint32_t jm = k < G1 ? (((uint32_t)k + lr) & (G1 - 1))
                                           : G1 + (((uint32_t)(k - G1) + lr) & (uint32_t)(G2 > 0 ? G2 - 1 : 0)); /* j - 1 */
                const uint32_t e = (Rl[k >> 2] >> (8 * (k & 3))) & 0xffu;
                A[k] = cb + e * RS + (jm << 4);
                inc[k] = e == 255u ? WRAP : ((16u * (jm + 1u)) % 255u) * RS;
            }
            uint32_t z0 = 0;
#pragma unroll 1
            for (int w = 0; w < 8; ++w) {
                uint32_t word = 0;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    uint32_t acc[4] = {0x01010101u, 0x01010101u, 0x01010101u, 0x01010101u};
#pragma unroll
                    for (int k = 0; k < NT; k += 2) {
                        const lds_u32x4_t r1 = lds128(A[k]), r2 = lds128(A[k + 1]);
                        A[k] = chien_step<WRAP>(A[k], inc[k]);
                        A[k + 1] = chien_step<WRAP>(A[k + 1], inc[k + 1]);
                        acc[0] = xor3(acc[0], r1.x, r2.x);
                        acc[1] = xor3(acc[1], r1.y, r2.y);
                        acc[2] = xor3(acc[2], r1.z, r2.z);
                        acc[3] = xor3(acc[3], r1.w, r2.w);
                    }
                    word |= zero_bytes16(acc) << (16 * h);
                }
                if (w == 7)
                    word &= 0x7FFFFFFFu; /* i' = 255 repeats i' = 0 */
                if (w == 0) {
                    z0 = word & 1u; /* i' = 0 is the reference's last point, i = 255 */
                    word &= ~1u;
                }
                cnt += __popc(word);
                const uint32_t wb = 32u * (uint32_t)w;
                while (word != 0u) { /* at most deg <= 32 pushes per lane in all */
                    const uint32_t b = __builtin_ctz(word);
                    word &= word - 1u;
                    push(wb + b);
                }
            }
            if (z0)
                push(255u);
            cnt += z0;
        };
        const uint32_t degmax = wave_max_full(deg);
        if (degmax <= 16u)
            search(std::integral_constant<int, 16>{});
        else if (degmax <= 24u)
            search(std::integral_constant<int, 24>{});
        else
            search(std::integral_constant<int, 32>{});
        bool good = cnt == deg; /* src/decode.c:143-145 */
        if (P.pad > 0) {
            /* locations k = (i iprim - 1) mod 255 below pad fail, src/decode.c:132-134 */
            bool low = false;
#pragma unroll
            for (int n = 0; n < RS_NR; ++n) {
                const uint32_t i = (R[n >> 2] >> (8 * (n & 3))) & 0xffu;
                low |= (uint32_t)n < cnt && (int32_t)((i * P.iprim + 254u) % 255u) < P.pad;
            }
            good = good && !low;
        }
        if (fast) {
            uint4 *o = reinterpret_cast<uint4 *>(roots + cw * 32u);
            o[0] = make_uint4(R[0], R[1], R[2], R[3]);
            o[1] = make_uint4(R[4], R[5], R[6], R[7]);
        }
        if (fast && !good) {
            ok[cw] = 0;
            if (corrected)
                corrected[cw] = 0;
            meta[cw] = (uint8_t)(RS_ST_DONE << 5);
        }
    }
}

/* ------------------------------------------------------------------------ */
/* rs_forney32_k: magnitudes as slot records                                 */
/* ------------------------------------------------------------------------ */

/*
 * Root b of the list (newest first) is the reference's root n = deg - 1 - b;
 * num = sum_(m < deg) Omega_m alpha^(i m) and den = sum_h Lambda_(2h+1)
 * alpha^(2h i) (src/decode.c:159-191), each split at m = 16 as rs_era_k's (round 3),
 * magnitude alpha^(log num + log alpha^(i (fcr-1)) + 255 - log den) (no den =
 * 0 guard, as the reference); a zero numerator corrects nothing and is not
 * counted.  The record pairs magnitude b with list slot deg - 1 - b: the
 * slots reversed and shifted down by 32 - deg bytes (0xFF = no slot), so the
 * apply writes magnitude n at slot n as the reference does (:211-214).
 */
__global__ __launch_bounds__(XWG, 4) void rs_forney32_k(const RsDevTables *__restrict__ T, RsCorrParams P,
                                                       const uint8_t *__restrict__ pos8, size_t pos_stride,
                                                       size_t count, uint8_t *__restrict__ ext,
                                                       const uint8_t *__restrict__ roots,
                                                       uint8_t *__restrict__ meta, uint8_t *__restrict__ ok,
                                                       uint8_t *__restrict__ corrected, const uint32_t *__restrict__ npend,
                                                       uint32_t npar)
{
    if (npend && *npend == 0u) /* rs_era_bp_k decoded every codeword */
        return;
    __shared__ uint32_t lgf[512 * 32];
    fill_gfa<XWG>(lgf, T);
    __syncthreads();
    const GfA gf{lds_addr(lgf) + 4u * (threadIdx.x & 31u) + 1u};

    uint32_t it = 0;
    for (size_t base = (size_t)blockIdx.x * XWG; base < count; base += (size_t)gridDim.x * XWG, ++it) {
        prio_by_progress(it);
        const size_t cw = base + threadIdx.x;
        const bool valid = cw < count;
        const uint32_t st = valid ? meta[cw] : 0u;
        const bool fast = (st >> 5) == RS_ST_ERRATA;
        if (__ballot(fast) == 0ull)
            continue;
        const uint32_t deg = fast ? ((st & 31u) ? (st & 31u) : 32u) : 0u;
        uint32_t lw[RS_NR / 4], ow[RS_NR / 4], rl[RS_NR / 4];
#pragma unroll
        for (int k = 0; k < RS_NR / 4; ++k)
            lw[k] = ow[k] = 0xFFFFFFFFu, rl[k] = 0;
        if (fast) {
            const uint4 *e = reinterpret_cast<const uint4 *>(ext + cw * 64u);
            const uint4 a = e[0], b = e[1], c = e[2], d = e[3];
            lw[0] = a.x, lw[1] = a.y, lw[2] = a.z, lw[3] = a.w, lw[4] = b.x, lw[5] = b.y, lw[6] = b.z, lw[7] = b.w;
            ow[0] = c.x, ow[1] = c.y, ow[2] = c.z, ow[3] = c.w, ow[4] = d.x, ow[5] = d.y, ow[6] = d.z, ow[7] = d.w;
            const uint4 *r = reinterpret_cast<const uint4 *>(roots + cw * 32u);
            const uint4 r0 = r[0], r1 = r[1];
            rl[0] = r0.x, rl[1] = r0.y, rl[2] = r0.z, rl[3] = r0.w, rl[4] = r1.x, rl[5] = r1.y, rl[6] = r1.z,
            rl[7] = r1.w;
        }
        /* address-form logs: Omega_0..31 and the odd terms Lambda_1, 3, .., 31 (byte j - 1 of lw) */
        uint32_t opu[RS_NR], lod[RS_NR / 2];
#pragma unroll
        for (int m = 0; m < RS_NR; ++m)
            opu[m] = gf.afrom((ow[m >> 2] >> (8 * (m & 3))) & 0xffu);
#pragma unroll
        for (int h = 0; h < RS_NR / 2; ++h)
            lod[h] = gf.afrom((lw[(2 * h) >> 2] >> (8 * ((2 * h) & 3))) & 0xffu);
        const uint32_t degmax = wave_max_full(deg);
        uint32_t magp[RS_NR / 4] = {0, 0, 0, 0, 0, 0, 0, 0};
        uint32_t fixed = 0;
        /* the sums split at m = H, H = 8, 12 or 16 by the wave's degree
         * (Omega_m for m < deg <= 2H, Lambda_(2h+1) for h < H): the upper
         * halves' logs picked once, the chains run H steps */
        const uint32_t H = degmax <= 16u ? 8u : degmax <= 24u ? 12u : 16u;
        uint32_t oph[RS_NR / 2], ldh[RS_NR / 4];
#pragma unroll
        for (int b = 0; b < RS_NR / 2; ++b)
            oph[b] = H == 8u ? opu[b + 8] : H == 12u ? opu[b + 12 < RS_NR ? b + 12 : RS_NR - 1] : opu[b + 16];
#pragma unroll
        for (int h = 0; h < RS_NR / 4; ++h)
            ldh[h] = H == 8u ? lod[h + 4] : H == 12u ? lod[h + 6] : lod[h + 8];
#pragma unroll
        for (int n0 = 0; n0 < RS_NR; n0 += XR) {
            if ((uint32_t)n0 >= degmax) /* uniform */
                continue;
            uint32_t ir[XR], si[XR], s[XR], num[XR], den[XR], nh[XR], dh[XR];
#pragma unroll
            for (int t = 0; t < XR; ++t) {
                ir[t] = (rl[(n0 + t) >> 2] >> (8 * ((n0 + t) & 3))) & 0xffu;
                si[t] = 128u * (ir[t] == 255u ? 0u : ir[t]);
                s[t] = num[t] = den[t] = nh[t] = dh[t] = 0;
            }
#pragma unroll
            for (int b = 0; b < RS_NR / 2; ++b) {
                if ((uint32_t)b < H) { /* uniform */
#pragma unroll
                    for (int t = 0; t < XR; ++t) {
                        num[t] ^= gf.expa(opu[b] + s[t]);
                        nh[t] ^= gf.expa(oph[b] + s[t]);
                        if ((b & 1) == 0) {
                            den[t] ^= gf.expa(lod[b >> 1] + s[t]);
                            dh[t] ^= gf.expa(ldh[b >> 1] + s[t]);
                        }
                        s[t] = addmod7(s[t], si[t]);
                    }
                }
                if (b & 1) {
#pragma unroll
                    for (int t = 0; t < XR; ++t)
                        asm volatile("" : "+v"(num[t]), "+v"(den[t]), "+v"(nh[t]), "+v"(dh[t]));
                    __builtin_amdgcn_sched_barrier(0); /* two powers at a time: registers */
                }
            }
#pragma unroll
            for (int t = 0; t < XR; ++t) { /* s = 128 (H i mod 255) */
                num[t] ^= gf.expa(gf.loga(nh[t]) + s[t]);
                den[t] ^= gf.expa(gf.loga(dh[t]) + s[t]);
                /* alpha^(log num + ln2 + 255 - log den) from the address forms
                 * (den != 0 at the deg distinct roots), reduced once */
                const uint32_t l2s = P.fcr == 1u ? 0u
                                                 : 128u * mod255((uint32_t)((int32_t)ir[t] * ((int32_t)P.fcr - 1) +
                                                                            (int32_t)RS_NN));
                const uint32_t x = gf.loga(num[t]) - gf.loga(den[t]) + 255u * 128u + gf.pofs + l2s;
                const bool z = (uint32_t)(n0 + t) < deg && num[t] != 0u;
                fixed += z ? 1u : 0u;
                magp[(n0 + t) >> 2] |= (z ? gf.expa(min(x, x - 255u * 128u)) : 0u) << (8 * ((n0 + t) & 3));
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (fast) {
            /* slot of record entry b: list slot deg - 1 - b (0xFF past deg) */
            const uint32_t *pw = reinterpret_cast<const uint32_t *>(pos8 + cw * pos_stride);
            uint32_t X[RS_NR / 4];
#pragma unroll
            for (int k = 0; k < RS_NR / 4; ++k) /* reversed: byte j = slot 31 - j (the row's npar slots only) */
                X[k] = __builtin_amdgcn_perm(0u, 4u * (RS_NR / 4 - 1 - k) < npar ? pw[RS_NR / 4 - 1 - k] : 0u,
                                             0x00010203u);
            const uint32_t sh = RS_NR - deg; /* bytes: X <- X >> 8 sh, 0xFF shifted in */
#pragma unroll
            for (int bit = 1; bit < 16; bit <<= 1) {
                const bool c = ((sh >> 2) & (uint32_t)bit) != 0u;
                uint32_t Y[RS_NR / 4];
#pragma unroll
                for (int k = 0; k < RS_NR / 4; ++k)
                    Y[k] = c ? (k + bit < RS_NR / 4 ? X[k + bit] : 0xFFFFFFFFu) : X[k];
#pragma unroll
                for (int k = 0; k < RS_NR / 4; ++k)
                    X[k] = Y[k];
            }
            const uint32_t sb = sh & 3u;
            uint32_t pk[RS_NR / 4];
#pragma unroll
            for (int k = 0; k < RS_NR / 4; ++k)
                pk[k] = __builtin_amdgcn_alignbyte(k + 1 < RS_NR / 4 ? X[k + 1] : 0xFFFFFFFFu, X[k], sb);
            uint4 *e = reinterpret_cast<uint4 *>(ext + cw * 64u);
            e[0] = make_uint4(pk[0], pk[1], pk[2], pk[3]);
            e[1] = make_uint4(pk[4], pk[5], pk[6], pk[7]);
            e[2] = make_uint4(magp[0], magp[1], magp[2], magp[3]);
            e[3] = make_uint4(magp[4], magp[5], magp[6], magp[7]);
            meta[cw] = (uint8_t)(RS_ST_FAST << 5); /* a record for rs_apply_k */
            ok[cw] = 1;
            if (corrected)
                corrected[cw] = (uint8_t)fixed;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* launchers                                                                 */
/* ------------------------------------------------------------------------ */

extern "C" hipError_t rsk_ebm(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, const uint8_t *pos8,
                              size_t pos_stride, const uint8_t *cnt, size_t count, uint8_t *ok, uint8_t *corrected,
                              uint32_t only_pend, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rs_ebm_k, dim3(errata_grid(count, num_cu)), dim3(XWG), 0, stream, tab, *prm, ws->syn, pos8,
                       pos_stride, cnt, count, ws->ext, ws->meta, ws->list, ws->nlist, ok, corrected, only_pend,
                       (uint32_t)RS_NR);
    return hipGetLastError();
}

/* a byte-symbol code of npar < 32 roots (syndromes from rsk_syndrome_reset_nr,
 * rows of npar slots, pos_stride >= npar): npar iterations, at most npar
 * erasures; Chien (rsk_chien32) as for 32 */
extern "C" hipError_t rsk_ebm_nr(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws,
                                 const uint8_t *pos8, size_t pos_stride, const uint8_t *cnt, size_t count, uint8_t *ok,
                                 uint8_t *corrected, uint32_t npar, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rs_ebm_k, dim3(errata_grid(count, num_cu)), dim3(XWG), 0, stream, tab, *prm, ws->syn, pos8,
              pos_stride, cnt, count, ws->ext, ws->meta, ws->list, ws->nlist, ok, corrected, 0u, npar);
    return hipGetLastError();
}

extern "C" hipError_t rsk_chien32(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, size_t count,
                                  uint8_t *ok, uint8_t *corrected, uint32_t only_pend, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rs_chien32_k, dim3(errata_grid(count, num_cu)), dim3(XWG), 0, stream, tab, *prm, count,
                       ws->ext, ws->meta, ws->roots, ok, corrected, only_pend ? ws->nlist + 1 : nullptr);
    return hipGetLastError();
}

extern "C" hipError_t rsk_forney32(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws,
                                   const uint8_t *pos8, size_t pos_stride, size_t count, uint8_t *ok,
                                   uint8_t *corrected, uint32_t only_pend, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rs_forney32_k, dim3(errata_grid(count, num_cu)), dim3(XWG), 0, stream, tab, *prm, pos8,
                       pos_stride, count, ws->ext, ws->roots, ws->meta, ok, corrected, only_pend ? ws->nlist + 1 : nullptr,
                       (uint32_t)RS_NR);
    return hipGetLastError();
}

extern "C" hipError_t rsk_forney32_nr(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws,
                                      const uint8_t *pos8, size_t pos_stride, size_t count, uint8_t *ok,
                                      uint8_t *corrected, uint32_t npar, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rs_forney32_k, dim3(errata_grid(count, num_cu)), dim3(XWG), 0, stream, tab, *prm, pos8, pos_stride,
              count, ws->ext, ws->roots, ws->meta, ok, corrected, (const uint32_t *)nullptr, npar);
    return hipGetLastError();
}
