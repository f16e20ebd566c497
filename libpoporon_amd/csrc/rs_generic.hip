/*
 * rs_generic.hip -- RS over GF(2^m), any parameters with m <= 8 (gfx950).
 *
 * The fast kernels (rs_kernels.hip, rs_correct.hip) are specialised for
 * symbol_size 8 and num_roots 32.  Every other parameter set that the
 * reference accepts and that fits byte symbols (2 <= m <= 8, any primitive
 * field polynomial, any fcr, any prim with a primitive inverse, 1 <= num_roots
 * < 2^m - 1) is served here, with the reference's integer semantics step by
 * step:
 *   rsg_encode_k   systematic LFSR                      src/encode.c:120-143
 *   rsg_decode_k   syndromes (Horner per root)          src/decode.c:375-415
 *                  erasure locator, BM, Chien, Omega,
 *                  Forney, re-syndrome check, apply     src/decode.c:17-230
 *                  branch logic (ext. syndrome/erasure) src/decode.c:431-487
 *   rsg_check_k    "any syndrome nonzero" only
 * in two families:
 *   rsg_*    one codeword per lane (large batches of short codes), below;
 *   rsgw_*   one codeword per wave (single calls, small batches, long codes,
 *            the split decode's lists) and rsgw_serve_k, the single-call
 *            server of general-parameter handles: after rsg_check_k.
 * api.cpp gen_wave() picks the family; both give the same bytes.
 *
 * Per lane: every per-codeword array (syndromes, locator, B,
 * Omega, roots, locations, magnitudes; num_roots + 1 bytes each) lives in
 * LDS laid out [index][lane], so lanes of a wave touch consecutive bytes.
 * With m <= 8 every field element and every log (A0 = 2^m - 1 is the log of
 * zero) fits a byte.  The GF tables (log, antilog, generator) are 768 bytes
 * of LDS shared by the workgroup.
 *
 * gf_mod (src/internal/common.h:102-110) takes a uint16 and, for m <= 8,
 * equals (v mod 2^16) mod (2^m - 1) for every argument (checked exhaustively
 * in tests/test_library_cpu.py); the kernels compute it with a reciprocal
 * multiply (exact for arguments < 2^16).
 */
#include <hip/hip_runtime.h>

#include <algorithm>

#include "rs_generic.h"
#include "rs_device.h" /* RS_LAUNCH */

#define G_WG_MAX 256

struct GMod {
    uint32_t nn, magic; /* magic = floor(2^32 / nn) + 1 */
    /* gf_mod of the uint16 truncation of v */
    __device__ __forceinline__ uint32_t operator()(uint32_t v) const
    {
        const uint32_t x = v & 0xffffu;
        const uint32_t q = __umulhi(x, magic);
        return x - q * nn;
    }
};

/* LDS tables (768 B) + per-lane arrays [slot][index][lane] (bytes) */
struct GShared {
    uint8_t *alog, *log, *gen;
    uint8_t *lane; /* start of the per-lane area */
    uint32_t wg;
    __device__ __forceinline__ uint8_t *arr(uint32_t slot, uint32_t nr1) const { return lane + slot * nr1 * wg; }
};

__device__ __forceinline__ GShared g_setup(const RsGenTables *__restrict__ T, uint8_t *smem)
{
    GShared s;
    s.alog = smem;
    s.log = smem + 256;
    s.gen = smem + 512;
    s.lane = smem + 768;
    s.wg = blockDim.x;
    for (uint32_t t = threadIdx.x; t < 768u; t += blockDim.x)
        smem[t] = t < 256u ? T->alog[t] : (t < 512u ? T->log[t - 256u] : T->gen[t - 512u]);
    __syncthreads();
    return s;
}

/* per-lane view of one LDS array: element i of this lane */
struct LaneArr {
    uint8_t *p;
    uint32_t wg;
    __device__ __forceinline__ uint8_t &operator[](uint32_t i) const { return p[i * wg]; }
};

/* ------------------------------------------------------------------------ */
/* encode, src/encode.c:120-143                                             */
/* ------------------------------------------------------------------------ */

/* The shift register is a ring in LDS: logical byte j is physical
 * (head + j) mod nr, so the reference's memmove is a head increment. */
__global__ __launch_bounds__(G_WG_MAX) void rsg_encode_k(const RsGenTables *__restrict__ T, RsGenParams P,
                                                          const uint8_t *__restrict__ data, size_t dstride,
                                                          uint8_t *__restrict__ parity, size_t pstride, size_t count)
{
    extern __shared__ uint8_t smem[];
    const GShared s = g_setup(T, smem);
    const GMod mod{P.nn, P.magic};
    const uint32_t nr = P.nroots, A0 = P.nn;
    const LaneArr reg{s.arr(0, nr + 1u) + threadIdx.x, s.wg};
    for (size_t cw = (size_t)blockIdx.x * blockDim.x + threadIdx.x; cw < count;
         cw += (size_t)gridDim.x * blockDim.x) {
        const uint8_t *d = data + cw * dstride;
        for (uint32_t j = 0; j < nr; ++j)
            reg[j] = 0;
        uint32_t head = 0;
        for (uint32_t b = 0; b < P.size; ++b) {
            const uint32_t fb = s.log[((uint32_t)d[b] & A0) ^ reg[head]];
            if (fb != A0) {
                uint32_t ph = head;
                for (uint32_t j = 1; j < nr; ++j) {
                    ph = ph + 1u == nr ? 0u : ph + 1u;
                    reg[ph] = (uint8_t)(reg[ph] ^ s.alog[mod(fb + s.gen[nr - j])]);
                }
            }
            /* shift: the old head slot becomes logical byte nr-1 */
            reg[head] = fb != A0 ? s.alog[mod(fb + s.gen[0])] : (uint8_t)0;
            head = head + 1u == nr ? 0u : head + 1u;
        }
        uint8_t *p = parity + cw * pstride;
        for (uint32_t j = 0, ph = head; j < nr; ++j, ph = ph + 1u == nr ? 0u : ph + 1u)
            p[j] = reg[ph];
    }
}

/* ------------------------------------------------------------------------ */
/* syndromes, src/decode.c:375-415 (log form out; returns the nonzero flag) */
/* ------------------------------------------------------------------------ */

__device__ __forceinline__ bool g_syndromes(const GShared &s, const GMod &mod, const RsGenParams &P,
                                            const uint8_t *d, const uint8_t *par, const LaneArr &S)
{
    const uint32_t nr = P.nroots, A0 = P.nn;
    const uint32_t first = (uint32_t)d[0] & A0;
    for (uint32_t i = 0; i < nr; ++i)
        S[i] = (uint8_t)first;
    const uint32_t total = P.size + nr;
    for (uint32_t b = 1; b < total; ++b) {
        const uint32_t in = (uint32_t)(b < P.size ? d[b] : par[b - P.size]) & A0;
        /* (fcr + i) * prim, as the reference's int arithmetic before the
         * uint16 truncation inside gf_mod */
        uint32_t step = P.fcr * P.prim;
        for (uint32_t i = 0; i < nr; ++i, step += P.prim) {
            const uint32_t v = S[i];
            S[i] = (uint8_t)(v ? (in ^ s.alog[mod((uint32_t)s.log[v] + step)]) : in);
        }
    }
    uint32_t flag = 0;
    for (uint32_t i = 0; i < nr; ++i) {
        const uint32_t v = S[i];
        flag |= v;
        S[i] = s.log[v];
    }
    return flag != 0;
}

/* ------------------------------------------------------------------------ */
/* correction, src/decode.c:17-230                                          */
/* ------------------------------------------------------------------------ */

template <typename PosT>
__device__ bool g_correct(const GShared &s, const GMod &mod, const RsGenParams &P, uint8_t *data, uint8_t *parity,
                          const LaneArr &S, uint32_t ne, const PosT *pos, bool eras_apply, uint32_t &corrected)
{
    const uint32_t nr = P.nroots, A0 = P.nn, nr1 = nr + 1u;
    const int32_t pad = P.pad;
    const uint32_t t = threadIdx.x;
    const LaneArr lam{s.arr(1, nr1) + t, s.wg}, B{s.arr(2, nr1) + t, s.wg}, om{s.arr(3, nr1) + t, s.wg};
    const LaneArr roots{s.arr(4, nr1) + t, s.wg}, locs{s.arr(5, nr1) + t, s.wg}, mag{s.arr(6, nr1) + t, s.wg};
    const uint8_t *alog = s.alog, *lg = s.log;

    /* erasure locator prod(1 + X_l x), X_l = alpha^(prim (nn-1-(pos+pad))), src/decode.c:31-47 */
    for (uint32_t i = 0; i <= nr; ++i)
        lam[i] = 0;
    lam[0] = 1;
    if (ne > 0) {
        lam[1] = alog[mod(P.prim * (A0 - 1u - ((uint32_t)pos[0] + (uint32_t)pad)))];
        for (uint32_t i = 1; i < ne; ++i) {
            const uint32_t xl = mod(P.prim * (A0 - 1u - ((uint32_t)pos[i] + (uint32_t)pad)));
            for (uint32_t j = i + 1u; j > 0u; --j) {
                const uint32_t l = lg[lam[j - 1u]];
                if (l != A0)
                    lam[j] = (uint8_t)(lam[j] ^ alog[mod(xl + l)]);
            }
        }
    }
    for (uint32_t i = 0; i <= nr; ++i)
        B[i] = lg[lam[i]];

    /* Berlekamp-Massey (Karn's form with erasures), src/decode.c:49-96.
     * One top-down pass per iteration updates Lambda in place (it reads B
     * at i-1 before that slot is rewritten) and builds the new B from the
     * old Lambda, so no temporary polynomial is needed. */
    uint32_t L = ne;
    for (uint32_t r = ne + 1u; r <= nr; ++r) {
        uint32_t disc = 0;
        for (uint32_t i = 0; i < r; ++i) {
            const uint32_t li = lam[i], si = S[r - i - 1u];
            if (li != 0u && si != A0)
                disc ^= alog[mod((uint32_t)lg[li] + si)];
        }
        disc = lg[disc];
        if (disc == A0) {
            for (uint32_t i = nr; i > 0u; --i)
                B[i] = B[i - 1u];
            B[0] = (uint8_t)A0;
            continue;
        }
        const bool lengthen = 2u * L <= r + ne - 1u;
        for (uint32_t i = nr + 1u; i-- > 0u;) {
            const uint32_t old = lam[i];
            if (i > 0u) {
                const uint32_t b = B[i - 1u];
                if (b != A0)
                    lam[i] = (uint8_t)(old ^ alog[mod(disc + b)]);
            }
            if (lengthen)
                B[i] = (uint8_t)(old == 0u ? A0 : mod((uint32_t)lg[old] - disc + A0));
            else
                B[i] = i > 0u ? B[i - 1u] : (uint8_t)A0;
        }
        if (lengthen)
            L = r + ne - L;
    }

    /* locator to log form, degree, src/decode.c:98-110 */
    uint32_t deg = 0;
    for (uint32_t i = 0; i <= nr; ++i) {
        const uint32_t l = lg[lam[i]];
        lam[i] = (uint8_t)l;
        if (l != A0)
            deg = i;
    }
    if (deg == 0)
        return false;

    /* Chien search, src/decode.c:112-145; B is the register copy */
    for (uint32_t j = 1; j <= nr; ++j)
        B[j] = lam[j];
    uint32_t cnt = 0;
    {
        int32_t k = (int16_t)(uint16_t)(P.iprim - 1u);
        for (uint32_t i = 1; i <= A0; ++i, k = (int16_t)mod((uint32_t)(k + (int32_t)P.iprim))) {
            uint32_t acc = 1;
            for (uint32_t j = deg; j > 0u; --j) {
                const uint32_t rj = B[j];
                if (rj != A0) {
                    const uint32_t v = mod(rj + j);
                    B[j] = (uint8_t)v;
                    acc ^= alog[v];
                }
            }
            if (acc != 0u)
                continue;
            if (k < pad)
                return false;
            roots[cnt] = (uint8_t)i;
            locs[cnt] = (uint8_t)k;
            if (++cnt == deg)
                break;
        }
    }
    if (cnt != deg)
        return false;

    /* Omega = S Lambda mod x^deg, log form, src/decode.c:147-158 */
    for (uint32_t i = 0; i < deg; ++i) {
        uint32_t acc = 0;
        for (uint32_t j = 0; j <= i; ++j) {
            const uint32_t sv = S[i - j], lv = lam[j];
            if (sv != A0 && lv != A0)
                acc ^= alog[mod(sv + lv)];
        }
        om[i] = lg[acc];
    }

    /* Forney, src/decode.c:159-191 (corrected counts nonzero numerators) */
    corrected = 0;
    const uint32_t dtop = (deg < nr - 1u ? deg : nr - 1u) & ~1u;
    for (uint32_t jj = cnt; jj-- > 0u;) {
        const uint32_t rt = roots[jj];
        uint32_t num = 0;
        for (uint32_t i = 0; i < deg; ++i) {
            const uint32_t o = om[i];
            if (o != A0)
                num ^= alog[mod(o + i * rt)];
        }
        if (num == 0u) {
            mag[jj] = 0;
            continue;
        }
        const uint32_t num2 = alog[mod((uint32_t)((int32_t)rt * ((int32_t)P.fcr - 1) + (int32_t)A0))];
        uint32_t den = 0;
        for (int32_t i = (int32_t)dtop; i >= 0; i -= 2) {
            const uint32_t l1 = lam[(uint32_t)i + 1u];
            if (l1 != A0)
                den ^= alog[mod(l1 + (uint32_t)i * rt)];
        }
        mag[jj] = alog[mod((uint32_t)lg[num] + lg[num2] + A0 - lg[den])];
        ++corrected;
    }

    /* re-syndrome check, src/decode.c:193-209 (int16 exponent) */
    for (uint32_t i = 0; i < nr; ++i) {
        uint32_t acc = 0;
        for (uint32_t j = 0; j < cnt; ++j) {
            const uint32_t mj = mag[j];
            if (mj == 0u)
                continue;
            const int32_t kk = (int16_t)(uint16_t)((P.fcr + i) * P.prim * (A0 - (uint32_t)locs[j] - 1u));
            acc ^= alog[mod((uint32_t)((int32_t)lg[mj] + kk))];
        }
        if (acc != alog[S[i]])
            return false;
    }

    /* apply, src/decode.c:211-227 */
    if (eras_apply) {
        /* quirk Q1/Q2: magnitude j (ascending location) goes to list slot j;
         * slots past data[] address parity (p < size + nr) or are dropped */
        for (uint32_t i = 0; i < cnt; ++i) {
            const uint32_t p = (uint32_t)pos[i];
            if (p < P.size)
                data[p] ^= mag[i];
            else if (p < P.size + nr)
                parity[p - P.size] ^= mag[i];
        }
    } else {
        for (uint32_t i = 0; i < cnt; ++i) {
            const int32_t p = (int32_t)locs[i] - pad;
            if (p >= 0 && p < (int32_t)P.size)
                data[p] ^= mag[i];
            else if (p >= (int32_t)P.size && p < (int32_t)(P.size + nr))
                parity[p - (int32_t)P.size] ^= mag[i];
            else
                return false;
        }
    }
    return true;
}

/* Full decode of one batch: branch logic of src/decode.c:431-487.
 * ext: external log-form syndromes (nroots u16 per codeword at ext_stride),
 * values > nn refuse the codeword (out-of-table in the reference).
 * pos/cnt: erasure lists (erasure-object mode), counts > nroots refused. */
/* list != NULL: the codewords list[0 .. *list_n) only (the split decode's
 * hand-off, rsg_decode_list; length read on the device) */
template <typename PosT>
__global__ __launch_bounds__(G_WG_MAX) void rsg_decode_k(const RsGenTables *__restrict__ T, RsGenParams P,
                                                          uint8_t *data, size_t dstride, uint8_t *parity,
                                                          size_t pstride, size_t count,
                                                          const uint16_t *__restrict__ ext, size_t ext_stride,
                                                          const PosT *__restrict__ pos, size_t pos_stride,
                                                          const uint8_t *__restrict__ cntv, uint8_t *__restrict__ ok,
                                                          uint8_t *__restrict__ corrected,
                                                          const uint32_t *__restrict__ list,
                                                          const uint32_t *__restrict__ list_n)
{
    extern __shared__ uint8_t smem[];
    const GShared s = g_setup(T, smem);
    const GMod mod{P.nn, P.magic};
    const uint32_t nr = P.nroots, A0 = P.nn;
    const LaneArr S{s.arr(0, nr + 1u) + threadIdx.x, s.wg};
    const size_t n = list ? (size_t)*list_n : count;
    for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < n; idx += (size_t)gridDim.x * blockDim.x) {
        const size_t cw = list ? (size_t)list[idx] : idx;
        uint8_t *d = data + cw * dstride;
        uint8_t *par = parity + cw * pstride;
        uint32_t fixed = 0;
        bool good;
        if (ext) {
            const uint16_t *e = ext + cw * ext_stride;
            bool any = false, bad = false;
            for (uint32_t i = 0; i < nr; ++i) {
                const uint32_t v = e[i];
                bad |= v > A0;
                any |= v != A0;
                S[i] = (uint8_t)v;
            }
            good = !bad && (!any || g_correct<PosT>(s, mod, P, d, par, S, 0u, (const PosT *)nullptr, false, fixed));
            if (bad)
                fixed = 0;
        } else if (pos) {
            const uint32_t ne = cntv[cw];
            /* clean: success whatever the count (src/decode.c:468); dirty with
             * ne > nr overflows the reference's locator (quirk Q5): refused */
            const bool dirty = g_syndromes(s, mod, P, d, par, S);
            good = !dirty || (ne <= nr && g_correct<PosT>(s, mod, P, d, par, S, ne, pos + cw * pos_stride, true, fixed));
        } else {
            good = !g_syndromes(s, mod, P, d, par, S) ||
                   g_correct<PosT>(s, mod, P, d, par, S, 0u, (const PosT *)nullptr, false, fixed);
        }
        ok[cw] = good ? 1 : 0;
        if (corrected)
            corrected[cw] = (uint8_t)fixed;
    }
}

__global__ __launch_bounds__(G_WG_MAX) void rsg_check_k(const RsGenTables *__restrict__ T, RsGenParams P,
                                                         const uint8_t *__restrict__ data, size_t dstride,
                                                         const uint8_t *__restrict__ parity, size_t pstride,
                                                         size_t count, uint8_t *__restrict__ dirty,
                                                         uint16_t *__restrict__ syn, size_t syn_stride)
{
    extern __shared__ uint8_t smem[];
    const GShared s = g_setup(T, smem);
    const GMod mod{P.nn, P.magic};
    const LaneArr S{s.arr(0, P.nroots + 1u) + threadIdx.x, s.wg};
    for (size_t cw = (size_t)blockIdx.x * blockDim.x + threadIdx.x; cw < count;
         cw += (size_t)gridDim.x * blockDim.x) {
        const bool nz = g_syndromes(s, mod, P, data + cw * dstride, parity + cw * pstride, S);
        if (dirty)
            dirty[cw] = nz ? 1 : 0;
        if (syn) /* log form, the reference's uint16 array (src/decode.c:409-412) */
            for (uint32_t i = 0; i < P.nroots; ++i)
                syn[cw * syn_stride + i] = S[i];
    }
}


/* ======================================================================== */
/* one codeword per wave (rsgw_*): the same steps and integer semantics,     */
/* the polynomial coefficients, syndromes, Chien points and roots spread     */
/* over the 64 lanes (index i on lane i % 64, register slot i / 64)          */
/* ======================================================================== */
/* The one-codeword-per-lane kernels above run each codeword as one serial
 * chain of ~size * nroots dependent LDS lookups: ~1 ms for a single call of
 * RS(255,239)-sized codes, 23 ms for 200 roots.  Here a wave shares the
 * work of one codeword: syndromes as independent terms (or per-root Horner
 * where the reference's uint16 exponent truncation makes the multiplier
 * depend on the operand), BM with coefficient i on lane i % 64 (the
 * discrepancy by a DPP/permlane XOR reduction, B[i - 1] by a DPP shift),
 * Chien over all points at once, Omega / Forney / the re-syndrome check
 * with lanes over their indices, the apply from an LDS copy of the row. */
#define GW_WG 256
#ifndef GW_PHASE_STOP
#define GW_PHASE_STOP 0 /* experiment builds: 1..7 end the decode before a phase (tools/gw_batch.py --no-check) */
#endif
#define GW_Z 512u   /* log of zero in the sentinel arrays: any sum with it indexes al2's zero part */
#define GW_AL2 1536 /* al2[x] = alpha^(x mod nn) for x < 2 nn, 0 from there on */
#define GW_QS 16384 /* max size * nr with size + nr <= 255: 127 * 128 (u16: 32 KB) */

/* one codeword's LDS state; N = 4 x the lanes per codeword (indices i on
 * lane i % GL, register slot i / GL) */
template <int N>
struct alignas(16) GwRowT {
    uint8_t cw[N];    /* the received row [data | parity], raw bytes */
    uint16_t lr[N];   /* log of each masked byte (GW_Z: zero) */
    uint8_t S[N];     /* syndromes, log form (nn: zero) */
    uint16_t sz[N];   /* the same, GW_Z for zero */
    uint16_t lamz[N]; /* locator, log form, GW_Z for zero */
    uint16_t omz[N];  /* Omega, log form, GW_Z for zero */
    uint16_t lgm[N];  /* per root: log of its magnitude (0xffff: zero) ... */
    uint16_t lx[N];   /* ... and nn - 1 - its location (the re-syndrome check's factor) */
    uint8_t roots[N], locs[N], mag[N];
    uint32_t acc[N];  /* syndrome partial sums / erasure slots / apply deltas */
};
typedef GwRowT<256> GwWave;

struct GwSmem {
    uint8_t alog[256], log[256];
    uint16_t lgz[256]; /* log with GW_Z for zero */
    uint8_t al2[GW_AL2];
    GwWave w[GW_WG / 64];
};

/* GL lanes per codeword: 64 / GL codewords per wave (codes of up to 4 GL - 1
 * symbols; GL = 4, 8, 16, 32, 64) */
template <int GL>
struct GwSmemG {
    uint8_t alog[256], log[256];
    uint16_t lgz[256]; /* log with GW_Z for zero */
    uint8_t al2[GW_AL2];
    GwRowT<4 * GL> w[GW_WG / GL];
    uint8_t sideS[GW_WG / GL][4 * GL];   /* gw_decode_pair: the first codeword's syndromes ... */
    uint16_t sideSz[GW_WG / GL][4 * GL]; /* ... while the row holds the second */
    uint8_t sideLam[GW_WG / GL][8 * GL]; /* ... and the two locators until each one's finish */
};

/* lane order within a wave: LDS writes by some lanes, then reads by others */
__device__ __forceinline__ void gw_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

/* single calls on coherent host memory: every store of the block
 * acknowledged, then one system-scope release of the completion word */
__device__ __forceinline__ void gw_done(uint32_t *flag, uint32_t seq)
{
    if (flag) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
            __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

/* XOR over the wave, in every lane (permlane swaps across halves and rows,
 * DPP within a row) */
__device__ __forceinline__ uint32_t gw_xor(uint32_t v)
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

/* out[i] = v[i - 1] over the four register slots (index i = lane + 64 q);
 * out[0] = first.  DPP wave_shr:1, the slot's carry through lane 63 */
__device__ __forceinline__ void gw_shift(const uint32_t (&v)[4], uint32_t (&out)[4], uint32_t lane, uint32_t first,
                                         uint32_t nq)
{
    uint32_t carry = first;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        if ((uint32_t)q < nq) { /* slots past nq hold nothing (uniform) */
            const uint32_t top = (uint32_t)__builtin_amdgcn_readlane((int)v[q], 63);
            const uint32_t u = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[q], 0x138, 0xf, 0xf, true);
            out[q] = lane ? u : carry;
            carry = top;
        }
    }
}

/* The GL lanes of a wave that share one codeword (GL = 64: the whole wave;
 * 32: a half; 16: a DPP row; 8: a half-row; 4: a quad): the index within the group, the group's bits of
 * a ballot, the XOR over the group and the shift by one index (slot carry
 * from the group's last lane).  Groups run the same code; their branches
 * diverge per codeword. */
template <int GL>
struct GwGrp {
    uint32_t gl; /* lane within the group */
    uint32_t gb; /* the group's first lane in the wave */
    __device__ __forceinline__ explicit GwGrp(uint32_t lane) : gl(lane % GL), gb(lane - lane % GL) {}
    __device__ __forceinline__ uint64_t ballot(bool p) const
    {
        const uint64_t m = __ballot(p);
        if constexpr (GL == 64)
            return m;
        else
            return (m >> gb) & ((1ull << GL) - 1ull);
    }
    __device__ __forceinline__ bool any(bool p) const { return ballot(p) != 0ull; }
    __device__ __forceinline__ uint64_t below() const { return (1ull << gl) - 1ull; }
    __device__ __forceinline__ uint32_t xr(uint32_t v) const
    {
        if constexpr (GL == 64)
            return gw_xor(v);
        if constexpr (GL == 4) { /* pairs, then quads */
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false); /* quad_perm [1,0,3,2] */
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false); /* quad_perm [2,3,0,1] */
            return v;
        }
        if constexpr (GL == 8) { /* pairs, quads, then the half-row mirror joins the two quads */
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  /* quad_perm [1,0,3,2] */
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  /* quad_perm [2,3,0,1] */
            v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xf, 0xf, false); /* row_half_mirror */
            return v;
        }
        if constexpr (GL == 32) {
            const auto b = __builtin_amdgcn_permlane16_swap(v, v, false, false);
            v = b[0] ^ b[1];
        }
        v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xf, 0xf, false); /* row_ror:8 */
        v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x124, 0xf, 0xf, false); /* row_ror:4 */
        v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xf, 0xf, false);  /* quad_perm [2,3,0,1] */
        v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xf, 0xf, false);  /* quad_perm [1,0,3,2] */
        return v;
    }
    /* out[i] = v[i - 1] over the four slots (index i = gl + GL q), out[0] = first */
    __device__ __forceinline__ void shift(const uint32_t (&v)[4], uint32_t (&out)[4], uint32_t first,
                                          uint32_t nq) const
    {
        if constexpr (GL == 64) {
            gw_shift(v, out, gl, first, nq);
        } else if constexpr (GL == 32) {
            uint32_t carry = first;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((uint32_t)q < nq) {
                    const uint32_t t0 = (uint32_t)__builtin_amdgcn_readlane((int)v[q], 31);
                    const uint32_t t1 = (uint32_t)__builtin_amdgcn_readlane((int)v[q], 63);
                    const uint32_t u = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[q], 0x138, 0xf, 0xf, true);
                    out[q] = gl ? u : carry; /* wave_shr:1; each half's lane 0 takes the carry */
                    carry = gb ? t1 : t0;
                }
            }
        } else if constexpr (GL == 16) {
            uint32_t carry = first;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((uint32_t)q < nq) {
                    const uint32_t u = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[q], 0x121, 0xf, 0xf, false);
                    out[q] = gl ? u : carry; /* row_ror:1: lane 0 sees lane 15, the next slot's carry */
                    carry = u;
                }
            }
        } else if constexpr (GL == 4) {
            uint32_t carry = first;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((uint32_t)q < nq) {
                    const uint32_t u = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[q], 0x93, 0xf, 0xf, false);
                    out[q] = gl ? u : carry; /* quad_perm [3,0,1,2]: lane 0 sees lane 3, the next slot's carry */
                    carry = u;
                }
            }
        } else { /* GL == 8 */
            uint32_t carry = first;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if ((uint32_t)q < nq) {
                    const uint32_t u = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[q], 0x111, 0xf, 0xf, true);
                    const uint32_t hm = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v[q], 0x141, 0xf, 0xf, false);
                    out[q] = gl ? u : carry; /* row_shr:1; lane 0 of each half-row takes the carry */
                    carry = hm;              /* row_half_mirror: lane 0 (8) sees lane 7 (15) */
                }
            }
        }
    }
};

/* the tables: one global load per thread and table, al2 from the LDS copy
 * (its six entries per thread loaded from global one after another had cost
 * a few us per launch) */
__device__ __forceinline__ void gw_fill_al2(uint8_t *al2, const uint8_t *alog_lds, uint32_t nn)
{
    for (uint32_t x = threadIdx.x; x < GW_AL2; x += blockDim.x)
        al2[x] = x < nn ? alog_lds[x] : (x < 2u * nn ? alog_lds[x - nn] : (uint8_t)0);
}

template <typename SM>
__device__ __forceinline__ void gw_tables(SM &sm, const RsGenTables *__restrict__ T, uint32_t nn)
{
    for (uint32_t t = threadIdx.x; t < 256u; t += blockDim.x) {
        sm.alog[t] = T->alog[t];
        const uint32_t l = T->log[t];
        sm.log[t] = (uint8_t)l;
        sm.lgz[t] = t ? l : GW_Z;
    }
    __syncthreads();
    gw_fill_al2(sm.al2, sm.alog, nn);
}

/* sv[q] ^= sum over the row's bytes b < total of al2[lr[b] + e_q(b)], e_q
 * stepping down by sg[q] mod nn per byte: the byte logs read eight at a time
 * as one 16-byte broadcast (every lane of the group reads the same address;
 * the row's logs past `total` are GW_Z, so the last chunk needs no guard),
 * the NQ slots' lookups independent of each other and of the next byte's */
template <int NQ>
__device__ __forceinline__ void gw_syn_rows(const uint8_t *al2, const uint16_t *lr, uint32_t total, uint32_t nn,
                                            uint32_t (&e)[4], const uint32_t (&sg)[4], uint32_t (&sv)[4])
{
#pragma unroll 1
    for (uint32_t b0 = 0; b0 < total; b0 += 8u) {
        const uint4 v = *reinterpret_cast<const uint4 *>(lr + b0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t l = (w[k >> 1] >> (16 * (k & 1))) & 0xffffu;
#pragma unroll
            for (int q = 0; q < NQ; ++q) {
                sv[q] ^= al2[l + e[q]];
                const uint32_t t = e[q] - sg[q]; /* e - sg mod nn: the wrapped difference or it plus nn */
                e[q] = min(t, t + nn);
            }
        }
    }
}

/* syndromes of the row in W.cw / W.lr into W.S / W.sz; true if any is nonzero
 * (src/decode.c:375-415).  qf: (fcr + nr - 1) prim + nn - 1 < 2^16, so the
 * reference's Horner step multiplies by the constant alpha^((fcr + i) prim
 * mod nn) and S_i = sum_b r_b alpha^(s_i (total - 1 - b)): independent terms,
 * G = 64 / nr lanes per root for short root counts (partial sums XORed in
 * LDS).  Else the reference's Horner, one root per lane. */
template <int GL, typename SM, typename WT>
__device__ bool gw_syndromes(const SM &sm, WT &W, const RsGenParams &P, const GMod &mod, const GwGrp<GL> &G, bool qf)
{
    constexpr uint32_t GLU = GL;
    const uint32_t lane = G.gl;
    const uint32_t nr = P.nroots, nn = P.nn, A0 = P.nn, total = P.size + nr;
    const uint8_t *al2 = sm.al2, *lg = sm.log, *alog = sm.alog;
    uint32_t sv[4] = {0, 0, 0, 0};
    if (qf) {
        const uint32_t Gr = nr <= GLU / 2u ? GLU / nr : 1u;
        const uint32_t U = nr * Gr;
        if (Gr > 1u) {
            if (lane < nr)
                W.acc[lane] = 0;
            gw_sync();
        }
        /* G > 1: one unit per lane (q = 0); G = 1: units lane + 64 q, all over
         * every byte -- one broadcast read of the byte's log for all of them */
        const uint32_t g = Gr > 1u ? lane / nr : 0u;
        const uint32_t nq = (U + GLU - 1u) / GLU; /* register slots in use (uniform) */
        uint32_t e[4], sg[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t u = lane + GLU * q;
            const uint32_t i = Gr > 1u ? lane % nr : u;
            const uint32_t sx = mod((P.fcr + i) * P.prim);
            sg[q] = mod(sx * Gr);
            e[q] = g < total ? mod(sx * (total - 1u - g)) : 0u;
        }
        if (Gr > 1u) {
            if (lane < U) {
#pragma unroll 4
                for (uint32_t b = g; b < total; b += Gr) {
                    sv[0] ^= al2[W.lr[b] + e[0]];
                    e[0] = e[0] >= sg[0] ? e[0] - sg[0] : e[0] + nn - sg[0];
                }
            }
        } else if (nq == 1u) {
            gw_syn_rows<1>(al2, W.lr, total, nn, e, sg, sv);
        } else if (nq == 2u) {
            gw_syn_rows<2>(al2, W.lr, total, nn, e, sg, sv);
        } else {
            gw_syn_rows<4>(al2, W.lr, total, nn, e, sg, sv);
        }
        if (Gr > 1u && lane < U)
            atomicXor(&W.acc[lane % nr], sv[0]);
        if (Gr > 1u) {
            gw_sync();
            sv[0] = lane < nr ? W.acc[lane] : 0u;
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = lane + GLU * q;
            if (i < nr) {
                const uint32_t step = P.fcr * P.prim + i * P.prim; /* int arithmetic, truncated inside gf_mod */
                uint32_t v = (uint32_t)W.cw[0] & A0;
                for (uint32_t b = 1; b < total; ++b) {
                    const uint32_t in = (uint32_t)W.cw[b] & A0;
                    v = v ? (in ^ alog[mod((uint32_t)lg[v] + step)]) : in;
                }
                sv[q] = v;
            }
        }
    }
    bool nz = false;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = lane + GLU * q;
        if (i < nr) {
            const uint32_t l = lg[sv[q]];
            W.S[i] = (uint8_t)l;
            W.sz[i] = sv[q] ? l : GW_Z;
            nz |= sv[q] != 0u;
        }
    }
    gw_sync();
    return G.any(nz);
}

/* Chien sums over NP slots of points: acc[q] ^= sum_(j = 1..deg) al2[lamz[j] +
 * j pm[q] mod nn], the locator's logs read eight at a time as one 16-byte
 * broadcast (entries outside 1..deg masked to GW_Z: the array past nr is not
 * written) */
template <int NP>
__device__ __forceinline__ void gw_chien_rows(const uint8_t *al2, const uint16_t *lamz, uint32_t deg, uint32_t nn,
                                              const uint32_t (&pm)[4], uint32_t (&acc)[4])
{
    uint32_t tt[4] = {0, 0, 0, 0}; /* j pm mod nn */
#pragma unroll 1
    for (uint32_t j0 = 0; j0 <= deg; j0 += 8u) {
        const uint4 v = *reinterpret_cast<const uint4 *>(lamz + j0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t j = j0 + (uint32_t)k;
            const uint32_t lz = (j >= 1u && j <= deg) ? (w[k >> 1] >> (16 * (k & 1))) & 0xffffu : GW_Z;
#pragma unroll
            for (int q = 0; q < NP; ++q) {
                acc[q] ^= al2[lz + tt[q]];
                const uint32_t t = tt[q] + pm[q];
                tt[q] = min(t, t - nn); /* t < 2 nn: mod nn (t - nn wraps above t when t < nn) */
            }
        }
    }
}

#ifndef GW_NARROW
#define GW_NARROW 1 /* Berlekamp-Massey on fewer register slots while the high ones stay zero (gw_bm narrow) */
#endif

/* true when some group's B holds a nonzero at index GL NQ - 1 (its last lane,
 * slot NQ - 1): the next shift would carry it into slot NQ (wave-uniform) */
template <int NQ, int GL>
__device__ __forceinline__ bool gw_top_set(const GwGrp<GL> &G, const uint32_t (&B)[4])
{
    if constexpr (GL == 64)
        return (uint32_t)__builtin_amdgcn_readlane((int)B[NQ - 1], 63) != GW_Z;
    else
        return __ballot(G.gl == (uint32_t)GL - 1u && B[NQ - 1] != GW_Z) != 0ull;
}

/* Berlekamp-Massey, src/decode.c:49-96, iterations r0 .. nr over NQ register
 * slots (index i = gl + GL q): a zero discrepancy (disc = GW_Z) leaves Lambda
 * as it is -- every product lands on al2's zero region -- and only shifts B,
 * as the reference's `continue`.  B in GW_Z form; L returns the length.
 * narrow: the slots from NQ on hold zeros (Lambda 0, B GW_Z) and stay so
 * while B's top index GL NQ - 1 is zero before a shift (deg Lambda <= L,
 * deg x B <= r - L: a word with nr / 2 errors keeps both at most nr / 2, so
 * RS(255,155)'s 100 roots run on one slot of 64); the run stops before the
 * first iteration whose shift would carry a nonzero out and returns it for
 * a wider run to continue from (nr + 1: done) */
template <int NQ, int GL, typename SM>
__device__ __forceinline__ uint32_t gw_bm(const SM &sm, const uint16_t *sz, const GwGrp<GL> &G, uint32_t r0,
                                          uint32_t nr, uint32_t nn, uint32_t ne, bool narrow, uint32_t (&lam)[4],
                                          uint32_t (&B)[4], uint32_t &L)
{
    constexpr uint32_t GLU = GL;
    const uint16_t *lgz = sm.lgz;
    const uint8_t *al2 = sm.al2;
    uint32_t Bm[4];
    for (uint32_t r = r0; r <= nr; ++r) {
        if (narrow && gw_top_set<NQ>(G, B))
            return r;
        uint32_t part = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int32_t idx = (int32_t)r - 1 - (int32_t)(G.gl + GLU * q); /* S_(r-1-i); none for i >= r */
            const uint32_t sv = sz[idx > 0 ? idx : 0];
            part ^= al2[lgz[lam[q]] + (idx >= 0 ? sv : GW_Z)];
        }
        const uint32_t dv = G.xr(part);
        const uint32_t disc = lgz[dv];
        const bool lengthen = dv != 0u && 2u * L <= r + ne - 1u;
        G.shift(B, Bm, GW_Z, NQ);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const uint32_t old = lam[q];
            lam[q] = old ^ al2[disc + Bm[q]];
            const uint32_t t = lgz[old];
            const uint32_t v = t + nn - disc;
            const uint32_t bl = t == GW_Z ? GW_Z : (v >= nn ? v - nn : v);
            B[q] = lengthen ? bl : Bm[q];
        }
        if (lengthen)
            L = r + ne - L;
    }
    return nr + 1u;
}

/* src/decode.c:17-230 for the row in W (syndromes in W.S / W.sz): erasure
 * locator, BM, degree, Chien, Omega, Forney, re-syndrome check, apply
 * (in place in data / parity from W.cw).  Same results as g_correct. */
/* gw_bm for two codewords at once (errors mode, ne = 0), their iterations
 * interleaved in one instruction stream: every step of one codeword's chain
 * (lookups, the group XOR, the B shift) has the other's beside it, so the
 * wave waits on half as many latencies per codeword (long codes, whose
 * nr serial iterations bound a lone wave) */
template <int NQ, int GL, typename SM>
__device__ __forceinline__ uint32_t gw_bm2(const SM &sm, const uint16_t *szA, const uint16_t *szB,
                                           const GwGrp<GL> &G, uint32_t r0, uint32_t nr, uint32_t nn, bool narrow,
                                           uint32_t (&lamA)[4], uint32_t (&BA)[4], uint32_t &LA,
                                           uint32_t (&lamB)[4], uint32_t (&BB)[4], uint32_t &LB)
{
    constexpr uint32_t GLU = GL;
    const uint16_t *lgz = sm.lgz;
    const uint8_t *al2 = sm.al2;
    uint32_t BmA[4], BmB[4];
    for (uint32_t r = r0; r <= nr; ++r) {
        if (narrow && (gw_top_set<NQ>(G, BA) || gw_top_set<NQ>(G, BB)))
            return r;
        uint32_t pa = 0, pb = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const int32_t idx = (int32_t)r - 1 - (int32_t)(G.gl + GLU * q);
            const uint32_t ix = idx > 0 ? (uint32_t)idx : 0u;
            const uint32_t sa = szA[ix], sb = szB[ix];
            pa ^= al2[lgz[lamA[q]] + (idx >= 0 ? sa : GW_Z)];
            pb ^= al2[lgz[lamB[q]] + (idx >= 0 ? sb : GW_Z)];
        }
        const uint32_t dva = G.xr(pa), dvb = G.xr(pb);
        const uint32_t da = lgz[dva], db = lgz[dvb];
        const bool la = dva != 0u && 2u * LA <= r - 1u, lb = dvb != 0u && 2u * LB <= r - 1u;
        G.shift(BA, BmA, GW_Z, NQ);
        G.shift(BB, BmB, GW_Z, NQ);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
            const uint32_t oa = lamA[q], ob = lamB[q];
            lamA[q] = oa ^ al2[da + BmA[q]];
            lamB[q] = ob ^ al2[db + BmB[q]];
            const uint32_t ta = lgz[oa], tb = lgz[ob];
            const uint32_t va = ta + nn - da, vb = tb + nn - db;
            const uint32_t ba = ta == GW_Z ? GW_Z : (va >= nn ? va - nn : va);
            const uint32_t bb = tb == GW_Z ? GW_Z : (vb >= nn ? vb - nn : vb);
            BA[q] = la ? ba : BmA[q];
            BB[q] = lb ? bb : BmB[q];
        }
        if (la)
            LA = r - LA;
        if (lb)
            LB = r - LB;
    }
    return nr + 1u;
}

/* src/decode.c:98-230 after Berlekamp-Massey, for the locator lam (values,
 * index i = gl + GL q): degree, Chien, Omega, Forney, re-syndrome check,
 * apply (in place in data / parity from W.cw) */
template <typename PosT, int GL, typename SM, typename WT>
__device__ bool gw_finish(const SM &sm, WT &W, const RsGenParams &P, const GMod &mod, const GwGrp<GL> &G,
                          uint8_t *data, uint8_t *parity, const PosT *pos, bool eras_apply, uint32_t &corrected,
                          const uint32_t (&lam)[4])
{
    constexpr uint32_t GLU = GL;
    const uint32_t lane = G.gl;
    const uint32_t nr = P.nroots, nn = P.nn, A0 = P.nn, size = P.size;
    const int32_t pad = P.pad;
    const uint8_t *alog = sm.alog, *lg = sm.log, *al2 = sm.al2;
    const uint32_t nq = (nr + GLU) / GLU; /* register slots holding indices 0 .. nr (uniform) */
#if GW_PHASE_STOP == 2 /* experiment builds only: time the phases before this one */
    return false;
#endif
    /* locator to log form, degree, src/decode.c:98-110 */
    uint32_t deg = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = lane + GLU * q;
        const uint32_t l = lg[lam[q]];
        const bool valid = (uint32_t)q < nq && i <= nr;
        if (valid)
            W.lamz[i] = l == A0 ? GW_Z : l;
        const uint64_t m = G.ballot(valid && l != A0);
        if (m)
            deg = GLU * q + 63u - (uint32_t)__clzll((long long)m);
    }
    if (deg == 0u)
        return false;
    gw_sync();

#if GW_PHASE_STOP == 3 /* experiment builds only: time the phases before this one */
    return false;
#endif
    /* Chien search, src/decode.c:112-145: point i = lane + 1 + 64 q; the
     * first deg roots in ascending order, the padding check on each */
    {
        uint32_t acc[4], pm[4], tt[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t pt = lane + 1u + GLU * q;
            pm[q] = pt >= nn ? pt - nn : pt;
            acc[q] = 1;
            tt[q] = 0;
        }
        const uint32_t np = (nn + GLU - 1u) / GLU; /* slots holding the points 1 .. nn (uniform) */
        (void)tt;
        if (np == 1u)
            gw_chien_rows<1>(al2, W.lamz, deg, nn, pm, acc);
        else if (np == 2u)
            gw_chien_rows<2>(al2, W.lamz, deg, nn, pm, acc);
        else
            gw_chien_rows<4>(al2, W.lamz, deg, nn, pm, acc);
        uint32_t base = 0;
        bool padbad = false;
        const uint64_t below = G.below();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t pt = lane + 1u + GLU * q;
            const bool root = pt <= nn && acc[q] == 0u;
            const uint64_t m = G.ballot(root);
            const uint32_t rank = base + (uint32_t)__popcll(m & below);
            if (root && rank < deg) {
                const uint32_t k = mod(pt * P.iprim - 1u);
                W.roots[rank] = (uint8_t)pt;
                W.locs[rank] = (uint8_t)k;
                padbad |= (int32_t)k < pad;
            }
            base += (uint32_t)__popcll(m);
        }
        if (G.any(padbad) || base < deg)
            return false;
    }
    gw_sync();

#if GW_PHASE_STOP == 4 /* experiment builds only: time the phases before this one */
    return false;
#endif
    /* Omega = S Lambda mod x^deg, log form, src/decode.c:147-158 */
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = lane + GLU * q;
        if (i < deg) {
            uint32_t acc = 0;
#pragma unroll 4
            for (uint32_t j = 0; j <= i; ++j)
                acc ^= al2[W.sz[i - j] + W.lamz[j]];
            W.omz[i] = acc ? lg[acc] : GW_Z;
        }
    }
    gw_sync();

#if GW_PHASE_STOP == 5 /* experiment builds only: time the phases before this one */
    return false;
#endif
    /* Forney, src/decode.c:159-191 (corrected counts nonzero numerators) */
    const uint32_t dtop = (deg < nr - 1u ? deg : nr - 1u) & ~1u;
    uint32_t fixed = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t jj = lane + GLU * q;
        uint32_t num = 0;
        if (jj < deg) {
            const uint32_t rt = W.roots[jj];
            const uint32_t rm = rt >= nn ? rt - nn : rt;
            uint32_t t = 0;
#pragma unroll 4
            for (uint32_t i = 0; i < deg; ++i) {
                num ^= al2[W.omz[i] + t];
                t += rm;
                t = t >= nn ? t - nn : t;
            }
            uint32_t mg = 0;
            if (num != 0u) {
                const uint32_t num2 = alog[mod((uint32_t)((int32_t)rt * ((int32_t)P.fcr - 1) + (int32_t)A0))];
                uint32_t den = 0;
#pragma unroll 4
                for (int32_t i = (int32_t)dtop; i >= 0; i -= 2)
                    den ^= al2[W.lamz[(uint32_t)i + 1u] + mod((uint32_t)i * rt)];
                mg = alog[mod((uint32_t)lg[num] + lg[num2] + A0 - lg[den])];
            }
            W.mag[jj] = (uint8_t)mg;
            W.lgm[jj] = mg ? (uint32_t)lg[mg] : 0xffffu;
            W.lx[jj] = A0 - (uint32_t)W.locs[jj] - 1u;
        }
        fixed += (uint32_t)__popcll(G.ballot(jj < deg && num != 0u));
    }
    corrected = fixed;
    gw_sync();

#if GW_PHASE_STOP == 6 /* experiment builds only: time the phases before this one */
    return false;
#endif
    /* re-syndrome check, src/decode.c:193-209 (int16 exponent) */
    {
        bool bad = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = lane + GLU * q;
            if (i < nr) {
                uint32_t acc = 0;
                const uint32_t fi = (P.fcr + i) * P.prim;
#pragma unroll 4
                for (uint32_t j = 0; j < deg; ++j) {
                    const uint32_t lm = W.lgm[j];
                    const int32_t kk = (int16_t)(uint16_t)(fi * (uint32_t)W.lx[j]);
                    const uint32_t v = alog[mod((uint32_t)((int32_t)lm + kk))];
                    acc ^= lm == 0xffffu ? 0u : v;
                }
                bad |= acc != alog[W.S[i]];
            }
        }
        if (G.any(bad))
            return false;
    }

#if GW_PHASE_STOP == 7 /* experiment builds only: time the phases before this one */
    return false;
#endif
    /* apply, src/decode.c:211-227, from the row's copy in W.cw */
    const uint32_t total = size + nr;
    if (eras_apply) {
        /* quirk Q1/Q2: magnitude j goes to slot j (repeated slots accumulate);
         * slots past data[] address parity (p < size + nr) or are dropped */
        W.acc[lane] = 0;
        gw_sync();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t jj = lane + GLU * q;
            if (jj < deg) {
                const uint32_t p = (uint32_t)pos[jj], mg = W.mag[jj];
                if (mg != 0u && p < total)
                    atomicXor(&W.acc[p >> 2], mg << (8u * (p & 3u)));
            }
        }
        gw_sync();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t b = lane + GLU * q;
            if (b < total) {
                const uint32_t dl = (W.acc[b >> 2] >> (8u * (b & 3u))) & 0xffu;
                if (dl != 0u) {
                    const uint8_t v = (uint8_t)(W.cw[b] ^ dl);
                    if (b < size)
                        data[b] = v;
                    else
                        parity[b - size] = v;
                }
            }
        }
        return true;
    }
    /* error locations: the reference stops at the first one outside the row
     * (those before it applied) */
    uint32_t first_bad = deg;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t jj = lane + GLU * q;
        const int32_t p = (int32_t)W.locs[jj < 4u * GLU ? jj : 0u] - pad;
        const uint64_t m = G.ballot(jj < deg && !(p >= 0 && p < (int32_t)total));
        if (m != 0ull && first_bad == deg)
            first_bad = GLU * q + (uint32_t)__builtin_ctzll(m);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t jj = lane + GLU * q;
        if (jj < first_bad) {
            const uint32_t p = (uint32_t)((int32_t)W.locs[jj] - pad), mg = W.mag[jj];
            if (mg != 0u) {
                const uint8_t v = (uint8_t)(W.cw[p] ^ mg);
                if (p < size)
                    data[p] = v;
                else
                    parity[p - size] = v;
            }
        }
    }
    return first_bad == deg;
}

template <typename PosT, int GL, typename SM, typename WT>
__device__ bool gw_correct(const SM &sm, WT &W, const RsGenParams &P, const GMod &mod, const GwGrp<GL> &G,
                           uint8_t *data, uint8_t *parity, uint32_t ne, const PosT *pos, bool eras_apply,
                           uint32_t &corrected)
{
    constexpr uint32_t GLU = GL;
    const uint32_t lane = G.gl;
    const uint32_t nr = P.nroots, nn = P.nn, A0 = P.nn;
    const int32_t pad = P.pad;
    const uint8_t *al2 = sm.al2;
    const uint32_t nq = (nr + GLU) / GLU; /* register slots holding indices 0 .. nr (uniform) */
    uint32_t lam[4], B[4], Bm[4];
#pragma unroll
    for (int q = 0; q < 4; ++q)
        lam[q] = (lane + GLU * q) == 0u ? 1u : 0u;

    /* Sentinel logs: lgz[0] = GW_Z and W.sz use GW_Z for zero, and every sum
     * with a GW_Z operand indexes al2's zero region (512 + 254 and 1024 are
     * both >= 2 nn), so no step below branches on a zero operand: each
     * slot's lookups issue together instead of one guarded chain per slot */
    const uint16_t *lgz = sm.lgz;

    /* erasure locator prod (1 + X_l x), src/decode.c:31-47 */
    if (ne > 0u) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = lane + GLU * q;
            if (i < ne)
                W.acc[i] = (uint32_t)pos[i];
        }
        gw_sync();
        for (uint32_t e = 0; e < ne; ++e) {
            const uint32_t xl = mod(P.prim * (A0 - 1u - (W.acc[e] + (uint32_t)pad)));
            G.shift(lam, Bm, 0u, nq);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if ((uint32_t)q < nq)
                    lam[q] ^= al2[xl + lgz[Bm[q]]];
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
        B[q] = lgz[lam[q]]; /* B in GW_Z form */

    /* Berlekamp-Massey, src/decode.c:49-96 (gw_bm), the slot count a
     * compile-time constant so that the slots' lookups issue together */
    uint32_t L = ne;
    if (nq == 1u) {
        gw_bm<1>(sm, W.sz, G, ne + 1u, nr, nn, ne, false, lam, B, L);
    } else if (nq == 2u) { /* one slot while nothing reaches the second */
        const uint32_t r = GW_NARROW && ne < GLU ? gw_bm<1>(sm, W.sz, G, ne + 1u, nr, nn, ne, true, lam, B, L) : ne + 1u;
        if (r <= nr)
            gw_bm<2>(sm, W.sz, G, r, nr, nn, ne, false, lam, B, L);
    } else { /* two slots while nothing reaches the third */
        const uint32_t r = GW_NARROW && ne < 2u * GLU ? gw_bm<2>(sm, W.sz, G, ne + 1u, nr, nn, ne, true, lam, B, L) : ne + 1u;
        if (r <= nr)
            gw_bm<4>(sm, W.sz, G, r, nr, nn, ne, false, lam, B, L);
    }
    (void)Bm;
    return gw_finish<PosT>(sm, W, P, mod, G, data, parity, pos, eras_apply, corrected, lam);
}

/* One codeword on one wave, branch logic of src/decode.c:431-487: x (the
 * row's external log-form syndromes) or pos / ne (its erasure slots and
 * count) or neither; ok / corrected_num to okp / corp (corp may be NULL) */
template <typename PosT, int GL, typename SM, typename WT>
__device__ void gw_decode_one(const SM &sm, WT &W, const RsGenParams &P, const GMod &mod, const GwGrp<GL> &G,
                              bool qf, uint8_t *d, uint8_t *par, const uint16_t *x, const PosT *pos, uint32_t ne,
                              uint8_t *okp, uint8_t *corp)
{
    constexpr uint32_t GLU = GL;
    const uint32_t lane = G.gl;
    const uint32_t nr = P.nroots, A0 = P.nn, size = P.size, total = size + nr;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t b = lane + GLU * q;
        const uint32_t v = b < size ? d[b] : (b < total ? par[b - size] : 0u);
        const uint32_t m = v & A0;
        W.cw[b] = (uint8_t)v;
        W.lr[b] = m ? (uint32_t)sm.log[m] : GW_Z;
    }
    uint32_t fixed = 0;
    bool good;
    if (x) {
        bool bad = false, any = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t i = lane + GLU * q;
            if (i < nr) {
                const uint32_t v = x[i];
                bad |= v > A0;
                any |= v != A0;
                W.S[i] = (uint8_t)v;
                W.sz[i] = v == A0 ? GW_Z : (v & 0xffu);
            }
        }
        bad = G.any(bad);
        any = G.any(any);
        gw_sync();
        good = !bad &&
               (!any || gw_correct<PosT>(sm, W, P, mod, G, d, par, 0u, (const PosT *)nullptr, false, fixed));
    } else {
        gw_sync();
        const bool dirty = gw_syndromes(sm, W, P, mod, G, qf);
#if GW_PHASE_STOP == 1
        if (okp) { /* experiment builds only */
            if (lane == 0u)
                *okp = dirty;
            return;
        }
#endif
        if (pos)
            good = !dirty || (ne <= nr && gw_correct<PosT>(sm, W, P, mod, G, d, par, ne, pos, true, fixed));
        else
            good = !dirty || gw_correct<PosT>(sm, W, P, mod, G, d, par, 0u, (const PosT *)nullptr, false, fixed);
    }
    if (lane == 0u) {
        *okp = good ? 1 : 0;
        if (corp)
            *corp = (uint8_t)fixed;
    }
    gw_sync();
}

/* the row [data | parity] of one codeword into W.cw (and its logs into W.lr) */
template <int GL, typename SM, typename WT>
__device__ __forceinline__ void gw_load_row(const SM &sm, WT &W, const RsGenParams &P, const GwGrp<GL> &G,
                                            const uint8_t *d, const uint8_t *par, bool logs)
{
    constexpr uint32_t GLU = GL;
    const uint32_t size = P.size, total = size + P.nroots;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t b = G.gl + GLU * q;
        const uint32_t v = b < size ? d[b] : (b < total ? par[b - size] : 0u);
        const uint32_t m = v & P.nn;
        W.cw[b] = (uint8_t)v;
        if (logs)
            W.lr[b] = m ? (uint32_t)sm.log[m] : GW_Z;
    }
}

/* Two codewords on one wave, errors mode (no erasure list, no external
 * syndromes), nroots < 2 GL: syndromes of A (kept in the side buffer) and of
 * B (in the row), Berlekamp-Massey of both interleaved (gw_bm2), then the
 * rest for B and, with A's row reloaded and its syndromes restored, for A.
 * Same results as gw_decode_one on each. */
template <int GL, typename SM, typename WT>
__device__ void gw_decode_pair(const SM &sm, WT &W, uint8_t *sideS, uint16_t *sideSz, uint8_t *sideLam,
                               const RsGenParams &P,
                               const GMod &mod, const GwGrp<GL> &G, bool qf, uint8_t *dA, uint8_t *pA, uint8_t *okA,
                               uint8_t *corA, uint8_t *dB, uint8_t *pB, uint8_t *okB, uint8_t *corB)
{
    constexpr uint32_t GLU = GL;
    const uint32_t nr = P.nroots, nq = (nr + GLU) / GLU;
    const uint32_t lane = G.gl;
    gw_load_row(sm, W, P, G, dA, pA, true);
    gw_sync();
    const bool dirtyA = gw_syndromes(sm, W, P, mod, G, qf);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t i = lane + GLU * q;
        if (i < nr) {
            sideS[i] = W.S[i];
            sideSz[i] = W.sz[i];
        }
    }
    gw_load_row(sm, W, P, G, dB, pB, true);
    gw_sync();
    const bool dirtyB = gw_syndromes(sm, W, P, mod, G, qf);
    /* Berlekamp-Massey of the dirty ones (both: interleaved), each locator
     * parked in LDS, then one finish per dirty codeword: B (in the row), then
     * A with its row reloaded and its syndromes restored */
    uint32_t lam[4], Bl[4];
    if (dirtyA || dirtyB) {
        uint32_t lamB[4], BB[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            lam[q] = lamB[q] = (lane + GLU * q) == 0u ? 1u : 0u;
            Bl[q] = BB[q] = sm.lgz[lam[q]];
        }
        uint32_t L = 0;
        if (dirtyA && dirtyB) {
            uint32_t LA = 0, LB = 0;
            if (nq == 1u) {
                gw_bm2<1>(sm, sideSz, W.sz, G, 1u, nr, P.nn, false, lam, Bl, LA, lamB, BB, LB);
            } else { /* one slot while nothing reaches the second */
                const uint32_t r = GW_NARROW ? gw_bm2<1>(sm, sideSz, W.sz, G, 1u, nr, P.nn, true, lam, Bl, LA, lamB, BB, LB)
                                             : 1u;
                if (r <= nr)
                    gw_bm2<2>(sm, sideSz, W.sz, G, r, nr, P.nn, false, lam, Bl, LA, lamB, BB, LB);
            }
        } else if (nq == 1u) {
            gw_bm<1>(sm, dirtyA ? sideSz : W.sz, G, 1u, nr, P.nn, 0u, false, dirtyA ? lam : lamB, dirtyA ? Bl : BB, L);
        } else {
            const uint32_t r = GW_NARROW ? gw_bm<1>(sm, dirtyA ? sideSz : W.sz, G, 1u, nr, P.nn, 0u, true,
                                                    dirtyA ? lam : lamB, dirtyA ? Bl : BB, L)
                                           : 1u;
            if (r <= nr)
                gw_bm<2>(sm, dirtyA ? sideSz : W.sz, G, r, nr, P.nn, 0u, false, dirtyA ? lam : lamB, dirtyA ? Bl : BB, L);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            sideLam[lane + GLU * q] = (uint8_t)lam[q];
            sideLam[4u * GLU + lane + GLU * q] = (uint8_t)lamB[q];
        }
    }
    uint32_t fixA = 0, fixB = 0;
    bool goodA = true, goodB = true;
#pragma unroll 1
    for (int k = 0; k < 2; ++k) { /* k = 0: B, 1: A */
        if (k == 0 ? !dirtyB : !dirtyA)
            continue;
        if (k == 1) { /* the row holds B: A's bytes and syndromes back */
            gw_sync();
            gw_load_row(sm, W, P, G, dA, pA, false);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = lane + GLU * q;
                if (i < nr) {
                    W.S[i] = sideS[i];
                    W.sz[i] = sideSz[i];
                }
            }
        }
        gw_sync();
#pragma unroll
        for (int q = 0; q < 4; ++q)
            lam[q] = sideLam[(k == 0 ? 4u * GLU : 0u) + lane + GLU * q];
        uint32_t fix = 0;
        const bool good = gw_finish<uint8_t>(sm, W, P, mod, G, k == 0 ? dB : dA, k == 0 ? pB : pA,
                                             (const uint8_t *)nullptr, false, fix, lam);
        if (k == 0)
            goodB = good, fixB = fix;
        else
            goodA = good, fixA = fix;
    }
    if (lane == 0u) {
        *okA = goodA ? 1 : 0;
        *okB = goodB ? 1 : 0;
        if (corA) {
            *corA = (uint8_t)fixA;
            *corB = (uint8_t)fixB;
        }
    }
    gw_sync();
}

/* Full decode, one codeword per GL lanes (rsg_decode_k's modes: ext /
 * erasure slots / errors; list mode): GL = 64 one codeword per wave, 32 / 16
 * two / four per wave for codes of up to 127 / 63 symbols */
#ifndef GW_PAIR
#define GW_PAIR 1 /* rsgw_decode_k<., 64>: two codewords per pass in errors mode (gw_decode_pair) */
#endif
#ifndef GW_WAVES
#define GW_WAVES 4 /* waves per SIMD the decode kernel is register-bound to (124-128 VGPRs) */
#endif
template <typename PosT, int GL>
__global__ __launch_bounds__(GW_WG, GW_WAVES) void rsgw_decode_k(const RsGenTables *__restrict__ T, RsGenParams P,
                                                           uint8_t *data, size_t dstride, uint8_t *parity,
                                                           size_t pstride, size_t count,
                                                           const uint16_t *__restrict__ ext, size_t ext_stride,
                                                           const PosT *__restrict__ pos, size_t pos_stride,
                                                           const uint8_t *__restrict__ cntv, uint8_t *__restrict__ ok,
                                                           uint8_t *__restrict__ corrected,
                                                           const uint32_t *__restrict__ list,
                                                           const uint32_t *__restrict__ list_n, uint32_t *flag,
                                                           uint32_t seq)
{
    constexpr uint32_t CPB = GW_WG / GL; /* codewords per workgroup pass */
    const size_t n = list ? (size_t)*list_n : count;
    if ((size_t)blockIdx.x * CPB >= n)
        return;
    __shared__ GwSmemG<GL> sm;
    const uint32_t t = threadIdx.x;
    const GwGrp<GL> G(t & 63u);
    const uint32_t slot = t / GL;
    gw_tables(sm, T, P.nn);
    __syncthreads();
    auto &W = sm.w[slot];
    const GMod mod{P.nn, P.magic};
    const bool qf = (P.fcr + P.nroots - 1u) * P.prim + P.nn - 1u < 65536u;
    const size_t stride = (size_t)gridDim.x * CPB;
    /* long codes in errors mode: two codewords per pass, their BM interleaved */
    const bool pair = GL == 64 && GW_PAIR && !ext && !pos && P.nroots < 2u * GL && P.nroots >= 8u;
    for (size_t e = (size_t)blockIdx.x * CPB + slot; e < n; e += pair ? 2u * stride : stride) {
        const size_t cw = list ? (size_t)list[e] : e;
        if (pair && e + stride < n) {
            const size_t c2 = list ? (size_t)list[e + stride] : e + stride;
            gw_decode_pair<GL>(sm, W, sm.sideS[slot], sm.sideSz[slot], sm.sideLam[slot], P, mod, G, qf,
                               data + cw * dstride,
                               parity + cw * pstride, ok + cw, corrected ? corrected + cw : nullptr,
                               data + c2 * dstride, parity + c2 * pstride, ok + c2,
                               corrected ? corrected + c2 : nullptr);
            continue;
        }
        gw_decode_one<PosT, GL>(sm, W, P, mod, G, qf, data + cw * dstride, parity + cw * pstride,
                                ext ? ext + cw * ext_stride : nullptr, pos ? pos + cw * pos_stride : nullptr,
                                pos ? (uint32_t)cntv[cw] : 0u, ok + cw, corrected ? corrected + cw : nullptr);
    }
    gw_done(flag, seq);
}

/* check / syndromes, one codeword per wave (rsg_check_k's outputs) */
__global__ __launch_bounds__(GW_WG) void rsgw_check_k(const RsGenTables *__restrict__ T, RsGenParams P,
                                                       const uint8_t *__restrict__ data, size_t dstride,
                                                       const uint8_t *__restrict__ parity, size_t pstride,
                                                       size_t count, uint8_t *__restrict__ dirty,
                                                       uint16_t *__restrict__ syn, size_t syn_stride)
{
    if ((size_t)blockIdx.x * (GW_WG / 64) >= count)
        return;
    __shared__ GwSmem sm;
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    gw_tables(sm, T, P.nn);
    __syncthreads();
    GwWave &W = sm.w[wave];
    const GMod mod{P.nn, P.magic};
    const uint32_t nr = P.nroots, A0 = P.nn, size = P.size, total = size + nr;
    const bool qf = (P.fcr + nr - 1u) * P.prim + A0 - 1u < 65536u;
    for (size_t e = (size_t)blockIdx.x * (GW_WG / 64) + wave; e < count; e += (size_t)gridDim.x * (GW_WG / 64)) {
        const uint8_t *d = data + e * dstride, *par = parity + e * pstride;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const uint32_t b = lane + 64u * q;
            const uint32_t v = b < size ? d[b] : (b < total ? par[b - size] : 0u);
            const uint32_t m = v & A0;
            W.cw[b] = (uint8_t)v;
            W.lr[b] = m ? (uint32_t)sm.log[m] : GW_Z;
        }
        gw_sync();
        const bool nz = gw_syndromes(sm, W, P, mod, GwGrp<64>(lane), qf);
        if (dirty && lane == 0u)
            dirty[e] = nz ? 1 : 0;
        if (syn) /* log form, the reference's uint16 array (src/decode.c:409-412) */
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t i = lane + 64u * q;
                if (i < nr)
                    syn[e * syn_stride + i] = W.S[i];
            }
        gw_sync();
    }
}

/* Encode, one message per wave: parity = sum_b d_b Q[size - 1 - b], Q[d] the
 * parity of the message 1 followed by d zeros (RsGenTables::encq, built on
 * the host by the reference's LFSR, src/encode.c:120-143, which is linear
 * in the masked message bytes). */

/* the rows Q[0 .. size) into qs (nr logs each, GW_Z: zero): 16-byte chunks,
 * up to four per thread issued before any is used (a row per step, one load
 * at a time, had cost ~0.3 us each) */
__device__ __forceinline__ void gw_stage_rows(uint16_t *qs, const RsGenTables *__restrict__ T, uint32_t size,
                                              uint32_t nr)
{
    const uint32_t t = threadIdx.x, nt = blockDim.x;
    const uint32_t cpr = (nr + 15u) / 16u, nch = size * cpr;
    for (uint32_t x0 = t; x0 < nch; x0 += 4u * nt) {
        uint4 v[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t x = x0 + (uint32_t)k * nt;
            if (x < nch)
                v[k] = *reinterpret_cast<const uint4 *>(T->encq + (x / cpr) * 256u + (x % cpr) * 16u);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t x = x0 + (uint32_t)k * nt;
            if (x < nch) {
                const uint32_t r = x / cpr, c = x % cpr;
                const uint32_t w[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
                for (int j = 0; j < 16; ++j) {
                    const uint32_t pp = c * 16u + (uint32_t)j;
                    const uint32_t b = (w[j >> 2] >> (8 * (j & 3))) & 0xffu;
                    if (pp < nr)
                        qs[r * nr + pp] = b == 0xffu ? GW_Z : b;
                }
            }
        }
    }
}

/* one message on one wave (lr: the wave's 256-entry log row); by_byte: lanes
 * over the message bytes, one XOR reduction per parity byte (single calls of
 * messages longer than their parity: RS(255,207) 25 vs 43 us per call,
 * RS(255,55) 46 vs 31, profiles/r05_general_lat_auto.log); else lane p (and
 * p + 64 ...) owns parity byte p over size serial steps */
__device__ __forceinline__ void gw_encode_one(const uint8_t *al2, const uint8_t *lg, uint16_t *lr, const uint16_t *qs,
                                              const RsGenParams &P, uint32_t lane, bool by_byte, const uint8_t *d,
                                              uint8_t *out)
{
    const uint32_t A0 = P.nn, nr = P.nroots, size = P.size;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t b = lane + 64u * q;
        if (b < size) {
            const uint32_t m = (uint32_t)d[b] & A0;
            lr[b] = m ? (uint32_t)lg[m] : GW_Z;
        }
    }
    gw_sync();
    uint32_t acc[4] = {0, 0, 0, 0};
    const uint32_t nq = (nr + 63u) / 64u;
    if (by_byte) {
        uint32_t lb[4], rb[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t b = lane + 64u * k;
            lb[k] = b < size ? (uint32_t)lr[b] : GW_Z;
            rb[k] = b < size ? (size - 1u - b) * nr : 0u;
        }
        for (uint32_t p = 0; p < nr; ++p) {
            uint32_t x = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                x ^= al2[lb[k] + qs[rb[k] + p]];
            x = gw_xor(x);
            if ((p & 63u) == lane)
                acc[p >> 6] = x;
        }
    } else {
#pragma unroll 4
        for (uint32_t b = 0; b < size; ++b) {
            const uint32_t l = lr[b]; /* zero byte or zero entry: a sentinel sum, al2's zero part */
            const uint16_t *row = qs + (size - 1u - b) * nr;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t p = lane + 64u * q;
                if ((uint32_t)q < nq && p < nr)
                    acc[q] ^= al2[l + row[p]];
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const uint32_t p = lane + 64u * q;
        if (p < nr)
            out[p] = (uint8_t)acc[q];
    }
    gw_sync();
}

__global__ __launch_bounds__(GW_WG) void rsgw_encode_k(const RsGenTables *__restrict__ T, RsGenParams P,
                                                        const uint8_t *__restrict__ data, size_t dstride,
                                                        uint8_t *__restrict__ parity, size_t pstride, size_t count,
                                                        uint32_t *flag, uint32_t seq)
{
    const bool by_byte = count <= 64u && P.size > P.nroots; /* single calls and tiny batches: latency */
    if ((size_t)blockIdx.x * (GW_WG / 64) >= count)
        return;
    __shared__ uint8_t al2[GW_AL2];
    __shared__ uint8_t lg[256];
    __shared__ uint16_t lr[GW_WG / 64][256];
    __shared__ uint16_t qs[GW_QS]; /* size + nr <= 255 */
    __shared__ uint8_t alog[256];
    const uint32_t t = threadIdx.x, lane = t & 63u, wave = t >> 6;
    lg[t] = T->log[t];
    alog[t] = T->alog[t];
    gw_stage_rows(qs, T, P.size, P.nroots);
    __syncthreads();
    gw_fill_al2(al2, alog, P.nn);
    __syncthreads();
    for (size_t e = (size_t)blockIdx.x * (GW_WG / 64) + wave; e < count; e += (size_t)gridDim.x * (GW_WG / 64))
        gw_encode_one(al2, lg, lr[wave], qs, P, lane, by_byte, data + e * dstride, parity + e * pstride);
    gw_done(flag, seq);
}

/*
 * rsgw_serve_k: the general-parameter single-call server, rs_serve_k's
 * protocol (rs_single.hip) with one wave: it stays resident between
 * poporon_encode / poporon_decode calls of a general-parameter handle and
 * serves them from the handle's coherent host buffer (GZ_* payload, ZC_REQ /
 * ZC_FLAG / ZC_EXITED words), so a call costs no kernel launch.  Lane 0
 * polls the request word; encode stages the request's rows Q[0 .. size) and
 * runs gw_encode_one, decode gw_decode_one in the request's mode (0 errors,
 * 1 u32 erasure slots, 2 external syndromes); then the sequence word to
 * ZC_FLAG with a system-scope release.  It leaves after idle_ticks without a
 * request, after max_ticks in all, at RS_SRV_STOP, or when ZC_YIELD moves
 * off yv (another handle's batch), storing its id to ZC_EXITED (api.cpp
 * srv_call relaunches, or launches per call, for a request it did not see).
 */
__global__ __launch_bounds__(64) void rsgw_serve_k(const RsGenTables *__restrict__ T, RsGenParams P, uint8_t *zc,
                                                    uint32_t last, uint32_t id, uint32_t yv,
                                                    uint64_t idle_ticks, uint64_t max_ticks)
{
    __shared__ GwSmem sm;
    __shared__ uint16_t qs[GW_QS];
    __shared__ uint32_t cmd[4]; /* seq, op (0: leave), size, mode */
    const uint32_t lane = threadIdx.x;
    gw_tables(sm, T, P.nn);
    __syncthreads();
    GwWave &W = sm.w[0];
    const GMod mod{P.nn, P.magic};
    const bool qf = (P.fcr + P.nroots - 1u) * P.prim + P.nn - 1u < 65536u;
    uint64_t *req = reinterpret_cast<uint64_t *>(zc + ZC_REQ); /* ZC_REQ, ZC_YIELD */
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    uint64_t idle0 = t0;
    uint32_t staged = 0; /* message size whose rows Q[0 .. size) are in qs (0: none) */
    for (;;) {
        if (lane == 0) {
            uint32_t r = last, op = 0;
            for (;;) {
                /* the request word and ZC_YIELD in one 8-byte load */
                const uint64_t w = __hip_atomic_load(req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                r = (uint32_t)w;
                if (r != last) {
                    op = ZC_REQ_OP(r);
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
        if ((op != RS_SRV_ENCODE && op != RS_SRV_DECODE) || size == 0u || size + P.nroots > P.nn)
            break; /* uniform: idle, lifetime, RS_SRV_STOP; a malformed request also ends the launch */
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, ""); /* the payload's loads: after the request */
        RsGenParams Q = P;
        Q.size = size;
        Q.pad = (int32_t)(P.nn - P.nroots - size);
        if (op == RS_SRV_ENCODE) {
            if (size != staged) { /* the rows stay staged for the next request of this size */
                gw_stage_rows(qs, T, size, P.nroots);
                __syncthreads();
                staged = size;
            }
            gw_encode_one(sm.al2, sm.log, W.lr, qs, Q, lane, size > P.nroots, zc + GZ_DATA, zc + GZ_PAR);
        } else {
            gw_decode_one<uint32_t, 64>(sm, W, Q, mod, GwGrp<64>(lane), qf, zc + GZ_DATA, zc + GZ_PAR,
                                    mode == 2u ? reinterpret_cast<const uint16_t *>(zc + GZ_EXT) : nullptr,
                                    mode == 1u ? reinterpret_cast<const uint32_t *>(zc + GZ_POS) : nullptr,
                                    mode == 1u ? (uint32_t)zc[GZ_CNT] : 0u, zc + GZ_OK, zc + GZ_COR);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (lane == 0)
            __hip_atomic_store(reinterpret_cast<uint32_t *>(zc + ZC_FLAG), seq, __ATOMIC_RELEASE,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        last = seq;
        idle0 = __builtin_amdgcn_s_memrealtime();
    }
    if (lane == 0)
        __hip_atomic_store(reinterpret_cast<uint32_t *>(zc + ZC_EXITED), id, __ATOMIC_RELEASE,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

/* ------------------------------------------------------------------------ */
/* rsg_lfsr_k: batch encode of codes with more than 32 roots                */
/* ------------------------------------------------------------------------ */

/*
 * src/encode.c:120-143 as a table-driven LFSR, one codeword per lane: the
 * register is W = 16 NP bytes (byte i = byte i % 4 of dword i / 4; the
 * parity in bytes 0 .. nr-1, highest degree first, zeros behind them: the
 * generator g(x) x^(W - nr)), a step shifts it by one byte and XORs row fb
 * (fb = input byte ^ register byte 0; the rows of fb >= 2^m repeat those of
 * fb & nn, the reference's masking).  The rows are tab->lrow, staged in LDS
 * as RP copies (gl_copies), lane l reading copy l % RP ((fb NP + piece) RP + copy
 * 16-byte units: lanes of different copies hit different bank slots).  The
 * per-row table keeps the reference's literal use of the generator's logs,
 * so the result is the reference's for every generator.  Against
 * rsgw_encode_k's table of message-position rows (size x nr products per
 * codeword over the wave): nr / 16 16-byte reads per message byte.
 */
#define GL_WG 256
#define GL_LDS (64u * 1024u) /* dynamic LDS per workgroup */

template <int NP>
constexpr uint32_t gl_copies() /* table copies in GL_LDS */
{
    return std::max<uint32_t>(1u, std::min<uint32_t>(16u, GL_LDS / (4096u * NP)));
}

template <int NP>
__global__ __launch_bounds__(GL_WG) void rsg_lfsr_k(const RsGenTables *__restrict__ T, uint32_t size, uint32_t nr,
                                                    const uint8_t *__restrict__ data, size_t dstride,
                                                    uint8_t *__restrict__ parity, size_t pstride, size_t count)
{
    constexpr uint32_t RP = gl_copies<NP>();
    extern __shared__ uint4 lrows[]; /* [(fb NP + piece) RP + copy] */
    for (uint32_t u = threadIdx.x; u < 256u * NP; u += blockDim.x) {
        const uint32_t fb = u / NP, j = u % NP;
        const uint4 v = *reinterpret_cast<const uint4 *>(T->lrow + fb * 256u + 16u * j);
        for (uint32_t r = 0; r < RP; ++r)
            lrows[u * RP + r] = v;
    }
    __syncthreads();
    const uint4 *tab = lrows + threadIdx.x % RP;
    const uint32_t rs = NP * RP; /* units per row */
    for (size_t cw = (size_t)blockIdx.x * blockDim.x + threadIdx.x; cw < count;
         cw += (size_t)gridDim.x * blockDim.x) {
        uint32_t X[4 * NP];
#pragma unroll
        for (int k = 0; k < 4 * NP; ++k)
            X[k] = 0;
        auto step = [&](uint32_t d) __attribute__((always_inline)) {
            const uint4 *row = tab + ((X[0] ^ d) & 0xffu) * rs;
            uint4 v[NP];
#pragma unroll
            for (int j = 0; j < NP; ++j)
                v[j] = row[j * RP];
#pragma unroll
            for (int k = 0; k < 4 * NP - 1; ++k)
                X[k] = __builtin_amdgcn_alignbyte(X[k + 1], X[k], 1);
            X[4 * NP - 1] >>= 8;
#pragma unroll
            for (int j = 0; j < NP; ++j) {
                X[4 * j] ^= v[j].x;
                X[4 * j + 1] ^= v[j].y;
                X[4 * j + 2] ^= v[j].z;
                X[4 * j + 3] ^= v[j].w;
            }
        };
        /* the message as aligned dwords that hold its bytes (no load past
         * them), re-aligned by the row's byte offset */
        const uint8_t *p = data + cw * dstride;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        const uint32_t *w = reinterpret_cast<const uint32_t *>(a & ~uintptr_t(3));
        const uint32_t sh = (uint32_t)(a & 3u), nd = (sh + size + 3u) >> 2;
        uint32_t cur = size ? w[0] : 0u; /* size 0: zero parity, nothing read */
        uint32_t q = 0, i = 0;
        for (; i + 4u <= size; i += 4u, ++q) {
            const uint32_t nxt = q + 1u < nd ? w[q + 1u] : 0u;
            const uint32_t m = __builtin_amdgcn_alignbyte(nxt, cur, sh);
            step(m);
            step(m >> 8);
            step(m >> 16);
            step(m >> 24);
            cur = nxt;
        }
        if (i < size) {
            const uint32_t nxt = q + 1u < nd ? w[q + 1u] : 0u;
            const uint32_t m = __builtin_amdgcn_alignbyte(nxt, cur, sh);
            for (uint32_t b = 0; b < size - i; ++b)
                step(m >> (8u * b));
        }
        /* the first nr register bytes: whole dwords as unaligned dword
         * stores, the last 0..3 bytes one by one */
        typedef __attribute__((address_space(1))) uint32_t gu32s __attribute__((aligned(1)));
        uint8_t *o = parity + cw * pstride;
        const uint32_t nw = nr >> 2, nt = nr & 3u;
        uint32_t tail = 0;
#pragma unroll
        for (int k = 0; k < 4 * NP; ++k) {
            if ((uint32_t)k < nw)
                *(gu32s *)(uintptr_t)(o + 4 * k) = X[k];
            tail = (uint32_t)k == nw ? X[k] : tail;
        }
        for (uint32_t b = 0; b < nt; ++b)
            o[4u * nw + b] = (uint8_t)(tail >> (8u * b));
    }
}

template <int NP>
static void rsg_lfsr_launch(const RsGenTables *tab, const RsGenParams &P, const uint8_t *data, size_t dstride,
                            uint8_t *parity, size_t pstride, size_t count, int num_cu, hipStream_t stream,
                            uint32_t np)
{
    if constexpr (NP <= 16) {
        if (np != (uint32_t)NP) {
            rsg_lfsr_launch<NP + 1>(tab, P, data, dstride, parity, pstride, count, num_cu, stream, np);
            return;
        }
        const size_t lds = (size_t)4096u * NP * gl_copies<NP>();
        const size_t need = (count + GL_WG - 1) / GL_WG;
        const size_t cap = (size_t)(num_cu > 0 ? num_cu : 256) * 2u;
        const dim3 grid((uint32_t)std::max<size_t>(1, std::min(need, cap)));
        RS_LAUNCH(rsg_lfsr_k<NP>, grid, dim3(GL_WG), lds, stream, tab, P.size, P.nroots, data, dstride, parity,
                  pstride, count);
    }
}

extern "C" hipError_t rsg_lfsr_encode(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data,
                                      size_t dstride, uint8_t *parity, size_t pstride, size_t count, int num_cu,
                                      hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const uint32_t np = (prm->nroots + 15u) / 16u;
    if (np < 1u || np > 16u)
        return hipErrorInvalidValue;
    rsg_lfsr_launch<1>(tab, *prm, data, dstride, parity, pstride, count, num_cu, stream, np);
    return hipGetLastError();
}

/* ------------------------------------------------------------------------ */
/* launchers                                                                */
/* ------------------------------------------------------------------------ */

/* workgroup size and LDS bytes for `slots` per-lane arrays of nroots+1 bytes */
static void g_shape(const RsGenParams &P, uint32_t slots, uint32_t &wg, size_t &lds)
{
    const size_t per_lane = (size_t)slots * (P.nroots + 1u);
    wg = G_WG_MAX;
    while (wg > 64u && 768u + per_lane * wg > 64u * 1024u)
        wg -= 64u;
    lds = 768u + per_lane * wg;
}

static dim3 g_grid(size_t count, uint32_t wg, int num_cu, size_t lds)
{
    const size_t per_cu = std::max<size_t>(1, std::min<size_t>(8, (160u * 1024u) / lds));
    const size_t need = (count + wg - 1) / wg;
    const size_t cap = (size_t)(num_cu > 0 ? num_cu : 256) * per_cu;
    return dim3((uint32_t)std::max<size_t>(1, std::min(need, cap)));
}

extern "C" hipError_t rsg_encode(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                                 uint8_t *parity, size_t pstride, size_t count, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    uint32_t wg;
    size_t lds;
    g_shape(*prm, 1, wg, lds);
    RS_LAUNCH(rsg_encode_k, g_grid(count, wg, num_cu, lds), dim3(wg), lds, stream, tab, *prm, data, dstride,
                       parity, pstride, count);
    return hipGetLastError();
}

extern "C" hipError_t rsg_decode(const RsGenTables *tab, const RsGenParams *prm, uint8_t *data, size_t dstride,
                                 uint8_t *parity, size_t pstride, size_t count, const uint16_t *ext,
                                 size_t ext_stride, const uint8_t *pos8, const uint32_t *pos32, size_t pos_stride,
                                 const uint8_t *cnt, uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    uint32_t wg;
    size_t lds;
    g_shape(*prm, 7, wg, lds);
    const dim3 grid = g_grid(count, wg, num_cu, lds);
    if (pos32)
        RS_LAUNCH(rsg_decode_k<uint32_t>, grid, dim3(wg), lds, stream, tab, *prm, data, dstride, parity,
                           pstride, count, ext, ext_stride, pos32, pos_stride, cnt, ok, corrected, nullptr, nullptr);
    else
        RS_LAUNCH(rsg_decode_k<uint8_t>, grid, dim3(wg), lds, stream, tab, *prm, data, dstride, parity,
                           pstride, count, ext, ext_stride, pos8, pos_stride, cnt, ok, corrected, nullptr, nullptr);
    return hipGetLastError();
}

/* decode of the codewords list[0 .. *list_n) (at most count; the grid is
 * sized for a list of up to 1/16 of the batch and loops past it): errors
 * only, with external log-form syndromes (ext), or with u8 erasure slots
 * (pos8 / pos_stride / cnt) */
extern "C" hipError_t rsg_decode_list(const RsGenTables *tab, const RsGenParams *prm, uint8_t *data, size_t dstride,
                                      uint8_t *parity, size_t pstride, size_t count, const uint32_t *list,
                                      const uint32_t *list_n, const uint16_t *ext, size_t ext_stride,
                                      const uint8_t *pos8, size_t pos_stride, const uint8_t *cnt, uint8_t *ok,
                                      uint8_t *corrected, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    uint32_t wg;
    size_t lds;
    g_shape(*prm, 7, wg, lds);
    RS_LAUNCH(rsg_decode_k<uint8_t>, g_grid((count + 15) / 16, wg, num_cu, lds), dim3(wg), lds, stream, tab, *prm,
              data, dstride, parity, pstride, count, ext, ext_stride, pos8, pos_stride, cnt, ok, corrected, list,
              list_n);
    return hipGetLastError();
}

extern "C" hipError_t rsg_check(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                                const uint8_t *parity, size_t pstride, size_t count, uint8_t *dirty, uint16_t *syn,
                                size_t syn_stride, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    uint32_t wg;
    size_t lds;
    g_shape(*prm, 1, wg, lds);
    RS_LAUNCH(rsg_check_k, g_grid(count, wg, num_cu, lds), dim3(wg), lds, stream, tab, *prm, data, dstride,
                       parity, pstride, count, dirty, syn, syn_stride);
    return hipGetLastError();
}

/* ---- one codeword per wave ---- */
static dim3 gw_grid(size_t waves, int num_cu)
{
    const size_t need = (waves + GW_WG / 64 - 1) / (GW_WG / 64);
    const size_t cap = (size_t)(num_cu > 0 ? num_cu : 256) * 8u;
    return dim3((uint32_t)std::max<size_t>(1, std::min(need, cap)));
}

extern "C" hipError_t rsgw_encode(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                                  uint8_t *parity, size_t pstride, size_t count, uint32_t *flag, uint32_t seq,
                                  int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rsgw_encode_k, gw_grid(count, num_cu), dim3(GW_WG), 0, stream, tab, *prm, data, dstride, parity, pstride,
              count, flag, seq);
    return hipGetLastError();
}

/* lanes per codeword of a decode batch: sixteen codewords per wave for codes
 * of up to 15 symbols, eight up to 31, four up to 63, two up to 127, from
 * GW_GROUP_MIN codewords on (single
 * calls and small batches keep the whole wave: the shortest chain per
 * codeword) */
#ifndef GW_GROUP_MIN
#define GW_GROUP_MIN 256
#endif
template <typename PosT>
static void rsgw_decode_launch(const RsGenTables *tab, const RsGenParams *prm, uint8_t *data, size_t dstride,
                               uint8_t *parity, size_t pstride, size_t count, const uint16_t *ext, size_t ext_stride,
                               const PosT *pos, size_t pos_stride, const uint8_t *cnt, uint8_t *ok, uint8_t *corrected,
                               const uint32_t *list, const uint32_t *list_n, uint32_t *flag, uint32_t seq, int num_cu,
                               hipStream_t stream)
{
    /* a list: the grid for up to 1/16 of the batch, looping past it */
    const size_t units = list ? (count + 15) / 16 : count;
    const uint32_t gl = (list || count < GW_GROUP_MIN) ? 64u
                        : prm->nn <= 15u                  ? 4u
                        : prm->nn <= 31u                  ? 8u
                        : prm->nn <= 63u                  ? 16u
                        : prm->nn <= 127u                 ? 32u
                                                          : 64u;
    const dim3 grid = gw_grid((units * gl + 63u) / 64u, num_cu);
    if (gl == 4u)
        RS_LAUNCH((rsgw_decode_k<PosT, 4>), grid, dim3(GW_WG), 0, stream, tab, *prm, data, dstride, parity, pstride,
                  count, ext, ext_stride, pos, pos_stride, cnt, ok, corrected, list, list_n, flag, seq);
    else if (gl == 8u)
        RS_LAUNCH((rsgw_decode_k<PosT, 8>), grid, dim3(GW_WG), 0, stream, tab, *prm, data, dstride, parity, pstride,
                  count, ext, ext_stride, pos, pos_stride, cnt, ok, corrected, list, list_n, flag, seq);
    else if (gl == 16u)
        RS_LAUNCH((rsgw_decode_k<PosT, 16>), grid, dim3(GW_WG), 0, stream, tab, *prm, data, dstride, parity, pstride,
                  count, ext, ext_stride, pos, pos_stride, cnt, ok, corrected, list, list_n, flag, seq);
    else if (gl == 32u)
        RS_LAUNCH((rsgw_decode_k<PosT, 32>), grid, dim3(GW_WG), 0, stream, tab, *prm, data, dstride, parity, pstride,
                  count, ext, ext_stride, pos, pos_stride, cnt, ok, corrected, list, list_n, flag, seq);
    else
        RS_LAUNCH((rsgw_decode_k<PosT, 64>), grid, dim3(GW_WG), 0, stream, tab, *prm, data, dstride, parity, pstride,
                  count, ext, ext_stride, pos, pos_stride, cnt, ok, corrected, list, list_n, flag, seq);
}

extern "C" hipError_t rsgw_decode(const RsGenTables *tab, const RsGenParams *prm, uint8_t *data, size_t dstride,
                                  uint8_t *parity, size_t pstride, size_t count, const uint16_t *ext, size_t ext_stride,
                                  const uint8_t *pos8, const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt,
                                  uint8_t *ok, uint8_t *corrected, const uint32_t *list, const uint32_t *list_n,
                                  uint32_t *flag, uint32_t seq, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    if (pos32)
        rsgw_decode_launch<uint32_t>(tab, prm, data, dstride, parity, pstride, count, ext, ext_stride, pos32,
                                     pos_stride, cnt, ok, corrected, list, list_n, flag, seq, num_cu, stream);
    else
        rsgw_decode_launch<uint8_t>(tab, prm, data, dstride, parity, pstride, count, ext, ext_stride, pos8, pos_stride,
                                    cnt, ok, corrected, list, list_n, flag, seq, num_cu, stream);
    return hipGetLastError();
}

extern "C" hipError_t rsgw_check(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                                 const uint8_t *parity, size_t pstride, size_t count, uint8_t *dirty, uint16_t *syn,
                                 size_t syn_stride, int num_cu, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    RS_LAUNCH(rsgw_check_k, gw_grid(count, num_cu), dim3(GW_WG), 0, stream, tab, *prm, data, dstride, parity, pstride,
              count, dirty, syn, syn_stride);
    return hipGetLastError();
}

extern "C" hipError_t rsgw_serve(const RsGenTables *tab, const RsGenParams *prm, uint8_t *zc_dev, uint32_t last,
                                 uint32_t id, uint32_t yv, uint64_t idle_ticks, uint64_t max_ticks,
                                 hipStream_t stream)
{
    hipLaunchKernelGGL(rsgw_serve_k, dim3(1), dim3(64), 0, stream, tab, *prm, zc_dev, last, id, yv, idle_ticks,
                       max_ticks);
    return hipGetLastError();
}
