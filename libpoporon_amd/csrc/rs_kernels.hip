/*
 * rs_kernels.hip -- RS(n, n-32) over GF(2^8) on CDNA4 (gfx950).
 *
 * Kernels
 *   rs_lfsr_k<MODE_ENCODE>    parity = m(x) x^32 mod g(x)          (src/encode.c:120-143)
 *   rs_lfsr_k<MODE_SYNDROME>  the 32 syndromes of the received word (src/decode.c:375-415):
 *                             the received word c = d x^32 + p is the codeword of
 *                             its data plus E' = p + (d x^32 mod g), so
 *                             S_i = c(beta_i) = E'(beta_i): 223 LFSR steps (the
 *                             encode's) instead of 255, then E' -> S by tables
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
 * tables that turn E' into syndromes with 128 ds_read_b128 per codeword:
 * 160 KB, the whole LDS.
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

#include <type_traits>

#include "rs_device.h"
#include "rs_lane.h"

/* global-memory views (global_load, not flat_load) */
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) const u32x4 gu32x4;
typedef __attribute__((address_space(1))) const uint32_t gu32;

#define LFSR_WG 1024
#ifndef LFSR_PREFETCH
#define LFSR_PREFETCH 0 /* rolling prefetch of the next codeword's chunks: measured slower (0.127 vs 0.118 ms encode) */
#endif
#ifndef LFSR_STAGGER
#define LFSR_STAGGER 0 /* (experiment) odd waves sleep LFSR_STAGGER x 8128 cycles first */
#endif
#define LFSR_REPL 16
#ifndef LFSR_BLOCKS
#define LFSR_BLOCKS 1 /* PATH_BLOCKS for sizes 16..256 other than the full RS(255,223) (0: the dword path) */
#endif
#ifndef LFSR_BLOCKS_ALL
#define LFSR_BLOCKS_ALL 0 /* (experiment) PATH_BLOCKS for the full RS(255,223) too */
#endif
#ifndef LFSR_USTORE
#define LFSR_USTORE 1
#endif

/* ------------------------------------------------------------------------ */
/* LFSR (encode / syndromes / check)                                        */
/* ------------------------------------------------------------------------ */

/*
 * Interleaved shift register.  The 32 register bytes p_0..p_31 (p_0 = the
 * highest-degree remainder coefficient, the next feedback) are kept as 8
 * dwords, logical dword k = bytes (p_k, p_k+8, p_k+16, p_k+24), and logical
 * dword k lives in X[(k + r) & 7] after r steps.  One step
 *     fb = p_0 ^ d;  p'_j = p_j+1 ^ row[fb]_j;  p'_31 = row[fb]_31
 * is then a renaming of the dwords (logical k+1 becomes k) plus one 8-bit
 * shift of the dword that wraps around (logical 0 -> 7), and the row table
 * (T->lfsr) stores rows in the same interleaved order.  Two steps' row XORs
 * fuse into one v_bitop3_b32 (3-way XOR) per dword; only the dword that feeds the next
 * step is brought up to date eagerly.  With the rotation r a compile-time
 * constant (fully unrolled loops) a step costs ~8 VALU + 2 ds_read_b128,
 * against ~20 VALU for a funnel-shifted register.
 */
__device__ __forceinline__ void il_rows(uint32_t (&R)[8], uint32_t fb, const uint4 *__restrict__ tab)
{
    const uint4 a = tab[fb * (2 * LFSR_REPL)];
    const uint4 b = tab[fb * (2 * LFSR_REPL) + LFSR_REPL];
    R[0] = a.x, R[1] = a.y, R[2] = a.z, R[3] = a.w;
    R[4] = b.x, R[5] = b.y, R[6] = b.z, R[7] = b.w;
}

/* one step at rotation r; d holds the input byte in bits 0..7 (upper bits ignored) */
__device__ __forceinline__ void il_step(uint32_t (&X)[8], int r, uint32_t d, const uint4 *__restrict__ tab)
{
    uint32_t R[8];
    il_rows(R, __builtin_amdgcn_bitop3_b32(X[r & 7], d, 0xffu, 0x28), tab); /* (x ^ d) & 0xff, full rate */
    X[r & 7] = (X[r & 7] >> 8) ^ R[7];
#pragma unroll
    for (int k = 0; k < 7; ++k)
        X[(r + 1 + k) & 7] ^= R[k];
}

/* two steps at rotation r, r+1 */
__device__ __forceinline__ void il_pair(uint32_t (&X)[8], int r, uint32_t d0, uint32_t d1,
                                        const uint4 *__restrict__ tab)
{
    uint32_t Ra[8], Rb[8];
    const int i0 = r & 7, i1 = (r + 1) & 7;
    il_rows(Ra, __builtin_amdgcn_bitop3_b32(X[i0], d0, 0xffu, 0x28), tab); /* (x ^ d) & 0xff */
    X[i1] ^= Ra[0]; /* next logical 0: needed now */
    const uint32_t w = X[i0] >> 8;
    il_rows(Rb, __builtin_amdgcn_bitop3_b32(X[i1], d1, 0xffu, 0x28), tab);
#pragma unroll
    for (int j = 1; j < 7; ++j)
        X[(r + 1 + j) & 7] = xor3(X[(r + 1 + j) & 7], Ra[j], Rb[j - 1]);
    X[i0] = xor3(w, Ra[7], Rb[6]);
    X[i1] = (X[i1] >> 8) ^ Rb[7];
}

/* X[(k + r) & 7] -> X[k], r uniform at run time */
__device__ __forceinline__ void il_normalize(uint32_t (&X)[8], uint32_t r)
{
#pragma unroll
    for (int s = 1; s < 8; s <<= 1) {
        const bool c = (r & (uint32_t)s) != 0u;
        uint32_t T[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            T[k] = c ? X[(k + s) & 7] : X[k];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            X[k] = T[k];
    }
}

/* register byte m (0 = highest degree) at rotation r */
__device__ __forceinline__ uint32_t il_byte(const uint32_t (&X)[8], int r, int m)
{
    return (X[(m + r) & 7] >> (8 * (m >> 3))) & 0xffu;
}

/* the 32 register bytes in order, as 8 dwords (byte m of the register = byte m & 3 of dword m >> 2) */
__device__ __forceinline__ void il_bytes(uint32_t (&P)[8], const uint32_t (&X)[8], int r)
{
#pragma unroll
    for (int q = 0; q < 8; ++q)
        P[q] = il_byte(X, r, 4 * q) | (il_byte(X, r, 4 * q + 1) << 8) | (il_byte(X, r, 4 * q + 2) << 16) |
               (il_byte(X, r, 4 * q + 3) << 24);
}

/* Feed n bytes starting at p (any alignment), rotation 0 on entry and on
 * exit.  Only aligned dwords that contain at least one message byte are
 * loaded, so no load can cross into an unmapped page. */
__device__ __forceinline__ void lfsr_feed(uint32_t (&X)[8], const uint8_t *p, uint32_t n, const uint4 *__restrict__ tab)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    gu32 *w = reinterpret_cast<gu32 *>(a & ~uintptr_t(3));
    const uint32_t sh = static_cast<uint32_t>(a & 3u);
    const uint32_t nd = (sh + n + 3u) >> 2; /* dwords holding message bytes */
    if (n == 0)
        return;
    uint32_t cur = w[0];
    uint32_t q = 0;
    uint32_t i = 0;
    for (; i + 16u <= n; i += 16u, q += 4u) { /* 16 steps: the rotation comes back to 0 */
        const uint32_t w1 = (q + 1u < nd) ? w[q + 1u] : 0u;
        const uint32_t w2 = (q + 2u < nd) ? w[q + 2u] : 0u;
        const uint32_t w3 = (q + 3u < nd) ? w[q + 3u] : 0u;
        const uint32_t w4 = (q + 4u < nd) ? w[q + 4u] : 0u;
        const uint32_t m[4] = {__builtin_amdgcn_alignbyte(w1, cur, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                               __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
#pragma unroll
        for (int b = 0; b < 16; b += 2)
            il_pair(X, b, m[b >> 2] >> (8 * (b & 3)), m[(b + 1) >> 2] >> (8 * ((b + 1) & 3)), tab);
        cur = w4;
    }
    if (i < n) {
        const uint32_t w1 = (q + 1u < nd) ? w[q + 1u] : 0u;
        const uint32_t w2 = (q + 2u < nd) ? w[q + 2u] : 0u;
        const uint32_t w3 = (q + 3u < nd) ? w[q + 3u] : 0u;
        const uint32_t w4 = (q + 4u < nd) ? w[q + 4u] : 0u;
        const uint32_t m[4] = {__builtin_amdgcn_alignbyte(w1, cur, sh), __builtin_amdgcn_alignbyte(w2, w1, sh),
                               __builtin_amdgcn_alignbyte(w3, w2, sh), __builtin_amdgcn_alignbyte(w4, w3, sh)};
        const uint32_t left = n - i; /* uniform */
#pragma unroll
        for (int b = 0; b < 16; b += 2) {
            if ((uint32_t)b + 1u < left)
                il_pair(X, b, m[b >> 2] >> (8 * (b & 3)), m[(b + 1) >> 2] >> (8 * ((b + 1) & 3)), tab);
            else if ((uint32_t)b < left)
                il_step(X, b, m[b >> 2] >> (8 * (b & 3)), tab);
        }
        il_normalize(X, left & 7u);
    }
}

/* The 32 bytes at p (any alignment) as 8 dwords in order: only aligned
 * dwords that hold one of them are loaded (no read past the bytes' page). */
__device__ __forceinline__ void load32_any(uint32_t (&Q)[8], const uint8_t *p)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    gu32 *w = reinterpret_cast<gu32 *>(a & ~uintptr_t(3));
    const uint32_t sh = static_cast<uint32_t>(a & 3u);
    uint32_t W[9];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        W[k] = w[k];
    W[8] = sh ? w[8] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        Q[k] = __builtin_amdgcn_alignbyte(W[k + 1], W[k], sh);
}

/* The first n < 32 bytes at p (any alignment) as 8 dwords in order, zeros
 * behind them: only aligned dwords that hold one of the n bytes are loaded
 * (the parity of a code with n < 32 roots; the row may end right after it) */
__device__ __forceinline__ void load_n_any(uint32_t (&Q)[8], const uint8_t *p, uint32_t n)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    gu32 *w = reinterpret_cast<gu32 *>(a & ~uintptr_t(3));
    const uint32_t sh = static_cast<uint32_t>(a & 3u);
    const uint32_t nd = (sh + n + 3u) >> 2; /* dwords holding the n bytes */
    uint32_t W[9];
#pragma unroll
    for (int k = 0; k < 9; ++k)
        W[k] = (uint32_t)k < nd ? w[k] : 0u;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t v = __builtin_amdgcn_alignbyte(W[k + 1], W[k], sh);
        const uint32_t have = n > 4u * k ? n - 4u * k : 0u; /* bytes of dword k inside the n */
        Q[k] = have >= 4u ? v : v & ((1u << (8u * have)) - 1u);
    }
}

/* Where the next codeword's bytes of one stream are: its 16-byte aligned
 * chunks and the offset of the first byte in the first chunk.  With no next
 * codeword for this lane (valid = false) the chunks are read from `fallback`
 * (a mapped row) and never used: every load is unconditional, so the loop
 * stays straight-line and the compiler's wait counts stay exact.  The
 * pointer is explicitly global: a flat load would also count against
 * lgkmcnt, and every LDS wait of the LFSR steps would then wait for HBM. */

struct NextSrc {
    gu32x4 *c16;
    uint32_t sh;
    __device__ __forceinline__ NextSrc(const uint8_t *p, bool valid, const uint8_t *fallback)
    {
        const uintptr_t a = reinterpret_cast<uintptr_t>(valid ? p : fallback);
        c16 = reinterpret_cast<gu32x4 *>(a & ~uintptr_t(15));
        sh = static_cast<uint32_t>(a & 15u);
    }
};

/* Fixed-length stream of N message bytes at any alignment, in registers: the
 * 16-byte aligned chunks that hold message bytes (dwordx4 loads), re-aligned
 * on use: dword k = bytes [4k, 4k+4) = funnel of stream dwords q = k + sh/4
 * and q+1 by sh%4 bytes, with the per-lane q offset resolved by a 2-level
 * select (no dynamic register indexing).
 *
 * Rolling prefetch: lfsr_stream() reloads the chunks with the NEXT
 * codeword's chunks as soon as the message dwords that read them have been
 * consumed, so the next codeword's loads are in flight during this
 * codeword's LFSR steps (no extra registers; without it every lane's loads
 * and LFSR steps alternate and HBM idles during the compute). */
template <int N>
struct Stream {
    static constexpr int NCH = (N + 30) / 16; /* chunks covering up to 15 + N bytes */
    uint32_t D[NCH * 4 + 4];
    uint32_t sdw, sb;
    __device__ __forceinline__ void chunk(int c, const NextSrc &n)
    {
        /* a chunk past the message may lie on an unmapped page: read chunk 0
         * instead (its bytes are never fed) */
        const u32x4 v = n.c16[(uint32_t)(16 * c) < n.sh + (uint32_t)N ? c : 0];
        D[4 * c] = v.x;
        D[4 * c + 1] = v.y;
        D[4 * c + 2] = v.z;
        D[4 * c + 3] = v.w;
    }
    /* second refill batch of lfsr_stream: chunks [NCH/2, NCH), then switch */
    __device__ __forceinline__ void refill_tail(const NextSrc &n)
    {
#pragma unroll
        for (int c = NCH / 2; c < NCH; ++c)
            chunk(c, n);
        retarget(n);
    }
    __device__ __forceinline__ void retarget(const NextSrc &n)
    {
        sdw = n.sh >> 2;
        sb = n.sh & 3u;
    }
    __device__ __forceinline__ void load(const NextSrc &n)
    {
#pragma unroll
        for (int c = 0; c < NCH; ++c)
            chunk(c, n);
#pragma unroll
        for (int t = 0; t < 4; ++t)
            D[NCH * 4 + t] = 0;
        retarget(n);
    }
    __device__ __forceinline__ uint32_t at(int q) const /* stream dword q + sdw */
    {
        const uint32_t t0 = (sdw & 1u) ? D[q + 1] : D[q];
        const uint32_t t1 = (sdw & 1u) ? D[q + 3] : D[q + 2];
        return (sdw & 2u) ? t1 : t0;
    }
    __device__ __forceinline__ uint32_t word(int k) const /* message dword k */
    {
        return __builtin_amdgcn_alignbyte(at(k + 1), at(k), sb);
    }
};

/* Byte i of a fixed-length stream (any upper bits; compile-time i after unrolling) */
template <int N>
__device__ __forceinline__ uint32_t stream_byte(const Stream<N> &s, int i)
{
    return s.word(i >> 2) >> (8 * (i & 3));
}

/* The bytes [I0, I1) of s, starting at rotation R0 + I0; s is refilled with
 * the stream `next` in two batches of consecutive chunks (each batch's loads
 * of a row hit the same few cache lines back to back): chunks [0, NCH/2)
 * here, as soon as the last of them is dead (chunk c is dead once message
 * dword 4c+3, i.e. byte 16c+15, has been fed), the rest by the caller
 * (Stream::refill_tail) once the stream is consumed. */
/* compile-time loop: f(std::integral_constant<int, i>) for i = I, I+S, ... < E
 * (fully unrolled by construction, so register arrays indexed by i stay in
 * registers however large the body) */
template <int I, int E, int S, class F>
__device__ __forceinline__ void static_for(F &&f)
{
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        static_for<I + S, E, S>(f);
    }
}

template <int N, int R0, int I0 = 0, int I1 = N, bool REFILL = true, class S = Stream<N>>
__device__ __forceinline__ void lfsr_stream(uint32_t (&X)[8], S &s, const NextSrc &next,
                                            const uint4 *__restrict__ tab)
{
    static_assert(I0 % 2 == 0 && (I1 % 2 == 0 || I1 == N), "byte ranges split at pairs");
    constexpr int NA = Stream<N>::NCH / 2;
    constexpr int IA = 16 * (NA - 1) + 14; /* pair after which chunks [0, NA) are dead */
    static_for<I0, I1 - 1, 2>([&](auto ic) __attribute__((always_inline)) {
        constexpr int i = decltype(ic)::value;
        il_pair(X, R0 + i, stream_byte(s, i), stream_byte(s, i + 1), tab);
        if constexpr (REFILL && i == IA) {
#pragma unroll
            for (int c = 0; c < NA; ++c)
                s.chunk(c, next);
        }
        (void)next;
    });
    if constexpr (I1 == N) {
        if constexpr (N & 1)
            il_step(X, R0 + N - 1, stream_byte(s, N - 1), tab);
        /* the caller refills the rest (s.refill_tail) after its stores, so
         * that the next iteration's first wait covers only the first batch */
    }
}

/* Store the 32-byte register at any alignment without touching neighbours:
 * up to 3 leading bytes, aligned dwords, up to 3 trailing bytes. */
__device__ __forceinline__ void store32_any(uint8_t *o, const uint32_t (&P)[8])
{
    const uint32_t lead = (uint32_t)((4u - (reinterpret_cast<uintptr_t>(o) & 3u)) & 3u);
    const uint32_t X[9] = {P[0], P[1], P[2], P[3], P[4], P[5], P[6], P[7], 0u};
    if (lead == 0u) {
        uint32_t *o4 = reinterpret_cast<uint32_t *>(o);
#pragma unroll
        for (int k = 0; k < 8; ++k)
            o4[k] = P[k];
        return;
    }
    /* bytes 0 .. lead-1 */
    o[0] = (uint8_t)P[0];
    if (lead > 1u)
        o[1] = (uint8_t)(P[0] >> 8);
    if (lead > 2u)
        o[2] = (uint8_t)(P[0] >> 16);
    /* 7 aligned dwords: bytes lead + 4j .. lead + 4j + 3 */
    uint32_t *o4 = reinterpret_cast<uint32_t *>(o + lead);
#pragma unroll
    for (int j = 0; j < 7; ++j)
        o4[j] = __builtin_amdgcn_alignbyte(X[j + 1], X[j], lead);
    /* bytes lead + 28 .. 31 */
    const uint32_t t = __builtin_amdgcn_alignbyte(X[8], X[7], lead);
    uint8_t *ot = o + lead + 28;
    ot[0] = (uint8_t)t;
    if (lead < 3u)
        ot[1] = (uint8_t)(t >> 8);
    if (lead < 2u)
        ot[2] = (uint8_t)(t >> 16);
}


#define MODE_ENCODE 0
#define MODE_SYNDROME 1
#define MODE_CHECK 2
#define FULL_K 223 /* message length of the full-length RS(255,223) code: fixed-stream path */

#define PATH_GENERIC 0 /* any size, any alignment: dword loads per 16 bytes */
#define PATH_SPLIT 1   /* size 223: data stream (rolling prefetch) + separate parity stream */
#define PATH_CONTIG 2  /* size 223, parity right after the data: one 255-byte stream (rolling prefetch) */
#define PATH_BLOCKS 3  /* 16 <= size <= 256 (shortened codes, fewer roots): 16-byte blocks behind leading zeros, one kernel per block count */

/* what the kernel does with the final register (encode: the parity bytes P, in order; syndrome / check: E') */
template <int MODE>
__device__ __forceinline__ void lfsr_epilogue(const uint32_t (&P)[8], const uint4 *__restrict__ synt, size_t cw,
                                              uint8_t *__restrict__ parity, size_t pstride,
                                              uint8_t *__restrict__ out, uint32_t npar = RS_NR)
{
    if (MODE == MODE_ENCODE && npar < RS_NR) {
        /* a generator of degree npar < 32 run as g(x) x^(32 - npar): its
         * parity is the register's first npar bytes (rsk_encode_nr): whole
         * dwords as unaligned dword stores (the first four as one 16-byte
         * store), the last 0..3 bytes one by one */
        typedef unsigned u32x4s __attribute__((ext_vector_type(4), aligned(1)));
        typedef __attribute__((address_space(1))) u32x4s gu32x4s;
        typedef __attribute__((address_space(1))) uint32_t gu32s __attribute__((aligned(1)));
        uint8_t *o = parity + cw * pstride;
        const uint32_t nd = npar >> 2, nt = npar & 3u;
        uint32_t tail = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (k == 0 && nd >= 4u) /* uniform */
                *(gu32x4s *)(uintptr_t)o = u32x4s{P[0], P[1], P[2], P[3]};
            else if ((uint32_t)k < nd && !(k < 4 && nd >= 4u))
                *(gu32s *)(uintptr_t)(o + 4 * k) = P[k];
            tail = (uint32_t)k == nd ? P[k] : tail;
        }
        for (uint32_t b = 0; b < nt; ++b)
            o[4u * nd + b] = (uint8_t)(tail >> (8u * b));
        return;
    }
    if (MODE == MODE_SYNDROME) {
        /* S = sum over the bytes m of E' of T_m,lo[e_m & 15] ^ T_m,hi[e_m >> 4] */
        uint32_t S[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if ((P[0] | P[1] | P[2] | P[3] | P[4] | P[5] | P[6] | P[7]) != 0u) {
#pragma unroll
            for (uint32_t m = 0; m < RS_NR; ++m) {
                const uint32_t rm = (P[m >> 2] >> (8u * (m & 3u))) & 0xffu;
                const uint4 *t0 = synt + (m * 4u) * 16u;
                const uint4 l0 = t0[rm & 15u], l1 = t0[16u + (rm & 15u)];
                const uint4 h0 = t0[32u + (rm >> 4)], h1 = t0[48u + (rm >> 4)];
                S[0] = xor3(S[0], l0.x, h0.x);
                S[1] = xor3(S[1], l0.y, h0.y);
                S[2] = xor3(S[2], l0.z, h0.z);
                S[3] = xor3(S[3], l0.w, h0.w);
                S[4] = xor3(S[4], l1.x, h1.x);
                S[5] = xor3(S[5], l1.y, h1.y);
                S[6] = xor3(S[6], l1.z, h1.z);
                S[7] = xor3(S[7], l1.w, h1.w);
            }
        }
        uint4 *o = reinterpret_cast<uint4 *>(out + cw * RS_NR);
        o[0] = make_uint4(S[0], S[1], S[2], S[3]);
        o[1] = make_uint4(S[4], S[5], S[6], S[7]);
    } else if (MODE == MODE_CHECK) {
        out[cw] = (P[0] | P[1] | P[2] | P[3] | P[4] | P[5] | P[6] | P[7]) != 0u;
    } else {
#if LFSR_USTORE /* two unaligned 16-byte stores (gfx950 supports them, tools/probes/unaligned.hip) */
        typedef unsigned u32x4s __attribute__((ext_vector_type(4), aligned(1)));
        typedef __attribute__((address_space(1))) u32x4s gu32x4s;
        gu32x4s *o = (gu32x4s *)(uintptr_t)(parity + cw * pstride);
        const u32x4s a = {P[0], P[1], P[2], P[3]}, b = {P[4], P[5], P[6], P[7]};
        o[0] = a;
        o[1] = b;
#else
        store32_any(parity + cw * pstride, P);
#endif
    }
}

template <int MODE, int PATH, int NB = 0>
__global__ __launch_bounds__(LFSR_WG) void rs_lfsr_k(const RsDevTables *__restrict__ T,
                                                      const uint8_t *__restrict__ data, size_t dstride,
                                                      uint8_t *__restrict__ parity, size_t pstride, uint32_t size,
                                                      size_t count, uint8_t *__restrict__ out,
                                                      uint32_t *__restrict__ reset, uint32_t npar)
{
    if (reset && blockIdx.x == 0 && threadIdx.x == 0) {
        reset[0] = 0u; /* the split decode's list length, before any later launch on the stream */
        reset[1] = 0u; /* and the erasure decode's count of codewords left to the errata kernels */
    }
    __shared__ uint4 lds[512 * LFSR_REPL + (MODE == MODE_SYNDROME ? 32 * 2 * 2 * 16 : 0)];
    for (uint32_t t = threadIdx.x; t < 512u * LFSR_REPL; t += LFSR_WG)
        lds[t] = T->lfsr[t / LFSR_REPL];
    if (MODE == MODE_SYNDROME)
        for (uint32_t t = threadIdx.x; t < 32u * 2 * 2 * 16; t += LFSR_WG)
            lds[512 * LFSR_REPL + t] = T->synt[t];
    __syncthreads();
    const uint4 *tab = lds + (threadIdx.x & (LFSR_REPL - 1));
    const uint4 *synt = lds + 512 * LFSR_REPL;

    const size_t step = (size_t)gridDim.x * LFSR_WG;
    const size_t cw0 = (size_t)blockIdx.x * LFSR_WG + threadIdx.x;
    constexpr bool PF = LFSR_PREFETCH != 0;
    if (LFSR_STAGGER && ((threadIdx.x >> 6) & 1u)) /* experiment: desynchronise odd waves' load bursts */
        for (int k = 0; k < LFSR_STAGGER; ++k)
            __builtin_amdgcn_s_sleep(127);
    if (PATH == PATH_GENERIC) {
        uint32_t it = 0;
        for (size_t cw = cw0; cw < count; cw += step, ++it) {
            prio_by_progress(it);
            uint32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint32_t P[8];
            lfsr_feed(X, data + cw * dstride, size, tab);
            il_bytes(P, X, 0);
            if (MODE != MODE_ENCODE) { /* E' = received parity + parity of the received data */
                uint32_t Q[8];
                if (npar < RS_NR) /* g(x) x^(32 - npar): E' in the first npar bytes, zeros behind */
                    load_n_any(Q, parity + cw * pstride, npar);
                else
                    load32_any(Q, parity + cw * pstride);
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    P[q] ^= Q[q];
            }
            lfsr_epilogue<MODE>(P, synt, cw, parity, pstride, out, npar);
        }
    } else if constexpr (PATH == PATH_BLOCKS) {
        /* The message as NB = ceil(size / 16) whole 16-byte blocks behind
         * z = 16 NB - size leading zeros (a zero fed into a zero register
         * leaves it zero: the remainder is unchanged), one kernel per NB (no
         * guards, compile-time rotations).  The virtual stream starts at
         * p = msg - z; chunk c is the aligned 16 bytes at align16(p) + 16 c,
         * loaded only where it overlaps the message (and, for the syndromes
         * of rows with the parity right behind the data, the parity), else
         * msg's own chunk (in bounds, never fed); virtual dword j is the
         * funnel of chunk dwords j + sdw, j + sdw + 1 by sb bytes (per lane:
         * p's offset in its chunk); block 0's first z bytes (the previous
         * row's, or a stand-in chunk's) are masked to zero.  The received
         * parity is then virtual dwords 4 NB .. 4 NB + 7, or (elsewhere) loaded
         * three blocks before the end. */
        static_assert(NB >= 1 && NB <= 16, "PATH_BLOCKS: one kernel per block count");
        constexpr int NC = MODE == MODE_ENCODE ? NB + 1 : NB + 3; /* chunks covering 15 + 16 NB (+ 32) bytes */
        const uint32_t z = 16u * NB - size;
        const bool pin = MODE != MODE_ENCODE && parity == data + size && pstride == dstride; /* uniform */
        const uint32_t ext = size + (pin ? npar : 0u);
        uint32_t zmask[4], pmask[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t lo = z > 4u * k ? min(z - 4u * k, 4u) : 0u; /* leading zero bytes of dword k */
            zmask[k] = lo >= 4u ? 0u : ~0u << (8u * lo);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const uint32_t hi = npar > 4u * k ? min(npar - 4u * k, 4u) : 0u; /* parity bytes of dword k */
            pmask[k] = hi >= 4u ? ~0u : (1u << (8u * hi)) - 1u;
        }
        uint32_t it = 0;
        for (size_t cw = cw0; cw < count; cw += step, ++it) {
            prio_by_progress(it);
            const uintptr_t m = reinterpret_cast<uintptr_t>(data + cw * dstride);
            const uintptr_t pv = m - z, c0 = pv & ~uintptr_t(15), mc = m & ~uintptr_t(15);
            const uint32_t sdw = (uint32_t)(pv & 15u) >> 2, sb = (uint32_t)pv & 3u;
            uint32_t D[4 * NC]; /* at(q) reads D[q .. q + 3]: q <= 4 NB (+ 8) */
            /* chunks cf .. cl overlap the row (cf = the chunk holding msg, 0 or 1) */
            gu32x4 *cb = reinterpret_cast<gu32x4 *>(c0);
            const uint32_t cf = (uint32_t)((mc - c0) >> 4), cl = (uint32_t)((((m + ext - 1u) & ~uintptr_t(15)) - c0) >> 4);
            gu32x4 *ca[NC];
            static_for<0, NC, 1>([&](auto cc) __attribute__((always_inline)) {
                constexpr int c = decltype(cc)::value;
                ca[c] = cb + (((uint32_t)c >= cf && (uint32_t)c <= cl) ? (uint32_t)c : cf);
            });
            __builtin_amdgcn_sched_barrier(0);
            auto chunk = [&](auto cc) __attribute__((always_inline)) {
                constexpr int c = decltype(cc)::value;
                const u32x4 v = *ca[c];
                D[4 * c] = v.x, D[4 * c + 1] = v.y, D[4 * c + 2] = v.z, D[4 * c + 3] = v.w;
            };
            /* the message's chunks back to back (a row's chunks share its few
             * cache lines: spread out, the lines leave the L1 between them),
             * the parity's two later */
            static_for<0, NB + 1, 1>(chunk);
            __builtin_amdgcn_sched_barrier(0);
            auto at = [&](int q) __attribute__((always_inline)) { /* chunk dword q + sdw */
                const uint32_t t0 = (sdw & 1u) ? D[q + 1] : D[q];
                const uint32_t t1 = (sdw & 1u) ? D[q + 3] : D[q + 2];
                return (sdw & 2u) ? t1 : t0;
            };
            uint32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint32_t P[8], Q[8];
            static_for<0, NB, 1>([&](auto bc) __attribute__((always_inline)) {
                constexpr int b = decltype(bc)::value;
                if constexpr (MODE != MODE_ENCODE && b == (NB > 3 ? NB - 3 : 0)) {
                    static_for<NB + 1, NC, 1>(chunk);
                    if (!pin) { /* uniform */
                        if (npar < RS_NR)
                            load_n_any(Q, parity + cw * pstride, npar);
                        else
                            load32_any(Q, parity + cw * pstride);
                    }
                }
                uint32_t W[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    W[j] = __builtin_amdgcn_alignbyte(at(4 * b + j + 1), at(4 * b + j), sb);
                    if (b == 0)
                        W[j] &= zmask[j];
                }
#pragma unroll
                for (int i = 0; i < 16; i += 2)
                    il_pair(X, i, W[i >> 2] >> (8 * (i & 3)), W[(i + 1) >> 2] >> (8 * ((i + 1) & 3)), tab);
            });
            il_bytes(P, X, 0);
            if constexpr (MODE != MODE_ENCODE) { /* E' = received parity + parity of the received data */
                if (pin) {
#pragma unroll
                    for (int k = 0; k < 8; ++k)
                        Q[k] = __builtin_amdgcn_alignbyte(at(4 * NB + k + 1), at(4 * NB + k), sb) & pmask[k];
                }
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    P[q] ^= Q[q];
            }
            lfsr_epilogue<MODE>(P, synt, cw, parity, pstride, out, npar);
        }
    } else if (PATH == PATH_CONTIG && MODE != MODE_ENCODE) {
        /* data || parity as one 255-byte stream */
        Stream<FULL_K + RS_NR> sc;
        if constexpr (PF) {
            sc.load(NextSrc(data + cw0 * dstride, cw0 < count, data));
            __builtin_amdgcn_s_waitcnt(0); /* nothing pending at the loop head but the loop's own refills */
        }
        uint32_t it = 0;
        for (size_t cw = cw0; cw < count; cw += step, ++it) {
            prio_by_progress(it);
            const size_t cn = cw + step;
            uint32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint32_t P[8];
            const NextSrc nx(data + cn * dstride, cn < count, data + cw * dstride);
            if constexpr (!PF)
                sc.load(NextSrc(data + cw * dstride, true, nullptr));
            /* the 223 data bytes (two loops, each fully unrolled), then E' =
             * that parity + the received one (stream bytes 223..254) */
            lfsr_stream<FULL_K + RS_NR, 0, 0, 128, PF>(X, sc, nx, tab);
            lfsr_stream<FULL_K + RS_NR, 0, 128, FULL_K - 1, PF>(X, sc, nx, tab);
            il_step(X, FULL_K - 1, stream_byte(sc, FULL_K - 1), tab);
            il_bytes(P, X, FULL_K & 7);
            static_assert(FULL_K % 4 == 3, "parity dword q = bytes 223 + 4q .. 226 + 4q");
            static_for<0, 8, 1>([&](auto qc) __attribute__((always_inline)) { /* compile-time indices: D stays in registers */
                constexpr int q = decltype(qc)::value;
                P[q] ^= __builtin_amdgcn_alignbyte(sc.word(56 + q), sc.word(55 + q), 3);
            });
            lfsr_epilogue<MODE>(P, synt, cw, parity, pstride, out);
            if constexpr (PF)
                sc.refill_tail(nx);
        }
    } else {
        Stream<FULL_K> sd;
        if constexpr (PF) {
            sd.load(NextSrc(data + cw0 * dstride, cw0 < count, data));
            __builtin_amdgcn_s_waitcnt(0); /* nothing pending at the loop head but the loop's own refills */
        }
        uint32_t it = 0;
        for (size_t cw = cw0; cw < count; cw += step, ++it) {
            prio_by_progress(it);
            const size_t cn = cw + step;
            const NextSrc dn(data + cn * dstride, cn < count, data + cw * dstride);
            uint32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            uint32_t P[8];
            if constexpr (!PF)
                sd.load(NextSrc(data + cw * dstride, true, nullptr));
            if (MODE != MODE_ENCODE) {
                /* the 32 parity bytes: loaded two thirds into the data (in
                 * flight for ~70 steps, live only from there on) */
                lfsr_stream<FULL_K, 0, 0, 150, PF>(X, sd, dn, tab);
                Stream<RS_NR> sp;
                sp.load(NextSrc(parity + cw * pstride, true, nullptr));
                lfsr_stream<FULL_K, 0, 150, FULL_K, PF>(X, sd, dn, tab);
                il_bytes(P, X, FULL_K & 7);
                static_for<0, 8, 1>([&](auto qc) __attribute__((always_inline)) { /* E' = that parity + the received one */
                    constexpr int q = decltype(qc)::value;
                    P[q] ^= sp.word(q);
                });
            } else {
                lfsr_stream<FULL_K, 0, 0, FULL_K, PF>(X, sd, dn, tab);
                il_bytes(P, X, FULL_K & 7);
            }
            lfsr_epilogue<MODE>(P, synt, cw, parity, pstride, out);
            if constexpr (PF)
                sd.refill_tail(dn);
        }
    }
}


static int persistent_grid(size_t count, int wg, int num_cu) /* one round: 2 and 4 measured slower (remainder) */
{
    size_t need = (count + wg - 1) / wg;
    size_t g = (size_t)(num_cu > 0 ? num_cu : 256);
    return (int)(need < g ? (need ? need : 1) : g);
}

/* rs_lfsr_k<MODE, PATH_BLOCKS, NB> for NB = nb */
template <int MODE, int NB>
static void launch_blocks(uint32_t nb, dim3 grid, dim3 block, hipStream_t stream, const RsDevTables *tab,
                          const uint8_t *data, size_t dstride, uint8_t *par, size_t pstride, uint32_t size,
                          size_t count, uint8_t *out, uint32_t *reset, uint32_t npar)
{
    if constexpr (NB <= 16) {
        if (nb == (uint32_t)NB)
            RS_LAUNCH((rs_lfsr_k<MODE, PATH_BLOCKS, NB>), grid, block, 0, stream, tab, data, dstride, par, pstride,
                      size, count, out, reset, npar);
        else
            launch_blocks<MODE, NB + 1>(nb, grid, block, stream, tab, data, dstride, par, pstride, size, count, out,
                                        reset, npar);
    }
}

template <int MODE>
static hipError_t launch_lfsr(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                              size_t pstride, uint32_t size, size_t count, uint8_t *out, int num_cu,
                              hipStream_t stream, uint32_t *reset = nullptr, uint32_t npar = RS_NR)
{
    if (count == 0)
        return hipSuccess;
    const dim3 grid(persistent_grid(count, LFSR_WG, num_cu)), block(LFSR_WG);
    uint8_t *par = const_cast<uint8_t *>(parity);
    if ((size != FULL_K || npar != RS_NR || LFSR_BLOCKS_ALL) && size >= 16u && size <= 256u && LFSR_BLOCKS)
        launch_blocks<MODE, 1>((size + 15u) >> 4, grid, block, stream, tab, data, dstride, par, pstride, size, count,
                               out, reset, npar);
    else if (size != FULL_K || npar != RS_NR)
        RS_LAUNCH((rs_lfsr_k<MODE, PATH_GENERIC>), grid, block, 0, stream, tab, data, dstride, par, pstride,
                           size, count, out, reset, npar);
    else if (MODE != MODE_ENCODE && parity == data + FULL_K && pstride == dstride)
        RS_LAUNCH((rs_lfsr_k<MODE, PATH_CONTIG>), grid, block, 0, stream, tab, data, dstride, par, pstride,
                           size, count, out, reset, npar);
    else
        RS_LAUNCH((rs_lfsr_k<MODE, PATH_SPLIT>), grid, block, 0, stream, tab, data, dstride, par, pstride,
                           size, count, out, reset, npar);
    return hipGetLastError();
}

extern "C" hipError_t rsk_encode(const RsDevTables *tab, const uint8_t *data, size_t dstride, uint8_t *parity,
                                 size_t pstride, uint32_t size, size_t count, int num_cu, hipStream_t stream)
{
    return launch_lfsr<MODE_ENCODE>(tab, data, dstride, parity, pstride, size, count, nullptr, num_cu, stream);
}

/* Byte-symbol codes with npar < 32 roots (the general-parameter handles):
 * the same LFSR with g'(x) = g(x) x^(32 - npar), whose rows the host builds
 * with zeros in the low 32 - npar bytes (api.cpp build_lfsr_rows):
 * m(x) x^32 mod g' = (m(x) x^npar mod g) x^(32 - npar), so the register's
 * first npar bytes are the parity, highest degree first, the rest stay 0. */
extern "C" hipError_t rsk_encode_nr(const RsDevTables *tab, const uint8_t *data, size_t dstride, uint8_t *parity,
                                    size_t pstride, uint32_t size, size_t count, uint32_t npar, int num_cu,
                                    hipStream_t stream)
{
    return launch_lfsr<MODE_ENCODE>(tab, data, dstride, parity, pstride, size, count, nullptr, num_cu, stream, nullptr,
                                    npar);
}

extern "C" hipError_t rsk_syndrome(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                   size_t pstride, uint32_t size, size_t count, uint8_t *syn, int num_cu,
                                   hipStream_t stream)
{
    return launch_lfsr<MODE_SYNDROME>(tab, data, dstride, parity, pstride, size, count, syn, num_cu, stream);
}

extern "C" hipError_t rsk_syndrome_reset(const RsDevTables *tab, const uint8_t *data, size_t dstride,
                                         const uint8_t *parity, size_t pstride, uint32_t size, size_t count,
                                         uint8_t *syn, uint32_t *reset, int num_cu, hipStream_t stream)
{
    return launch_lfsr<MODE_SYNDROME>(tab, data, dstride, parity, pstride, size, count, syn, num_cu, stream, reset);
}

/* the same for a byte-symbol code of npar < 32 roots (tab built by
 * api.cpp build_tables_nr: LFSR rows of g(x) x^(32 - npar), syndrome tables
 * S_i = sum_(m < npar) E'_m beta_i^(npar - 1 - m) for i < npar, zero rows
 * elsewhere): npar syndromes, zeros behind them */
extern "C" hipError_t rsk_syndrome_reset_nr(const RsDevTables *tab, const uint8_t *data, size_t dstride,
                                            const uint8_t *parity, size_t pstride, uint32_t size, size_t count,
                                            uint8_t *syn, uint32_t *reset, uint32_t npar, int num_cu,
                                            hipStream_t stream)
{
    return launch_lfsr<MODE_SYNDROME>(tab, data, dstride, parity, pstride, size, count, syn, num_cu, stream, reset,
                                      npar);
}

/* poly-form syndromes (rsk_syndrome's output) -> the reference's log form:
 * uint16 log S_i (255 = zero) and the "any nonzero" flag (src/decode.c:409-414) */
__global__ __launch_bounds__(256) void rs_synlog_k(const RsDevTables *__restrict__ T, const uint8_t *__restrict__ syn,
                                                   size_t count, uint16_t *__restrict__ out, size_t stride,
                                                   uint8_t *__restrict__ flag, uint32_t nout)
{
    __shared__ uint8_t lg[256];
    lg[threadIdx.x] = T->log[threadIdx.x];
    __syncthreads();
    const size_t cw = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (cw >= count)
        return;
    uint32_t any = 0;
    for (uint32_t i = 0; i < RS_NR; ++i) {
        const uint32_t v = syn[cw * RS_NR + i];
        any |= v;
        if (out && i < nout) /* nout = num_roots (zeros behind the syndromes of a code with fewer roots) */
            out[cw * stride + i] = lg[v];
    }
    if (flag)
        flag[cw] = any != 0u;
}

extern "C" hipError_t rsk_syn_log(const RsDevTables *tab, const uint8_t *syn, size_t count, uint16_t *out,
                                  size_t stride, uint8_t *flag, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const size_t blocks = (count + 255) / 256;
    RS_LAUNCH(rs_synlog_k, dim3((uint32_t)blocks), dim3(256), 0, stream, tab, syn, count, out, stride, flag,
              (uint32_t)RS_NR);
    return hipGetLastError();
}

extern "C" hipError_t rsk_syn_log_nr(const RsDevTables *tab, const uint8_t *syn, size_t count, uint16_t *out,
                                     size_t stride, uint8_t *flag, uint32_t npar, hipStream_t stream)
{
    if (count == 0)
        return hipSuccess;
    const size_t blocks = (count + 255) / 256;
    RS_LAUNCH(rs_synlog_k, dim3((uint32_t)blocks), dim3(256), 0, stream, tab, syn, count, out, stride, flag, npar);
    return hipGetLastError();
}

/* External log-form syndromes (the config's "syndrome" branch, src/decode.c:
 * 446-464) -> the split decode's poly-form syndromes (32 B per codeword,
 * zeros past npar).  A value above 255 (out of table in the reference) makes
 * the codeword the list's: its syndromes are written as zeros (the split
 * kernels pass it by as clean) and the list kernel, reading the external
 * syndromes itself, refuses it (ok 0, corrected 0).  *nlist must be 0. */
__global__ __launch_bounds__(256) void rs_ext_syn_k(const RsDevTables *__restrict__ T, const uint16_t *__restrict__ ext,
                                                    size_t ext_stride, size_t count, uint32_t npar,
                                                    uint8_t *__restrict__ syn, uint32_t *__restrict__ list,
                                                    uint32_t *__restrict__ nlist)
{
    __shared__ uint8_t ex[256];
    ex[threadIdx.x] = T->exp2[threadIdx.x];
    __syncthreads();
    const size_t cw = (size_t)blockIdx.x * 256u + threadIdx.x;
    if (cw >= count)
        return;
    const uint16_t *e = ext + cw * ext_stride;
    uint32_t w[RS_NR / 4] = {0, 0, 0, 0, 0, 0, 0, 0};
    bool bad = false;
#pragma unroll
    for (uint32_t i = 0; i < RS_NR; ++i) {
        if (i < npar) { /* uniform */
            const uint32_t v = e[i];
            bad |= v > 255u;
            w[i >> 2] |= (v >= 255u ? 0u : (uint32_t)ex[v]) << (8u * (i & 3u));
        }
    }
    if (bad) {
#pragma unroll
        for (int k = 0; k < RS_NR / 4; ++k)
            w[k] = 0;
        list[atomicAdd(nlist, 1u)] = (uint32_t)cw;
    }
    uint4 *o = reinterpret_cast<uint4 *>(syn + cw * RS_NR);
    o[0] = make_uint4(w[0], w[1], w[2], w[3]);
    o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

extern "C" hipError_t rsk_ext_syn(const RsDevTables *tab, const uint16_t *ext, size_t ext_stride, size_t count,
                                  uint32_t npar, uint8_t *syn, uint32_t *list, uint32_t *nlist, hipStream_t stream)
{
    const hipError_t me = hipMemsetAsync(nlist, 0, 2 * sizeof(uint32_t), stream);
    if (me != hipSuccess)
        return me;
    if (count == 0)
        return hipSuccess;
    const size_t blocks = (count + 255) / 256;
    RS_LAUNCH(rs_ext_syn_k, dim3((uint32_t)blocks), dim3(256), 0, stream, tab, ext, ext_stride, count, npar, syn, list,
              nlist);
    return hipGetLastError();
}

extern "C" hipError_t rsk_check(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                size_t pstride, uint32_t size, size_t count, uint8_t *flag, int num_cu,
                                hipStream_t stream)
{
    return launch_lfsr<MODE_CHECK>(tab, data, dstride, parity, pstride, size, count, flag, num_cu, stream);
}

/* a code of npar < 32 roots: E' = the received parity + the data's, npar
 * bytes (the flag equals "any syndrome nonzero": distinct roots) */
extern "C" hipError_t rsk_check_nr(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                   size_t pstride, uint32_t size, size_t count, uint8_t *flag, uint32_t npar,
                                   int num_cu, hipStream_t stream)
{
    return launch_lfsr<MODE_CHECK>(tab, data, dstride, parity, pstride, size, count, flag, num_cu, stream, nullptr,
                                   npar);
}
