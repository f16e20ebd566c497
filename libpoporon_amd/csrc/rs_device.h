/*
 * rs_device.h -- parameter blocks shared by the host library and the HIP
 * kernels of libpoporon_amd (RS(n, n-32) over GF(2^8), gfx950).
 */
#ifndef POPORON_AMD_RS_DEVICE_H
#define POPORON_AMD_RS_DEVICE_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

/* Per-kernel timing (api.cpp KernelTimer): while set, every launch passes
 * these events to hipExtLaunchKernel, which stamps them at the kernel's own
 * start (first launch) and end (each launch; the last one stands), so a timed
 * interval holds no queueing or event-record gaps and agrees with a
 * rocprofv3 kernel trace.  Host-side, one per thread (the multi-GPU entry
 * points run one thread per device). */
struct RsLaunchTimer {
    hipEvent_t start, stop;
    int n;
};
extern thread_local RsLaunchTimer rs_launch_timer;
#define RS_LAUNCH(K, G, B, SH, S, ...)                                                                    \
    do {                                                                                                 \
        if (rs_launch_timer.stop)                                                                        \
            hipExtLaunchKernelGGL(K, G, B, SH, S, rs_launch_timer.n++ ? nullptr : rs_launch_timer.start, \
                                  rs_launch_timer.stop, 0u, __VA_ARGS__);                                \
        else                                                                                             \
            hipLaunchKernelGGL(K, G, B, SH, S, __VA_ARGS__);                                             \
    } while (0)

#define RS_NR 32      /* num_roots served by the kernels */
#define RS_A0 255u    /* log of zero */
#define RS_NN 255u    /* field size - 1 */

/*
 * Device-resident per-handle tables (one hipMalloc, built on the host by
 * api.cpp from the handle's GF tables and generator polynomial).
 *
 *  lfsr[fb*2 + h]  : 16-byte half h of the 32-byte LFSR row for feedback byte
 *                    fb: row byte m = alpha^(log fb + g[31-m]) with the
 *                    reference's gf_mod semantics (src/encode.c:126-140), so
 *                    that  p'_m = p_m+1 ^ row_m  is one encode step; stored
 *                    interleaved, dword k = row bytes (k, k+8, k+16, k+24)
 *                    (the register layout of rs_kernels.hip).
 *  exp2[x]         : alpha^(x mod 255) for x < 511 (exp2[255] = 1); exp2[511] = 0
 *                    (log-of-zero sentinel of the correction kernel).
 *  log[v]          : discrete log, log[0] = 255.
 */
struct RsDevTables {
    uint4 lfsr[512];
    uint8_t exp2[512];
    uint8_t log[256];
    /* synt: E' -> syndromes, nibble tables.  E' = the received parity +
     * the parity of the received data (32 bytes, byte m = coefficient of
     * x^(31-m)): the received word is a codeword + E'(x), so S_i = E'(beta_i).
     * For byte m, nibble half n (0 = low, 1 = high) and nibble value v, the
     * 32-byte row (S_i contribution, i = 0..31) is split in two 16-byte
     * planes h:
     *   synt[((m*2 + n)*2 + h)*16 + v]  = bytes i = 16h .. 16h+15 of
     *   (v << 4n) * beta_i^(31-m)   (see RsCorrParams for beta_i).
     * Plane-major layout keeps the 16 rows of a plane in 16 distinct LDS
     * bank slots. */
    uint4 synt[32 * 2 * 2 * 16];
    /* chien[(j-1)*256 + e] = 16 bytes alpha^(e + j*b), b = 0..15: the j-th
     * locator term at 16 consecutive points for a coefficient of log e;
     * entry e = 255 (log of zero) is an all-zero row.  Terms 1..16 serve
     * the error-mode kernels, 1..32 the errata Chien search. */
    uint4 chien[32 * 256];
    /* gfa: the LDS image of the split kernels' GF table (rs_fast.hip header),
     * dword x * 32 + r for x < 512 and replica r < 32:
     *   (exp2[x] << 8) | (la << 16),  la = 128 log x + 4r + 1 for 0 < x < 256,
     *   128 RS_Z0 + 4r for x = 0, 0 for x >= 256
     * (copied into LDS at address 0 by every workgroup: 4 uint4 per thread) */
    uint4 gfa[512 * 32 / 4];
    /* gfc: the LDS image of the general correction kernel's GF table
     * (rs_correct.hip), dword x * 32 + r: (exp2[x] << 8) | (s << 16) with s =
     * 128 log (x & 255), 0xFFFF for x & 255 = 0 */
    uint4 gfc[512 * 32 / 4];
    /* encq[d * 32 + m]: log (255 = zero) of parity byte m of the one-byte
     * message 1 followed by d zero bytes (d < 223): the LFSR is GF-linear, so
     * one codeword's parity is sum_j data_j encq[size - 1 - j] (rs_enc1_k) */
    uint8_t encq[255 * 32]; /* d < 223 (fast codes); d < 255 - nr for a code of nr < 32 roots, bytes m >= nr 255 */
};
#define RS_Z0 200u /* zero sentinel row of gfa (rs_fast.hip) */

/* Parameters of the decode kernels (by value); the syndromes are
 * S_i = c(beta_i), beta_i = alpha^(prim*(fcr+i)). */
struct RsCorrParams {
    uint32_t fcr, prim, iprim;
    uint32_t size;   /* message bytes per codeword (1..223) */
    int32_t pad;     /* 255 - 32 - size */
    uint32_t vfast;  /* (fcr+31)*prim*254 < 32768: verification exponents need no int16 emulation */
    uint32_t force_verify; /* run the re-syndrome check even where it provably passes (tests) */
    uint32_t nr;     /* num_roots: 32, or fewer (rs_dec1_k of a fewer-roots code) */
};

/*
 * Workspace of the split error-mode decode (rs_fast.hip), carved from one
 * device buffer for `cap` codewords (every array 16-byte aligned):
 *   syn   32 B  poly-form syndromes (rsk_syndrome)
 *   lam   16 B  log Lambda_1..16 (255 = zero)            (rsk_bm)
 *   om    16 B  log Omega_0..15 (255 = zero)             (rsk_bm)
 *   roots 32 B  root map over the points alpha^i', i' = 0..255 (rsk_chien),
 *               then the corrections: 16 locations, 16 magnitudes (rsk_forney)
 *   ext   64 B  errata decode (rs_errata.hip): log Lambda_1..32 || log
 *               Omega_0..31 (rsk_ebm), then the 64-byte correction record
 *               (rsk_forney32, rsk_correct_era_list)
 *   meta   1 B  state << 5 | deg(Lambda)                 (rsk_bm, rsk_chien;
 *               errata: deg & 31, 0 meaning 32)
 *   list   4 B  codewords handed to the general kernel (rsk_correct_list)
 *   nlist  the list's length, then the count of RS_ST_PEND codewords (both
 *          zeroed by rsk_syndrome_reset)
 */
#define RS_ST_DONE 0u /* ok / corrected written */
#define RS_ST_FAST 1u /* deg(Lambda) = L <= 16: Chien, then Forney */
#define RS_ST_LIST 2u /* on the list: the general kernel decodes it */
#define RS_ST_PEND 3u /* erasure mode: left by rs_era_bp_k for the errata kernels */
#define RS_ST_ERRATA 4u /* errata decode: deg(Lambda) = L (deg & 31), Chien and Forney next */

struct RsSplitWs {
    uint8_t *syn, *lam, *om, *roots, *ext, *meta;
    uint32_t *list, *nlist;
};

static inline size_t rs_ws_round16(size_t n) { return (n + 15) & ~(size_t)15; }

static inline size_t rs_ws_bytes(size_t cap)
{
    return 160 * cap + rs_ws_round16(cap) + rs_ws_round16(4 * cap) + 16;
}

static inline RsSplitWs rs_ws_carve(uint8_t *base, size_t cap)
{
    RsSplitWs w;
    w.syn = base;
    w.lam = w.syn + 32 * cap;
    w.om = w.lam + 16 * cap;
    w.roots = w.om + 16 * cap;
    w.ext = w.roots + 32 * cap;
    w.meta = w.ext + 64 * cap;
    w.list = (uint32_t *)(w.meta + rs_ws_round16(cap));
    w.nlist = (uint32_t *)((uint8_t *)w.list + rs_ws_round16(4 * cap));
    return w;
}

#ifdef __cplusplus
extern "C" {
#endif

/* Launchers (rs_kernels.hip).  All asynchronous on `stream`. */
hipError_t rsk_encode(const RsDevTables *tab, const uint8_t *data, size_t dstride, uint8_t *parity, size_t pstride,
                      uint32_t size, size_t count, int num_cu, hipStream_t stream);

/* the same LFSR for a byte-symbol code of npar < 32 roots (g(x) x^(32 - npar)
 * in tab->lfsr): npar parity bytes per codeword */
hipError_t rsk_encode_nr(const RsDevTables *tab, const uint8_t *data, size_t dstride, uint8_t *parity, size_t pstride,
                         uint32_t size, size_t count, uint32_t npar, int num_cu, hipStream_t stream);

/* 32 syndromes (poly form, S_i = c(beta_i)) per codeword into syn: the
 * encoder's LFSR over the data, XORed with the received parity (E'), and the
 * synt transform */
hipError_t rsk_syndrome(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                        size_t pstride, uint32_t size, size_t count, uint8_t *syn, int num_cu, hipStream_t stream);
/* the same, also zeroing *reset before any later launch on the stream runs
 * (the split decode's list length) */
hipError_t rsk_syndrome_reset(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                              size_t pstride, uint32_t size, size_t count, uint8_t *syn, uint32_t *reset, int num_cu,
                              hipStream_t stream);

/* One codeword per launch on one workgroup (rs_single.hip): the single-call
 * paths and batches of one.  flag (may be NULL): `seq` is stored there with
 * a system-scope release after every result (the host polls it).
 *   rsk_encode1  parity of a message of size <= 223
 *   rsk_decode1  rs_decode for one codeword: mode 0 plain, 1 erasure (pos8 or
 *                pos32 slots, count of cnt_bytes = 1 or 4 bytes at cnt), 2
 *                external log-form syndromes (ext, 32 x u16); ok / corrected
 *                one byte each */
hipError_t rsk_encode1(const RsDevTables *tab, const uint8_t *data, uint8_t *parity, uint32_t size, uint32_t *flag,
                       uint32_t seq, hipStream_t stream);
/* the same for a code of npar < 32 roots (encq of build_lfsr_rows), size <= 255 - npar */
hipError_t rsk_encode1_nr(const RsDevTables *tab, const uint8_t *data, uint8_t *parity, uint32_t size, uint32_t npar,
                          uint32_t *flag, uint32_t seq, hipStream_t stream);
hipError_t rsk_decode1(const RsDevTables *tab, const RsCorrParams *prm, uint32_t mode, uint8_t *data,
                       uint8_t *parity, const uint8_t *pos8, const uint32_t *pos32, const void *cnt,
                       uint32_t cnt_bytes, const uint16_t *ext, uint8_t *ok, uint8_t *corrected, uint32_t *flag,
                       uint32_t seq, hipStream_t stream);

/* The single-call server: one resident workgroup serving poporon_encode /
 * poporon_decode requests posted in the coherent host buffer (rs_single.hip
 * rs_serve_k); it leaves after idle_ticks (100 MHz) without a request,
 * max_ticks in all, or when ZC_YIELD differs from yv, storing `id` to
 * ZC_EXITED. */
hipError_t rsk_serve(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *zc_dev, uint32_t last, uint32_t id,
                     uint32_t yv, uint64_t idle_ticks, uint64_t max_ticks, hipStream_t stream);

/* layout of the coherent host buffer of the single-call API (GpuCtx::zc) */
#define ZC_DATA 0    /* message / data bytes (<= 223) */
#define ZC_PAR 256   /* 32 parity bytes */
#define ZC_POS 320   /* 32 erasure slots, u32 */
#define ZC_CNT 448   /* erasure count, u32 */
#define ZC_EXT 512   /* 32 external syndromes, u16 */
#define ZC_OK 576
#define ZC_COR 577
#define ZC_FLAG 640  /* u32 completion word */
/* the single-call server (rs_serve_k): request header written by the host
 * (ZC_REQ last, its own 64-byte line), the server's exit word, the stop word */
#define ZC_REQ 704   /* u32 request word: ZC_REQ_WORD(seq, op, size, mode) */
#define ZC_REQ_WORD(seq, op, size, mode) \
    ((((seq) & 0x3FFFu) << 18) | (((mode) & 3u) << 10) | (((op) & 3u) << 8) | ((size) & 0xFFu))
#define ZC_REQ_OP(w) (((w) >> 8) & 3u)    /* RS_SRV_ENCODE / RS_SRV_DECODE */
#define ZC_REQ_MODE(w) (((w) >> 10) & 3u) /* decode mode (rsk_decode1) */
#define ZC_REQ_SIZE(w) ((w) & 0xFFu)      /* message bytes (1..223) */
/* u32 beside ZC_REQ (one 8-byte poll reads both): bumped by a batch call of
 * another handle on the device (api.cpp yield_servers); a server launched at
 * another value leaves when no request is pending, so it does not hold a CU
 * under that batch's persistent grids */
#define ZC_YIELD 708
#define ZC_EXITED 768 /* u32: the id of the last server launch that has left */
/* general-parameter single calls (rsgw_*_k, one wave): a row of up to 255
 * symbols, up to 254 u32 slots / u16 syndromes */
#define GZ_DATA 1024 /* message / data bytes */
#define GZ_PAR 1280  /* parity bytes */
#define GZ_POS 1536  /* erasure slots, u32 */
#define GZ_CNT 2560  /* erasure count, u8 */
#define GZ_EXT 2576  /* external syndromes, u16 */
#define GZ_OK 3088
#define GZ_COR 3089
#define ZC_BYTES 4096
#define RS_SRV_ENCODE 1u
#define RS_SRV_DECODE 2u
#define RS_SRV_STOP 3u   /* the server leaves (poporon_destroy) */

/* rs_decode for one codeword per wave (rs_single.hip rs_wave_k), corrections
 * in place, ok / corrected per codeword: codewords list[0 .. *list_n) when
 * list != NULL (length read on the device), else 0 .. count - 1 (count bounds
 * the grid either way).  Syndromes: syn (poly form, 32 B per codeword, the
 * split decode's), syn16 (external log form), or neither: computed from the
 * codeword.  pos8 / pos32 (at most one) with u8 counts: erasure mode. */
hipError_t rsk_wave(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride, uint8_t *parity,
                    size_t pstride, size_t count, const uint32_t *list, const uint32_t *list_n, const uint8_t *syn,
                    const uint16_t *syn16, size_t syn16_stride, const uint8_t *pos8, const uint32_t *pos32,
                    size_t pos_stride, const uint8_t *cnt, uint8_t *ok, uint8_t *corrected, int num_cu,
                    hipStream_t stream);

/* poly syndromes (32 B per codeword, rsk_syndrome) -> log form: out[c*stride + i]
 * = log S_i (255 = zero), flag[c] = any S_i nonzero; out / flag may be NULL */
hipError_t rsk_syn_log(const RsDevTables *tab, const uint8_t *syn, size_t count, uint16_t *out, size_t stride,
                       uint8_t *flag, hipStream_t stream);

/* flag[c] = remainder of codeword c is nonzero */
hipError_t rsk_check(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity, size_t pstride,
                     uint32_t size, size_t count, uint8_t *flag, int num_cu, hipStream_t stream);
/* external log-form syndromes (npar per codeword, ext_stride apart) -> the
 * split decode's poly syndromes (syn); refused codewords (a value > 255) put
 * on the list with zero syndromes; zeroes nlist[0..1] first */
hipError_t rsk_ext_syn(const RsDevTables *tab, const uint16_t *ext, size_t ext_stride, size_t count, uint32_t npar,
                       uint8_t *syn, uint32_t *list, uint32_t *nlist, hipStream_t stream);
/* the same two for a byte-symbol code of npar < 32 roots (tables of
 * build_tables_nr): log-form syndromes S_0..S_(npar-1), the remainder flag */
hipError_t rsk_syn_log_nr(const RsDevTables *tab, const uint8_t *syn, size_t count, uint16_t *out, size_t stride,
                          uint8_t *flag, uint32_t npar, hipStream_t stream);
hipError_t rsk_check_nr(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                        size_t pstride, uint32_t size, size_t count, uint8_t *flag, uint32_t npar, int num_cu,
                        hipStream_t stream);

/*
 * Correction.  syn: 32 syndromes per codeword, poly form (from rsk_syndrome);
 * or, when syn16 is non-NULL, 32 log-form u16 syndromes per codeword
 * syn16_stride elements apart (the config's external "syndrome" branch;
 * values > 255 refuse the codeword).  pos8 / pos32 (at most one non-NULL)
 * select erasure mode with per-codeword slot arrays of pos_stride entries
 * and counts in cnt.
 */
hipError_t rsk_correct(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride, uint8_t *parity,
                       size_t pstride, size_t count, const uint8_t *syn, const uint16_t *syn16, size_t syn16_stride,
                       const uint8_t *pos8,
                       const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt, uint8_t *ok, uint8_t *corrected,
                       int num_cu, hipStream_t stream);

/* error-mode correction of the codewords list[0 .. *list_n) (count bounds the
 * grid; the length is read on the device) */
hipError_t rsk_correct_list(const RsDevTables *tab, const RsCorrParams *prm, uint8_t *data, size_t dstride,
                            uint8_t *parity, size_t pstride, size_t count, const uint8_t *syn, const uint32_t *list,
                            const uint32_t *list_n, uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream);

/*
 * Split error-mode decode (rs_fast.hip), after rsk_syndrome_reset into ws.syn:
 *   rsk_bm     Berlekamp-Massey + Omega -> ws.lam / ws.om / ws.meta; clean
 *              codewords finished; deg != L or L > 16 -> ws.list
 *   rsk_chien  root map -> ws.roots; root count != deg finished (failure)
 *   rsk_forney magnitudes -> ws.roots (as correction records), ok / corrected
 *   rsk_apply  the corrections into the codewords
 * then rsk_correct_list over ws.list.  Needs RsCorrParams.vfast.
 */
hipError_t rsk_bm(const RsDevTables *tab, const RsSplitWs *ws, size_t count, uint8_t *ok, uint8_t *corrected,
                  int num_cu, hipStream_t stream);
hipError_t rsk_chien(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, size_t count, uint8_t *ok,
                     uint8_t *corrected, int num_cu, hipStream_t stream);
hipError_t rsk_forney(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, uint8_t *data,
                      size_t dstride, uint8_t *parity, size_t pstride, size_t count, uint8_t *ok, uint8_t *corrected,
                      int num_cu, hipStream_t stream);
hipError_t rsk_apply(const RsCorrParams *prm, const RsSplitWs *ws, uint8_t *data, size_t dstride, uint8_t *parity,
                     size_t pstride, size_t count, hipStream_t stream);

/*
 * The same split decode for a byte-symbol code of npar < 32 roots (tab from
 * api.cpp build_tables_nr; RsCorrParams.pad = 255 - npar - size):
 *   rsk_syndrome_reset_nr  npar syndromes (zeros behind them) into ws.syn
 *   rsk_bm_nr              npar BM iterations; fast only while 2L <= npar
 *   rsk_chien, rsk_forney  unchanged (they depend on pad, fcr and prim only)
 *   rsk_apply_nr           positions below size + npar
 * then the general-parameter kernel over ws.list (rsg_decode_list).
 */
hipError_t rsk_syndrome_reset_nr(const RsDevTables *tab, const uint8_t *data, size_t dstride, const uint8_t *parity,
                                 size_t pstride, uint32_t size, size_t count, uint8_t *syn, uint32_t *reset,
                                 uint32_t npar, int num_cu, hipStream_t stream);
hipError_t rsk_bm_nr(const RsDevTables *tab, const RsSplitWs *ws, size_t count, uint32_t npar, uint8_t *ok,
                     uint8_t *corrected, int num_cu, hipStream_t stream);
hipError_t rsk_apply_nr(const RsCorrParams *prm, const RsSplitWs *ws, uint8_t *data, size_t dstride, uint8_t *parity,
                        size_t pstride, size_t count, uint32_t npar, hipStream_t stream);
/* and its errata decode (erasure batches, u8 slots, pos_stride >= npar, 4-byte
 * aligned rows of slots): rsk_ebm_nr, rsk_chien32, rsk_forney32_nr, the list
 * on the general kernel (rsg_decode_list in erasure mode), rsk_apply_era_nr */
hipError_t rsk_ebm_nr(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, const uint8_t *pos8,
                      size_t pos_stride, const uint8_t *cnt, size_t count, uint8_t *ok, uint8_t *corrected,
                      uint32_t npar, int num_cu, hipStream_t stream);
hipError_t rsk_forney32_nr(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, const uint8_t *pos8,
                           size_t pos_stride, size_t count, uint8_t *ok, uint8_t *corrected, uint32_t npar,
                           int num_cu, hipStream_t stream);
hipError_t rsk_apply_era_nr(const RsCorrParams *prm, const uint8_t *meta, const uint8_t *rec, uint8_t *data,
                            size_t dstride, uint8_t *parity, size_t pstride, size_t count, uint32_t npar,
                            hipStream_t stream);

/*
 * Split erasure-mode decode, after rsk_syndrome into ws.syn:
 *   rsk_correct_era_rec  the general kernel's erasure decode with the
 *                        corrections written as 64-byte records (32 slot
 *                        positions clamped to 255, 32 magnitudes) into rec,
 *                        meta[cw] = RS_ST_FAST where a record was written
 *   rsk_apply_era        the records into the codewords (rs_apply_k<32>)
 * rec: ws.ext.
 */
hipError_t rsk_correct_era_rec(const RsDevTables *tab, const RsCorrParams *prm, size_t count, const uint8_t *syn,
                               const uint8_t *pos8, const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt,
                               uint8_t *ok, uint8_t *corrected, uint8_t *rec, uint8_t *meta, int num_cu,
                               hipStream_t stream);
/* the 32-sorted-erasure kernel (rs_fast.hip: rs_era_bp_k, prim 1, 16-byte
 * aligned u8 slots): records (ws.ext) for its codewords, clean ones finished,
 * the rest RS_ST_PEND for the errata kernels (pend != 0) or onto ws.list
 * (zeroed by rsk_syndrome_reset) for rsk_correct_era_list */
hipError_t rsk_era(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, const uint8_t *pos8,
                   size_t pos_stride, const uint8_t *cnt, size_t count, uint8_t *ok, uint8_t *corrected, uint32_t pend,
                   int num_cu, hipStream_t stream);
hipError_t rsk_correct_era_list(const RsDevTables *tab, const RsCorrParams *prm, size_t count, const uint8_t *syn,
                                const uint8_t *pos8, size_t pos_stride, const uint8_t *cnt, uint8_t *ok,
                                uint8_t *corrected, uint8_t *rec, uint8_t *meta, const uint32_t *list,
                                const uint32_t *list_n, int num_cu, hipStream_t stream);
hipError_t rsk_apply_era(const RsCorrParams *prm, const uint8_t *meta, const uint8_t *rec, uint8_t *data,
                         size_t dstride, uint8_t *parity, size_t pstride, size_t count, hipStream_t stream);

/*
 * Split errata decode (rs_errata.hip): erasure mode with any count of u8
 * slots (pos_stride >= 32, 4-byte aligned rows) and errors, after
 * rsk_syndrome_reset into ws.syn:
 *   rsk_ebm      erasure locator + Berlekamp-Massey from r = count + 1 + Omega
 *                -> ws.ext (logs), ws.meta (RS_ST_ERRATA); clean codewords
 *                finished; deg != L, count > 32 or slots past the codeword ->
 *                ws.list.  only_pend: just the RS_ST_PEND codewords rsk_era left
 *   rsk_chien32  roots of Lambda (degree <= 32) -> ws.roots; count != deg
 *                finished (failure)
 *   rsk_forney32 magnitudes -> ws.ext as 64-byte records (root n's magnitude
 *                with list slot n, as the reference applies them), ok / corrected
 * then rsk_correct_era_list over ws.list (records into ws.ext) and
 * rsk_apply_era(ws.meta, ws.ext).
 */
hipError_t rsk_ebm(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, const uint8_t *pos8,
                   size_t pos_stride, const uint8_t *cnt, size_t count, uint8_t *ok, uint8_t *corrected,
                   uint32_t only_pend, int num_cu, hipStream_t stream);
hipError_t rsk_chien32(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, size_t count, uint8_t *ok,
                       uint8_t *corrected, uint32_t only_pend, int num_cu, hipStream_t stream);
hipError_t rsk_forney32(const RsDevTables *tab, const RsCorrParams *prm, const RsSplitWs *ws, const uint8_t *pos8,
                        size_t pos_stride, size_t count, uint8_t *ok, uint8_t *corrected, uint32_t only_pend,
                        int num_cu, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif
