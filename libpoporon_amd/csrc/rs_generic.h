/*
 * rs_generic.h -- tables, parameters and launchers of the general-parameter
 * RS kernels (rs_generic.hip): symbol_size 2..8, any num_roots < 2^m - 1.
 */
#ifndef POPORON_AMD_RS_GENERIC_H
#define POPORON_AMD_RS_GENERIC_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

/* device-resident per-handle tables, built by api.cpp from the handle's GF
 * tables (src/gf.c:29-86) and generator (src/rs.c:29-82) */
struct RsGenTables {
    uint8_t alog[256]; /* log2exp: alpha^i for i < nn, alog[nn] = 0 (entries past nn: 0) */
    uint8_t log[256];  /* exp2log: log[0] = nn (entries past nn: nn) */
    uint8_t gen[256];  /* generator, log form, gen[0..nroots] */
    /* parity of the message 1 followed by d zeros, row d (stride 256), log
     * form, 0xff: zero (the reference's LFSR, src/encode.c:120-143) */
    uint8_t encq[255 * 256];
    /* LFSR rows of rsg_lfsr_k: row fb, register byte i (< 256) = fb' * g_(nr-1-i)
     * for i < nr, 0 past it, fb' = fb & nn (src/encode.c:120-143's feedback
     * of a raw byte, the reference masking it to m bits) */
    uint8_t lrow[256 * 256];
};

struct RsGenParams {
    uint32_t m, nn, magic; /* nn = 2^m - 1; magic = floor(2^32 / nn) + 1 */
    uint32_t fcr, prim, iprim, nroots;
    uint32_t size; /* message bytes per codeword */
    int32_t pad;   /* nn - nroots - size (decode) */
};

#ifdef __cplusplus
extern "C" {
#endif

/* one codeword per wave (latency: single calls, small batches, lists,
 * long root counts); same arguments and results as rsg_encode / rsg_decode,
 * list / list_n as rsg_decode_list */
/* flag / seq (single calls on coherent host memory): the kernel stores seq
 * to *flag with a system-scope release after every result */
hipError_t rsgw_encode(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                       uint8_t *parity, size_t pstride, size_t count, uint32_t *flag, uint32_t seq, int num_cu,
                       hipStream_t stream);
hipError_t rsgw_decode(const RsGenTables *tab, const RsGenParams *prm, uint8_t *data, size_t dstride, uint8_t *parity,
                       size_t pstride, size_t count, const uint16_t *ext, size_t ext_stride, const uint8_t *pos8,
                       const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt, uint8_t *ok, uint8_t *corrected,
                       const uint32_t *list, const uint32_t *list_n, uint32_t *flag, uint32_t seq, int num_cu,
                       hipStream_t stream);

/* the general-parameter single-call server (rs_serve_k's protocol, GZ_* payload) */
hipError_t rsgw_serve(const RsGenTables *tab, const RsGenParams *prm, uint8_t *zc_dev, uint32_t last, uint32_t id,
                      uint32_t yv, uint64_t idle_ticks, uint64_t max_ticks, hipStream_t stream);
hipError_t rsgw_check(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                      const uint8_t *parity, size_t pstride, size_t count, uint8_t *dirty, uint16_t *syn,
                      size_t syn_stride, int num_cu, hipStream_t stream);

/* batch encode on a per-lane LFSR of 16 ceil(nr / 16) register bytes (rows
 * from tab->lrow staged in LDS): codes with more than 32 roots */
hipError_t rsg_lfsr_encode(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                           uint8_t *parity, size_t pstride, size_t count, int num_cu, hipStream_t stream);
hipError_t rsg_encode(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                      uint8_t *parity, size_t pstride, size_t count, int num_cu, hipStream_t stream);

/* ext (nroots u16 log-form syndromes per codeword, ext_stride elements apart)
 * selects the external-syndrome branch; else pos8/pos32 (at most one non-NULL,
 * pos_stride entries per codeword, counts in cnt) the erasure branch; else
 * errors-only decode. */
hipError_t rsg_decode(const RsGenTables *tab, const RsGenParams *prm, uint8_t *data, size_t dstride, uint8_t *parity,
                      size_t pstride, size_t count, const uint16_t *ext, size_t ext_stride, const uint8_t *pos8,
                      const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt, uint8_t *ok, uint8_t *corrected,
                      int num_cu, hipStream_t stream);
/* decode of the codewords list[0 .. *list_n) (the split decode's hand-off for
 * codes of fewer than 32 roots; length read on the device): errors only,
 * external syndromes (ext) or u8 erasure slots (pos8) */
hipError_t rsg_decode_list(const RsGenTables *tab, const RsGenParams *prm, uint8_t *data, size_t dstride,
                           uint8_t *parity, size_t pstride, size_t count, const uint32_t *list, const uint32_t *list_n,
                           const uint16_t *ext, size_t ext_stride, const uint8_t *pos8, size_t pos_stride,
                           const uint8_t *cnt, uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream);

/* dirty[c] = any syndrome nonzero (may be NULL); syn (may be NULL): the
 * nroots log-form syndromes of codeword c at syn[c*syn_stride ..] */
hipError_t rsg_check(const RsGenTables *tab, const RsGenParams *prm, const uint8_t *data, size_t dstride,
                     const uint8_t *parity, size_t pstride, size_t count, uint8_t *dirty, uint16_t *syn,
                     size_t syn_stride, int num_cu, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif
