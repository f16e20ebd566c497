/*
 * bch_device.h -- parameters and launchers of the binary BCH kernels
 * (bch.hip), built by api.cpp from a PPLN_FEC_BCH handle.
 */
#ifndef POPORON_AMD_BCH_DEVICE_H
#define POPORON_AMD_BCH_DEVICE_H

#include <stddef.h>
#include <stdint.h>

#include <hip/hip_runtime.h>

struct BchParams {
    uint32_t m, nn, t;     /* symbol size, 2^m - 1 (= codeword bits), correction capability */
    uint32_t k, pbits;     /* data bits, parity bits (src/bch.c:264-267) */
    uint32_t gen, gdeg;    /* binary generator polynomial and its degree */
    uint32_t dbytes, pbytes; /* byte images: (k + 7) / 8, (pbits + 7) / 8 */
    uint8_t alog[32], log[32]; /* GF(2^m) tables (m <= 5) */
};

#ifdef __cplusplus
extern "C" {
#endif

hipError_t bchk_encode(const BchParams *prm, const uint8_t *data, size_t dstride, uint8_t *parity, size_t pstride,
                       size_t count, int num_cu, hipStream_t stream);

/* ok[c] = decode result; corrected[c] = errors fixed (0 on failure); data bytes rewritten on success only */
hipError_t bchk_decode(const BchParams *prm, uint8_t *data, size_t dstride, const uint8_t *parity, size_t pstride,
                       size_t count, uint8_t *ok, uint8_t *corrected, int num_cu, hipStream_t stream);

#ifdef __cplusplus
}
#endif

#endif
