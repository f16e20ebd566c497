/*
 * poporon.h -- drop-in C API of libpoporon_amd (RS path on MI355X / gfx950).
 *
 * Same symbols, signatures, enums and macros as the reference's
 * include/poporon.h:22-99 (libpoporon, colopl/libpoporon), so existing
 * callers recompile and relink unchanged.  The Reed-Solomon and BCH codecs
 * are served by HIP kernels; LDPC is outside this build's scope: its config
 * constructors are exported so callers still link, but return NULL.
 *
 *   reference symbol                     replaced by (this header)
 *   poporon_rs_config_create    poporon.h:67-69   -> same, src/api.cpp
 *   poporon_ldpc_config_create  poporon.h:71-76   -> stub, returns NULL
 *   poporon_bch_config_create   poporon.h:78-79   -> same (BCH kernels, symbol_size 3..5)
 *   poporon_config_rs_default   poporon.h:81      -> same (8, 0x11D, 1, 1, 32)
 *   poporon_config_ldpc_default / _burst_resistant
 *                               poporon.h:82-83   -> stubs, return NULL
 *   poporon_config_bch_default  poporon.h:84      -> same (4, 0x13, 3)
 *   poporon_config_destroy      poporon.h:85
 *   poporon_create / _destroy   poporon.h:87-88
 *   poporon_encode              poporon.h:90      -> RS / BCH encode kernel (batch of one)
 *   poporon_decode              poporon.h:91      -> RS syndrome + correction / BCH decode kernels
 *   poporon_get_fec_type / _iterations_used / _parity_size / _info_size
 *                               poporon.h:93-96
 *   poporon_version_id / poporon_buildtime
 *                               poporon.h:98-99
 *
 * Batched, device-pointer and multi-GPU entry points: poporon_amd.h.
 */
#ifndef POPORON_H
#define POPORON_H

#include <stdbool.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "poporon/erasure.h"
#include "poporon/gf.h"
#include "poporon/rng.h"

#define POPORON_FEC_RS      1
#define POPORON_FEC_LDPC    2
#define POPORON_FEC_BCH     3
#define POPORON_FEC_UNKNOWN 255

#define POPORON_LDPC_RATE_1_3 0
#define POPORON_LDPC_RATE_1_2 1
#define POPORON_LDPC_RATE_2_3 2
#define POPORON_LDPC_RATE_3_4 3
#define POPORON_LDPC_RATE_4_5 4
#define POPORON_LDPC_RATE_5_6 5

#define POPORON_LDPC_MATRIX_RANDOM    1
#define POPORON_LDPC_MATRIX_QC_RANDOM 2

#ifdef __cplusplus
extern "C" {
#endif

typedef uint32_t poporon_buildtime_t;

typedef struct _poporon_t poporon_t;
typedef struct _poporon_config_t poporon_config_t;

typedef enum {
    PPLN_FEC_RS = POPORON_FEC_RS,
    PPLN_FEC_LDPC = POPORON_FEC_LDPC,
    PPLN_FEC_BCH = POPORON_FEC_BCH,
    PPLN_FEC_UNKNOWN = POPORON_FEC_UNKNOWN,
} poporon_fec_type_t;

typedef enum {
    PPRN_LDPC_RATE_1_3 = POPORON_LDPC_RATE_1_3,
    PPRN_LDPC_RATE_1_2 = POPORON_LDPC_RATE_1_2,
    PPRN_LDPC_RATE_2_3 = POPORON_LDPC_RATE_2_3,
    PPRN_LDPC_RATE_3_4 = POPORON_LDPC_RATE_3_4,
    PPRN_LDPC_RATE_4_5 = POPORON_LDPC_RATE_4_5,
    PPRN_LDPC_RATE_5_6 = POPORON_LDPC_RATE_5_6,
} poporon_ldpc_rate_t;

typedef enum {
    PPRN_LDPC_RANDOM = POPORON_LDPC_MATRIX_RANDOM,
    PPRN_LDPC_QC_RANDOM = POPORON_LDPC_MATRIX_QC_RANDOM,
} poporon_ldpc_matrix_type_t;

poporon_config_t *poporon_rs_config_create(uint8_t symbol_size, uint16_t generator_polynomial,
                                           uint16_t first_consecutive_root, uint16_t primitive_element,
                                           uint8_t num_roots, poporon_erasure_t *erasure, uint16_t *syndrome);

poporon_config_t *poporon_ldpc_config_create(size_t block_size, poporon_ldpc_rate_t rate,
                                             poporon_ldpc_matrix_type_t matrix_type, uint32_t column_weight,
                                             bool use_soft_decode, bool use_outer_interleave, bool use_inner_interleave,
                                             uint32_t interleave_depth, uint32_t lifting_factor,
                                             uint32_t max_iterations, const int8_t *soft_llr, size_t soft_llr_size,
                                             uint64_t seed);

poporon_config_t *poporon_bch_config_create(uint8_t symbol_size, uint16_t generator_polynomial,
                                            uint8_t correction_capability);

poporon_config_t *poporon_config_rs_default(void);
poporon_config_t *poporon_config_ldpc_default(size_t block_size, poporon_ldpc_rate_t rate);
poporon_config_t *poporon_config_ldpc_burst_resistant(size_t block_size, poporon_ldpc_rate_t rate);
poporon_config_t *poporon_config_bch_default(void);
void poporon_config_destroy(poporon_config_t *config);

poporon_t *poporon_create(const poporon_config_t *config);
void poporon_destroy(poporon_t *pprn);

bool poporon_encode(poporon_t *pprn, uint8_t *data, size_t size, uint8_t *parity);
bool poporon_decode(poporon_t *pprn, uint8_t *data, size_t size, uint8_t *parity, size_t *corrected_num);

poporon_fec_type_t poporon_get_fec_type(const poporon_t *pprn);
uint32_t poporon_get_iterations_used(const poporon_t *pprn);
size_t poporon_get_parity_size(const poporon_t *pprn);
size_t poporon_get_info_size(const poporon_t *pprn);

uint32_t poporon_version_id(void);
poporon_buildtime_t poporon_buildtime(void);

#ifdef __cplusplus
}
#endif

#endif /* POPORON_H */
