/*
 * poporon_amd.h -- batch extension of the poporon C API for MI355X.
 *
 * The reference has no batch API: callers loop poporon_encode/poporon_decode
 * one codeword at a time (include/poporon.h:90-91, src/encode.c:236-252,
 * src/decode.c:596-612).  These entry points take many codewords at once
 * behind the same handle.  Each per-codeword result equals what the
 * single-codeword call would return for that codeword (bytes, bool and
 * corrected_num), see tests/test_gpu_parity.py.
 *
 * Layout: codeword c's message is data[c*data_stride .. +size), its parity
 * parity[c*parity_stride .. +num_roots).  Strides and base pointers may have
 * any alignment; 4-byte aligned strides/bases take the fast load path.
 *
 * Device variants take device pointers (hipMalloc'd or any HIP-visible
 * allocation, e.g. a torch tensor's data_ptr()) and enqueue asynchronously on
 * `stream` (a hipStream_t; NULL = the null stream).  Host variants copy
 * through pinned staging in chunks and return when the results are in host
 * memory.  A handle is not reentrant (same rule as the reference handle).
 *
 * The batch calls serve RS handles and BCH handles (PPLN_FEC_BCH, symbol_size
 * 3..5): for BCH, `size` is the message byte count (>= the info byte image),
 * parity rows hold the parity byte image, and there are no erasure or
 * external-syndrome variants; d_corrected[c] = 0 where d_ok[c] = 0.
 *
 * Every entry point returns false and records a message (poporon_amd_last_error)
 * on invalid arguments, an unsupported configuration, or a HIP failure.  There
 * is no CPU fallback: without a usable GPU these calls fail.
 */
#ifndef POPORON_AMD_H
#define POPORON_AMD_H

#include <stddef.h>
#include <stdint.h>

#include "poporon.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Message for the last failing call on this thread ("" if none). */
const char *poporon_amd_last_error(void);

/* poporon_decode (RS) writes this to *corrected_num (and the handle's
 * last_corrected) when the call failed on the device side -- no usable GPU,
 * or a HIP error -- rather than on the codeword: the reference never reports
 * more than num_roots corrections, so a drop-in caller tells "device error"
 * from "uncorrectable" (false with 0..num_roots) without a new entry point. */
#define POPORON_AMD_DEVICE_ERROR ((size_t)-1)

/* Number of HIP devices visible (0 when no GPU / no runtime). */
int poporon_amd_device_count(void);

/* Bind the handle to HIP device `device` (default: the device current at the
 * handle's first GPU call).  Must be called before any GPU work. */
bool poporon_amd_set_device(poporon_t *pprn, int device);

/* Pre-size the handle's device workspace for batches of up to max_count
 * codewords, so that later device calls allocate nothing (graph capture). */
bool poporon_amd_reserve(poporon_t *pprn, size_t max_count);

/* True when the handle's parameters are served by the GPU kernels: byte
 * symbols (2 <= symbol_size <= 8) and 1 <= num_roots < 2^symbol_size - 1,
 * with any field polynomial, fcr and prim that poporon_create accepts.
 * RS(255,223)-shaped parameters (symbol_size 8, num_roots 32, generator
 * without zero coefficients, (fcr+31)*prim+254 < 65536) run on the fast
 * kernels, all others on the general-parameter kernels (same results,
 * lower throughput).  False otherwise (symbol_size 1 or > 8). */
bool poporon_amd_supported(const poporon_t *pprn);

/* ---- device-resident batches (asynchronous on `stream`) ------------------ */

bool poporon_encode_batch_device(poporon_t *pprn, const uint8_t *d_data, size_t data_stride, uint8_t *d_parity,
                                 size_t parity_stride, size_t size, size_t count, void *stream);

/*
 * Decode in place.  d_positions == NULL: errors-only decode (the handle's
 * erasure object and external syndromes, if configured, are NOT used by the
 * batch calls).  Otherwise erasure decode: codeword c's erasure list is
 * d_positions[c*positions_stride .. +num_roots] (uint8 positions into data[], slots
 * past the count are read exactly as the reference reads its erasure object,
 * quirks Q2/Q3), d_counts[c] its count (<= num_roots).
 * d_ok[c] = decode result (1/0); d_corrected[c] = corrected_num (may be NULL).
 */
bool poporon_decode_batch_device(poporon_t *pprn, uint8_t *d_data, size_t data_stride, uint8_t *d_parity,
                                 size_t parity_stride, size_t size, size_t count, const uint8_t *d_positions,
                                 size_t positions_stride, const uint8_t *d_counts, uint8_t *d_ok,
                                 uint8_t *d_corrected, void *stream);

/*
 * External-syndrome decode (the config's "syndrome" branch, src/decode.c:
 * 446-464) for a batch: codeword c's num_roots log-form syndromes (value
 * 2^symbol_size - 1 = zero, the reference's uint16 type) are
 * d_syndromes[c*syndrome_stride .. +num_roots].  All-zero syndromes leave the
 * codeword untouched with d_ok[c] = 1; otherwise the correction runs on them.
 * A value above 2^symbol_size - 1 (an out-of-table index in the reference)
 * gives d_ok[c] = 0, d_corrected[c] = 0.
 */
bool poporon_decode_batch_syndrome_device(poporon_t *pprn, uint8_t *d_data, size_t data_stride, uint8_t *d_parity,
                                          size_t parity_stride, size_t size, size_t count,
                                          const uint16_t *d_syndromes, size_t syndrome_stride, uint8_t *d_ok,
                                          uint8_t *d_corrected, void *stream);

/*
 * Syndromes of a batch (the reference's calculate_syndrome_u8, src/decode.c:
 * 375-415, per codeword): d_syndromes[c*syndrome_stride + i] = log S_i in the
 * reference's uint16 log form (2^symbol_size - 1 = zero), d_nonzero[c] = 1
 * when any S_i is nonzero.  Either output may be NULL (not both).  The
 * result feeds poporon_decode_batch_syndrome_device.
 */
bool poporon_syndrome_batch_device(poporon_t *pprn, const uint8_t *d_data, size_t data_stride,
                                   const uint8_t *d_parity, size_t parity_stride, size_t size, size_t count,
                                   uint16_t *d_syndromes, size_t syndrome_stride, uint8_t *d_nonzero, void *stream);

/* Screening without correction: d_dirty[c] = 1 when codeword c has a nonzero
 * syndrome (the reference's calculate_syndrome_u8 flag, src/decode.c:409-414),
 * else 0.  Reads data and parity only. */
bool poporon_check_batch_device(poporon_t *pprn, const uint8_t *d_data, size_t data_stride, const uint8_t *d_parity,
                                size_t parity_stride, size_t size, size_t count, uint8_t *d_dirty, void *stream);

/* ---- host-memory batches (synchronous) ------------------------------------ */

bool poporon_encode_batch(poporon_t *pprn, const uint8_t *data, size_t data_stride, uint8_t *parity,
                          size_t parity_stride, size_t size, size_t count);

bool poporon_decode_batch(poporon_t *pprn, uint8_t *data, size_t data_stride, uint8_t *parity, size_t parity_stride,
                          size_t size, size_t count, const uint8_t *positions, size_t positions_stride,
                          const uint8_t *counts, uint8_t *ok, uint8_t *corrected);

/* ---- in-library kernel timing ----------------------------------------------
 * When enabled, every kernel the handle launches is bracketed by HIP events
 * recorded on the stream it runs on.  poporon_amd_timing(pprn, 1) enables and
 * resets the totals; poporon_amd_timing_read waits for the recorded events and
 * returns the summed kernel time (ms) and launch count for one kernel id:
 * 0 = encode LFSR, 1 = remainder LFSR, 2 = correction (single kernel),
 * 3 = check LFSR; the split error-mode decode of large batches: 4 = BM +
 * Omega, 5 = Chien, 6 = Forney, 8 = apply, 7 = the one-codeword-per-wave
 * decoder over the codewords the split kernels hand on.  Erasure-mode
 * batches of that size: 1, 9 = the 32-sorted-erasure kernel (prim 1), 4 / 5
 * / 6 = the errata kernels, 7 = the same per-wave decoder over the rest, 8 =
 * apply.  A batch of one codeword: 10 = the one-workgroup decoder
 * (rs_dec1_k), 0 = encode (rs_enc1_k).  Batches of 2..16383 codewords: 11 =
 * the one-codeword-per-wave decoder (rs_wave_k, syndromes included).
 *
 * Error- and erasure-mode batches of at least 16384 codewords take the split
 * decode; POPORON_AMD_DECODE_PATH=split / single / wave in the environment
 * at poporon_create forces the split kernels, the lane-per-codeword general
 * kernel (rs_correct_k) or the per-wave decoder for every batch size. */
#define POPORON_AMD_KERNEL_ENCODE 0
#define POPORON_AMD_KERNEL_REMAINDER 1
#define POPORON_AMD_KERNEL_CORRECT 2
#define POPORON_AMD_KERNEL_CHECK 3
#define POPORON_AMD_KERNEL_BM 4
#define POPORON_AMD_KERNEL_CHIEN 5
#define POPORON_AMD_KERNEL_FORNEY 6
#define POPORON_AMD_KERNEL_LIST 7
#define POPORON_AMD_KERNEL_APPLY 8
#define POPORON_AMD_KERNEL_ERASURE 9
#define POPORON_AMD_KERNEL_SINGLE 10
#define POPORON_AMD_KERNEL_WAVE 11
bool poporon_amd_timing(poporon_t *pprn, int enable);
bool poporon_amd_timing_read(poporon_t *pprn, int kernel, double *total_ms, uint64_t *launches);

/* ---- deterministic payloads -------------------------------------------------
 * Write size bytes of rng's stream (the bytes poporon_rng_next(rng, dest, size)
 * would write, include/poporon/rng.h) into device memory d_dest, on stream
 * (the current HIP device), and advance rng as that call would.  The block
 * start states are derived on the host by GF(2) jump-ahead (rng.hip). */
bool poporon_amd_rng_fill_device(poporon_rng_t *rng, void *d_dest, size_t size, void *stream);

/* ---- multi-GPU: one handle per device, contiguous codeword ranges ----------
 * Codewords are independent, so a batch of count codewords is split into
 * contiguous ranges: device i (of G) takes [count*i/G, count*(i+1)/G)
 * (poporon_amd_multi_range).  No data moves between devices.  Per-codeword
 * results equal the single-device (and single-codeword) results.
 *
 * poporon_amd_multi_create makes one handle per listed device (devices NULL:
 * every visible device) from the same config (copied; erasure / syndrome
 * pointers borrowed as by poporon_create) and initialises each device.  A
 * device may be listed more than once (independent handles sharing it); each
 * listing is a full handle with its own streams, device tables (0.3 MB),
 * split-decode workspace (160 B per codeword of its largest decode batch),
 * single-call buffers and host-pipeline pinned slots, so repeats multiply
 * that memory (no cap: the caller chooses the list).
 * The host entry points take the arguments of poporon_encode_batch /
 * poporon_decode_batch and run one host thread per device over its range.
 * The device entry points take per-device pointer arrays: element i points to
 * device i's range of rows in that device's memory; the work is enqueued on
 * streams[i] (streams NULL: each device's null stream). */
typedef struct _poporon_multi_t poporon_multi_t;

poporon_multi_t *poporon_amd_multi_create(const poporon_config_t *config, const int *devices, size_t num_devices);
void poporon_amd_multi_destroy(poporon_multi_t *multi);
size_t poporon_amd_multi_device_count(const poporon_multi_t *multi);
/* device i's handle (e.g. for poporon_amd_timing); owned by the multi handle */
poporon_t *poporon_amd_multi_handle(poporon_multi_t *multi, size_t index);
/* the range [*first, *first + *n) of part `part` out of `parts` */
bool poporon_amd_multi_range(size_t count, size_t parts, size_t part, size_t *first, size_t *n);

bool poporon_encode_batch_multi(poporon_multi_t *multi, const uint8_t *data, size_t data_stride, uint8_t *parity,
                                size_t parity_stride, size_t size, size_t count);
bool poporon_decode_batch_multi(poporon_multi_t *multi, uint8_t *data, size_t data_stride, uint8_t *parity,
                                size_t parity_stride, size_t size, size_t count, const uint8_t *positions,
                                size_t positions_stride, const uint8_t *counts, uint8_t *ok, uint8_t *corrected);
bool poporon_encode_batch_multi_device(poporon_multi_t *multi, const uint8_t *const *d_data, size_t data_stride,
                                       uint8_t *const *d_parity, size_t parity_stride, size_t size, size_t count,
                                       void *const *streams);
bool poporon_decode_batch_multi_device(poporon_multi_t *multi, uint8_t *const *d_data, size_t data_stride,
                                       uint8_t *const *d_parity, size_t parity_stride, size_t size, size_t count,
                                       const uint8_t *const *d_positions, size_t positions_stride,
                                       const uint8_t *const *d_counts, uint8_t *const *d_ok,
                                       uint8_t *const *d_corrected, void *const *streams);

#ifdef __cplusplus
}
#endif

#endif /* POPORON_AMD_H */
