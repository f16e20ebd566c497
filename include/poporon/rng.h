/*
 * poporon/rng.h -- deterministic byte source (drop-in for the reference's
 * include/poporon/rng.h:14-33): xoshiro128++ seeded through splitmix32
 * (src/rng.c:17-132).  Declares exactly the reference's three functions;
 * the device-memory variant of the same stream is an extension and lives
 * in poporon_amd.h.
 */
#ifndef POPORON_RNG_H
#define POPORON_RNG_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#define POPORON_RNG_TYPE_XOSHIRO128PP 0

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    XOSHIRO128PP = POPORON_RNG_TYPE_XOSHIRO128PP
} poporon_rng_type_t;

typedef struct _poporon_rng_t poporon_rng_t;

/* seed: up to its first 4 bytes are used (NULL / 0 bytes: seed 0) */
poporon_rng_t *poporon_rng_create(poporon_rng_type_t type, void *seed, size_t seed_size);
void poporon_rng_destroy(poporon_rng_t *rng);

/* false for NULL arguments or size == 0; else size bytes, 4 per output word
 * (little-endian), a trailing partial word taking its low bytes */
bool poporon_rng_next(poporon_rng_t *rng, void *dest, size_t size);

#ifdef __cplusplus
}
#endif

#endif /* POPORON_RNG_H */
