/*
 * test_rs_api.c -- the reference's RS codec assertions, in C, against
 * libpoporon_amd.so through include/poporon.h only (a drop-in check: the
 * same source compiles against the reference's header).
 *
 * Follows the checks of /root/reference/tests/test_codec.c:
 *   encode: true, parity not all zero, NULL handle/data/parity -> false  (:40-76)
 *   external syndromes all A0 (255): decode leaves the word, 0 corrected (:78-121)
 *   erasure object with 16 positions: decode restores the data          (:123-168)
 *   decode: clean -> 0 corrected; 1..16 errors -> corrected = n and the
 *   data restored; 17 errors -> false; NULL handle/data/parity, size 0 ->
 *   false; corrected_num may be NULL                                     (:170-233)
 * with error positions drawn from a fixed-seed xorshift over the 64 data
 * bytes and random nonzero magnitudes (the reference's util.h uses 0xFF).
 *
 * `test_rs_api --no-gpu` runs only the argument checks, which fail before
 * any device work (the CPU test suite runs that mode).
 */
#include <poporon.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define NR 32
#define LEN 64

static int failures;
#define CHECK(cond)                                                                                                    \
    do {                                                                                                               \
        if (!(cond)) {                                                                                                 \
            fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #cond);                                   \
            failures++;                                                                                                \
        }                                                                                                              \
    } while (0)

static uint32_t rng_state = 0x2545F491u;
static uint32_t rnd(void)
{
    uint32_t x = rng_state;
    x ^= x << 13;
    x ^= x >> 17;
    x ^= x << 5;
    return rng_state = x;
}

static void random_bytes(uint8_t *p, size_t n)
{
    for (size_t i = 0; i < n; i++)
        p[i] = (uint8_t)rnd();
}

/* n distinct positions in [0, len): partial Fisher-Yates */
static void positions(uint32_t *pos, unsigned n, unsigned len)
{
    uint32_t perm[256];
    for (unsigned i = 0; i < len; i++)
        perm[i] = i;
    for (unsigned i = 0; i < n; i++) {
        unsigned j = i + rnd() % (len - i);
        uint32_t t = perm[i];
        perm[i] = perm[j];
        perm[j] = t;
        pos[i] = perm[i];
    }
}

static void corrupt(uint8_t *data, unsigned n, poporon_erasure_t *erasure)
{
    uint32_t pos[LEN];
    positions(pos, n, LEN);
    if (erasure) /* sorted, as the reference's apply pairs roots and slots in order (quirk Q1) */
        for (unsigned a = 1; a < n; a++)
            for (unsigned b = a; b > 0 && pos[b - 1] > pos[b]; b--) {
                uint32_t t = pos[b];
                pos[b] = pos[b - 1];
                pos[b - 1] = t;
            }
    for (unsigned i = 0; i < n; i++) {
        data[pos[i]] ^= (uint8_t)(1 + rnd() % 255);
        if (erasure)
            poporon_erasure_add_position(erasure, pos[i]);
    }
}

static poporon_t *rs_default(void)
{
    poporon_config_t *config = poporon_config_rs_default();
    poporon_t *pprn = poporon_create(config);
    poporon_config_destroy(config); /* the handle keeps its own copy */
    return pprn;
}

static void argument_checks(void)
{
    poporon_t *pprn = rs_default();
    uint8_t data[LEN] = {0}, parity[NR] = {0};
    size_t n = 99;
    CHECK(pprn != NULL);
    CHECK(poporon_get_fec_type(pprn) == PPLN_FEC_RS);
    CHECK(poporon_get_parity_size(pprn) == NR);
    CHECK(poporon_get_info_size(pprn) == 255 - NR);
    CHECK(poporon_get_iterations_used(pprn) == 0);
    CHECK(poporon_version_id() == 20000000u);
    CHECK(poporon_buildtime() > 0);
    CHECK(!poporon_encode(NULL, data, LEN, parity));
    CHECK(!poporon_encode(pprn, NULL, LEN, parity));
    CHECK(!poporon_encode(pprn, data, LEN, NULL));
    CHECK(!poporon_decode(NULL, data, LEN, parity, &n));
    CHECK(!poporon_decode(pprn, NULL, LEN, parity, &n));
    CHECK(!poporon_decode(pprn, data, LEN, NULL, &n));
    CHECK(!poporon_decode(pprn, data, 0, parity, &n));
    CHECK(poporon_create(NULL) == NULL);
    poporon_destroy(NULL);
    poporon_destroy(pprn);
}

static void codec_checks(void)
{
    poporon_t *pprn = rs_default();
    uint8_t data[LEN], work[LEN], parity[NR], pwork[NR];
    size_t n;
    int nonzero = 0;
    CHECK(pprn != NULL);

    /* encode */
    random_bytes(data, LEN);
    memset(parity, 0, NR);
    CHECK(poporon_encode(pprn, data, LEN, parity));
    for (unsigned i = 0; i < NR; i++)
        nonzero |= parity[i];
    CHECK(nonzero != 0);

    /* decode: clean word, then 1..16 errors */
    memcpy(work, data, LEN);
    memcpy(pwork, parity, NR);
    n = 99;
    CHECK(poporon_decode(pprn, work, LEN, pwork, &n));
    CHECK(n == 0);
    CHECK(memcmp(work, data, LEN) == 0);
    for (unsigned e = 1; e <= NR / 2; e++) {
        memcpy(work, data, LEN);
        memcpy(pwork, parity, NR);
        corrupt(work, e, NULL);
        n = 0;
        CHECK(poporon_decode(pprn, work, LEN, pwork, &n));
        CHECK(n == e);
        CHECK(memcmp(work, data, LEN) == 0 && memcmp(pwork, parity, NR) == 0);
    }
    /* beyond capacity */
    memcpy(work, data, LEN);
    memcpy(pwork, parity, NR);
    corrupt(work, NR / 2 + 1, NULL);
    n = 0;
    CHECK(!poporon_decode(pprn, work, LEN, pwork, &n));
    /* corrected_num may be NULL */
    memcpy(work, data, LEN);
    memcpy(pwork, parity, NR);
    corrupt(work, 1, NULL);
    CHECK(poporon_decode(pprn, work, LEN, pwork, NULL));
    CHECK(memcmp(work, data, LEN) == 0);
    poporon_destroy(pprn);

    /* external syndromes, all A0: nothing to correct */
    {
        uint16_t syndrome[NR];
        for (unsigned i = 0; i < NR; i++)
            syndrome[i] = 0xFF;
        poporon_config_t *config = poporon_rs_config_create(8, 0x11D, 1, 1, NR, NULL, syndrome);
        poporon_t *h = poporon_create(config);
        CHECK(config != NULL && h != NULL);
        CHECK(poporon_encode(h, data, LEN, parity));
        memcpy(work, data, LEN);
        n = 99;
        CHECK(poporon_decode(h, work, LEN, parity, &n));
        CHECK(n == 0);
        CHECK(memcmp(work, data, LEN) == 0);
        poporon_destroy(h);
        poporon_config_destroy(config);
    }

    /* erasures: 16 known positions (borrowed erasure object, read at decode) */
    {
        poporon_erasure_t *erasure = poporon_erasure_create(NR, NR / 2);
        poporon_config_t *config = poporon_rs_config_create(8, 0x11D, 1, 1, NR, erasure, NULL);
        poporon_t *h = poporon_create(config);
        CHECK(erasure != NULL && config != NULL && h != NULL);
        CHECK(poporon_encode(h, data, LEN, parity));
        memcpy(work, data, LEN);
        corrupt(work, NR / 2, erasure);
        n = 0;
        CHECK(poporon_decode(h, work, LEN, parity, &n));
        CHECK(memcmp(work, data, LEN) == 0);
        poporon_erasure_destroy(erasure);
        poporon_destroy(h);
        poporon_config_destroy(config);
    }
}

int main(int argc, char **argv)
{
    const int no_gpu = argc > 1 && strcmp(argv[1], "--no-gpu") == 0;
    argument_checks();
    if (!no_gpu)
        codec_checks();
    if (failures) {
        fprintf(stderr, "%d check(s) failed\n", failures);
        return 1;
    }
    printf("test_rs_api: all checks passed%s\n", no_gpu ? " (argument checks only)" : "");
    return 0;
}
