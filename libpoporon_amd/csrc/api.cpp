/*
 * api.cpp -- the poporon C API of libpoporon_amd (include/poporon.h,
 * include/poporon/erasure.h, include/poporon/gf.h, include/poporon_amd.h).
 *
 * Host side of the drop-in boundary.  Object lifetimes and argument rules
 * follow the reference:
 *   config objects         src/poporon.c:214-233, :281-284, :301-304
 *   handle create/destroy  src/poporon.c:57-110, :172-212
 *   getters, version       src/poporon.c:306-373
 *   erasure list           src/erasure.c:12-127
 *   GF handle              src/gf.c:12-91
 *   generator polynomial   src/rs.c:29-82
 *   encode/decode checks   src/encode.c:236-252, src/decode.c:418-429, :596-612
 * All RS arithmetic on codewords runs in the HIP kernels (rs_kernels.hip);
 * there is no CPU codec in this library.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "poporon.h"
#include "poporon_amd.h"
#include "rs_device.h"
#include "rs_generic.h"
#include "bch_device.h"

#ifndef POPORON_BUILDTIME
#define POPORON_BUILDTIME 1
#endif
#define POPORON_VERSION_ID 20000000

#define EXPORT extern "C" __attribute__((visibility("default")))

/* ------------------------------------------------------------------------ */
/* error reporting                                                          */
/* ------------------------------------------------------------------------ */

static thread_local std::string g_last_error;

static bool fail(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
static bool fail(const char *fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return false;
}

#define HIP_OK(expr)                                                                                                  \
    do {                                                                                                              \
        hipError_t e_ = (expr);                                                                                       \
        if (e_ != hipSuccess)                                                                                         \
            return fail("%s failed: %s", #expr, hipGetErrorString(e_));                                               \
    } while (0)

EXPORT const char *poporon_amd_last_error(void) { return g_last_error.c_str(); }

/* ------------------------------------------------------------------------ */
/* objects                                                                  */
/* ------------------------------------------------------------------------ */

struct _poporon_erasure_t {
    uint32_t capacity;
    uint32_t erasure_count;
    uint32_t *erasure_positions;
    uint16_t *corrections; /* never written; kept for layout/ownership parity */
};

struct _poporon_gf_t {
    uint8_t symbol_size;
    uint8_t field_size; /* uint8 like the reference struct (src/internal/common.h:46-52) */
    uint16_t *log2exp;
    uint16_t *exp2log;
    uint16_t generator_polynomial;
};

struct poporon_rs_t {
    poporon_gf_t *gf;
    uint16_t first_consecutive_root;
    uint16_t primitive_element;
    uint16_t num_roots;
    uint16_t *generator_polynomial; /* log form */
};

struct _poporon_config_t {
    poporon_fec_type_t fec_type;
    uint8_t symbol_size;
    uint16_t generator_polynomial;
    uint16_t first_consecutive_root;
    uint16_t primitive_element;
    uint8_t num_roots;
    poporon_erasure_t *erasure;
    uint16_t *syndrome;
    uint8_t correction_capability; /* BCH */
};

#define NKERN 12
struct TimedLaunch {
    int kernel;
    hipEvent_t a, b;
};

struct GpuCtx {
    bool timing = false;
    std::vector<TimedLaunch> pending;
    std::vector<hipEvent_t> event_pool;
    double total_ms[NKERN] = {};
    uint64_t launches[NKERN] = {};
    bool ready = false;
    int device = -1;
    int num_cu = 256;
    hipStream_t stream = nullptr;
    RsDevTables *tab = nullptr; /* device (fast kernels) */
    RsGenTables *gtab = nullptr; /* device (general-parameter kernels) */
    uint8_t *rem = nullptr;     /* device workspace: rs_ws_bytes(rem_cap) (rs_device.h) */
    size_t rem_cap = 0;
    /* Ordering of the workspace across streams: rem_done is recorded on the
     * stream of the last launch that read rem (rem_stream); a call on another
     * stream waits for it before overwriting rem. */
    hipEvent_t rem_done = nullptr;
    hipStream_t rem_stream = nullptr;
    bool rem_pending = false;
    /* single-codeword staging: device buffer + pinned host mirror, so that a
     * poporon_encode / poporon_decode call is one H2D copy, the kernels and
     * one D2H copy */
    uint8_t *stage = nullptr;
    uint8_t *hstage = nullptr;
    /* single-call paths without copies: ZC_BYTES of fine-grained (coherent,
     * GPU-uncached) host memory the kernels read and write directly (layout
     * ZC_* in rs_device.h); zc_dev is its device address, NULL if unavailable */
    uint8_t *zc = nullptr, *zc_dev = nullptr;
    uint32_t zc_seq = 0; /* completion words of the single-call kernels */
    /* the single-call server (rs_serve_k) on its own stream: srv_on while a
     * launch may still be serving, srv_id the id of the latest launch */
    hipStream_t sstream = nullptr;
    bool srv_on = false;
    uint32_t srv_id = 0;
    uint32_t srv_seq = 0; /* request words of the server (its own count: zc_seq also moves without it) */
    size_t stage_cap = 0;
    /* device registry (dev_register): batch_open while a batch call of this
     * handle is launching, then batch_ev (recorded behind its launches) until
     * the batch has run; other handles' servers stay off meanwhile */
    bool registered = false;
    bool batch_open = false;
    bool batch_ev_live = false;
    hipEvent_t batch_ev = nullptr;
    /* host-batch pipeline: PIPE_SLOTS chunks in flight, one stream each */
    struct PipeSlot {
        hipStream_t stream = nullptr;
        hipEvent_t done = nullptr;
        uint8_t *host = nullptr; /* pinned */
        uint8_t *dev = nullptr;
        size_t cap = 0;
        bool busy = false;
        size_t c0 = 0, n = 0; /* the chunk whose results the slot holds */
    } pipe[3];
};
#define PIPE_SLOTS 3

struct _poporon_t {
    poporon_fec_type_t fec_type;
    poporon_rs_t *rs;
    uint16_t primitive_inverse;
    poporon_erasure_t *erasure; /* borrowed, read live at every decode */
    uint16_t *ext_syndrome;     /* borrowed, read live at every decode */
    size_t last_corrected;
    bool supported; /* fast || generic */
    bool fast;      /* served by the RS(255,223) kernels (rs_kernels.hip, rs_correct.hip) */
    int decode_path; /* 0: by batch size, 1: split kernels (rs_fast.hip), 2: single kernel (rs_correct_k),
                      * 3: one codeword per wave (rs_wave_k) */
    bool generic;   /* served by the general-parameter kernels (rs_generic.hip) */
    bool lfsr_nr;   /* generic code, num_roots <= 32: batch encodes on the LFSR kernel (rsk_encode_nr) */
    bool nrsplit;   /* ... and large error-mode batches decode on the split kernels (params_nrsplit) */
    int gen_path;   /* general kernels: 0 by batch size, 1 one codeword per lane (rsg_*), 2 one per wave
                       (rsgw_*); POPORON_AMD_GENERIC=lane|wave */
    RsDevTables host_tab;
    RsCorrParams corr;
    RsGenTables gen_tab;
    RsGenParams gen;
    /* PPLN_FEC_BCH handles (rs == nullptr) */
    poporon_gf_t *bgf;
    BchParams bch;
    bool bch_ok; /* codewords fit 31 bits: served by bch.hip */
    GpuCtx gpu;
};

/* ------------------------------------------------------------------------ */
/* GF(2^m) and generator (host setup)                                       */
/* ------------------------------------------------------------------------ */

static inline uint8_t gf_mod(const poporon_gf_t *gf, uint16_t v)
{
    while (v >= gf->field_size) {
        v = (uint16_t)(v - gf->field_size);
        v = (uint16_t)((v >> gf->symbol_size) + (v & gf->field_size));
    }
    return (uint8_t)v;
}

EXPORT void poporon_gf_destroy(poporon_gf_t *gf)
{
    if (!gf)
        return;
    free(gf->log2exp);
    free(gf->exp2log);
    free(gf);
}

EXPORT poporon_gf_t *poporon_gf_create(uint8_t symbol_size, uint16_t generator_polynomial)
{
    if (symbol_size < 1 || symbol_size > 16)
        return nullptr;
    poporon_gf_t *gf = (poporon_gf_t *)calloc(1, sizeof(poporon_gf_t));
    if (!gf)
        return nullptr;
    gf->symbol_size = symbol_size;
    gf->field_size = (uint8_t)((1u << symbol_size) - 1u);
    gf->generator_polynomial = generator_polynomial;
    gf->log2exp = (uint16_t *)calloc((size_t)gf->field_size + 1, sizeof(uint16_t));
    gf->exp2log = (uint16_t *)calloc((size_t)gf->field_size + 1, sizeof(uint16_t));
    if (!gf->log2exp || !gf->exp2log) {
        poporon_gf_destroy(gf);
        return nullptr;
    }
    /* powers of x reduced by the field polynomial; log(0) = field_size */
    gf->exp2log[0] = gf->field_size;
    gf->log2exp[gf->field_size] = 0;
    uint16_t x = 1;
    for (uint8_t i = 0; i < gf->field_size; i++) {
        gf->exp2log[x] = i;
        gf->log2exp[i] = x;
        x = (uint16_t)(x << 1);
        if (x & (1u << symbol_size))
            x ^= generator_polynomial;
        x &= gf->field_size;
    }
    if (x != gf->log2exp[0]) { /* not primitive: the walk did not close */
        poporon_gf_destroy(gf);
        return nullptr;
    }
    return gf;
}

EXPORT uint8_t poporon_gf_mod(poporon_gf_t *gf, uint16_t value) { return gf ? gf_mod(gf, value) : 0; }

EXPORT void poporon_rs_destroy(poporon_rs_t *rs)
{
    if (!rs)
        return;
    poporon_gf_destroy(rs->gf);
    free(rs->generator_polynomial);
    free(rs);
}

/* g(x) = prod_{i<num_roots} (x - alpha^(prim*(fcr+i))), stored in log form.
 * The root exponent is a uint16 accumulator as in the reference. */
EXPORT poporon_rs_t *poporon_rs_create(uint8_t symbol_size, uint16_t generator_polynomial,
                                       uint16_t first_consecutive_root, uint16_t primitive_element, uint8_t num_roots)
{
    poporon_gf_t *gf = poporon_gf_create(symbol_size, generator_polynomial);
    if (!gf)
        return nullptr;
    poporon_rs_t *rs = (poporon_rs_t *)calloc(1, sizeof(poporon_rs_t));
    if (!rs) {
        poporon_gf_destroy(gf);
        return nullptr;
    }
    rs->gf = gf;
    rs->first_consecutive_root = first_consecutive_root;
    rs->primitive_element = primitive_element;
    rs->num_roots = num_roots;
    rs->generator_polynomial = (uint16_t *)calloc((size_t)num_roots + 1, sizeof(uint16_t));
    if (!rs->generator_polynomial) {
        poporon_rs_destroy(rs);
        return nullptr;
    }
    uint16_t *g = rs->generator_polynomial;
    g[0] = 1;
    uint16_t root = (uint16_t)(first_consecutive_root * primitive_element);
    for (uint16_t i = 0; i < num_roots; i++, root = (uint16_t)(root + primitive_element)) {
        g[i + 1] = 1;
        for (uint16_t j = i; j > 0; j--)
            g[j] = g[j] ? (uint16_t)(g[j - 1] ^ gf->log2exp[gf_mod(gf, (uint16_t)(gf->exp2log[g[j]] + root))])
                        : g[j - 1];
        g[0] = gf->log2exp[gf_mod(gf, (uint16_t)(gf->exp2log[g[0]] + root))];
    }
    for (uint16_t i = 0; i <= num_roots; i++)
        g[i] = gf->exp2log[g[i]];
    return rs;
}

/* ------------------------------------------------------------------------ */
/* erasure list                                                             */
/* ------------------------------------------------------------------------ */

EXPORT void poporon_erasure_destroy(poporon_erasure_t *e)
{
    if (!e)
        return;
    free(e->erasure_positions);
    free(e->corrections);
    free(e);
}

EXPORT poporon_erasure_t *poporon_erasure_create(uint16_t num_roots, uint32_t initial_capacity)
{
    const uint32_t cap = initial_capacity > 0 ? initial_capacity : (uint32_t)num_roots;
    poporon_erasure_t *e = (poporon_erasure_t *)calloc(1, sizeof(poporon_erasure_t));
    if (!e)
        return nullptr;
    /* zero-filled (the reference leaves slots uninitialised; see quirk Q3) */
    e->erasure_positions = (uint32_t *)calloc(cap ? cap : 1, sizeof(uint32_t));
    e->corrections = (uint16_t *)calloc(cap ? cap : 1, sizeof(uint16_t));
    if (!e->erasure_positions || !e->corrections) {
        poporon_erasure_destroy(e);
        return nullptr;
    }
    e->capacity = cap;
    e->erasure_count = 0;
    return e;
}

EXPORT poporon_erasure_t *poporon_erasure_create_from_positions(uint16_t num_roots, const uint32_t *positions,
                                                                uint32_t count)
{
    if (!positions || count == 0)
        return nullptr;
    poporon_erasure_t *e = poporon_erasure_create(num_roots, count > num_roots ? count : num_roots);
    if (!e)
        return nullptr;
    memcpy(e->erasure_positions, positions, (size_t)count * sizeof(uint32_t));
    e->erasure_count = count;
    return e;
}

EXPORT bool poporon_erasure_add_position(poporon_erasure_t *e, uint32_t position)
{
    if (!e)
        return false;
    if (e->erasure_count >= e->capacity) {
        uint32_t cap = e->capacity * 2;
        if (cap < e->capacity + 32)
            cap = e->capacity + 32;
        uint32_t *np = (uint32_t *)realloc(e->erasure_positions, (size_t)cap * sizeof(uint32_t));
        if (!np)
            return false;
        e->erasure_positions = np;
        uint16_t *nc = (uint16_t *)realloc(e->corrections, (size_t)cap * sizeof(uint16_t));
        if (!nc)
            return false;
        e->corrections = nc;
        memset(e->erasure_positions + e->capacity, 0, (size_t)(cap - e->capacity) * sizeof(uint32_t));
        e->capacity = cap;
    }
    e->erasure_positions[e->erasure_count++] = position;
    return true;
}

EXPORT void poporon_erasure_reset(poporon_erasure_t *e)
{
    if (e)
        e->erasure_count = 0;
}

/* ------------------------------------------------------------------------ */
/* configs                                                                  */
/* ------------------------------------------------------------------------ */

EXPORT poporon_config_t *poporon_rs_config_create(uint8_t symbol_size, uint16_t generator_polynomial,
                                                  uint16_t first_consecutive_root, uint16_t primitive_element,
                                                  uint8_t num_roots, poporon_erasure_t *erasure, uint16_t *syndrome)
{
    poporon_config_t *c = (poporon_config_t *)calloc(1, sizeof(poporon_config_t));
    if (!c)
        return nullptr;
    c->fec_type = PPLN_FEC_RS;
    c->symbol_size = symbol_size;
    c->generator_polynomial = generator_polynomial;
    c->first_consecutive_root = first_consecutive_root;
    c->primitive_element = primitive_element;
    c->num_roots = num_roots;
    c->erasure = erasure;
    c->syndrome = syndrome;
    return c;
}

EXPORT poporon_config_t *poporon_config_rs_default(void)
{
    return poporon_rs_config_create(8, 0x11D, 1, 1, 32, nullptr, nullptr);
}

/* LDPC is outside this build's scope: exported
 * so that callers link, but it constructs nothing. */
EXPORT poporon_config_t *poporon_ldpc_config_create(size_t, poporon_ldpc_rate_t, poporon_ldpc_matrix_type_t, uint32_t,
                                                    bool, bool, bool, uint32_t, uint32_t, uint32_t, const int8_t *,
                                                    size_t, uint64_t)
{
    fail("LDPC is not provided by libpoporon_amd");
    return nullptr;
}
EXPORT poporon_config_t *poporon_bch_config_create(uint8_t symbol_size, uint16_t generator_polynomial,
                                                   uint8_t correction_capability)
{
    poporon_config_t *c = (poporon_config_t *)calloc(1, sizeof(poporon_config_t));
    if (!c)
        return nullptr;
    c->fec_type = PPLN_FEC_BCH;
    c->symbol_size = symbol_size;
    c->generator_polynomial = generator_polynomial;
    c->correction_capability = correction_capability;
    return c;
}
EXPORT poporon_config_t *poporon_config_ldpc_default(size_t, poporon_ldpc_rate_t)
{
    fail("LDPC is not provided by libpoporon_amd");
    return nullptr;
}
EXPORT poporon_config_t *poporon_config_ldpc_burst_resistant(size_t, poporon_ldpc_rate_t)
{
    fail("LDPC is not provided by libpoporon_amd");
    return nullptr;
}
EXPORT poporon_config_t *poporon_config_bch_default(void) { return poporon_bch_config_create(4, 0x13, 3); }

EXPORT void poporon_config_destroy(poporon_config_t *config) { free(config); }

/* ------------------------------------------------------------------------ */
/* handle                                                                   */
/* ------------------------------------------------------------------------ */

static void build_decode_tables(poporon_t *h, uint32_t nr);

/* Kernel tables for the handle (see rs_device.h for their definitions). */
static void build_tables(poporon_t *h)
{
    const poporon_rs_t *rs = h->rs;
    const poporon_gf_t *gf = rs->gf;
    const uint16_t *g = rs->generator_polynomial;
    RsDevTables &t = h->host_tab;
    memset(&t, 0, sizeof(t));
    uint8_t row[32];
    for (uint32_t fb = 0; fb < 256; fb++) {
        for (uint32_t m = 0; m < 32; m++)
            row[m] = fb == 0 ? 0
                             : (uint8_t)gf->log2exp[gf_mod(gf, (uint16_t)(gf->exp2log[fb] + g[RS_NR - 1 - m]))];
        uint32_t il[8]; /* interleaved: dword k = row bytes k, k+8, k+16, k+24 */
        for (uint32_t k = 0; k < 8; k++)
            il[k] = (uint32_t)row[k] | ((uint32_t)row[k + 8] << 8) | ((uint32_t)row[k + 16] << 16) |
                    ((uint32_t)row[k + 24] << 24);
        memcpy(&t.lfsr[fb * 2], il, 16);
        memcpy(&t.lfsr[fb * 2 + 1], il + 4, 16);
    }
    /* encq: the LFSR above run on the message 1, 0, 0, ... (rs_enc1_k) */
    {
        uint8_t q[RS_NR];
        for (uint32_t m = 0; m < RS_NR; m++) /* one step with feedback 1 */
            q[m] = (uint8_t)gf->log2exp[gf_mod(gf, g[RS_NR - 1 - m])];
        for (uint32_t d = 0; d < 223; d++) {
            for (uint32_t m = 0; m < RS_NR; m++)
                t.encq[d * RS_NR + m] = (uint8_t)gf->exp2log[q[m]];
            const uint32_t fb = q[0]; /* next step, input byte 0 */
            for (uint32_t m = 0; m < RS_NR; m++) {
                const uint8_t sh = m + 1 < RS_NR ? q[m + 1] : 0;
                q[m] = sh ^ (fb == 0 ? 0
                                     : (uint8_t)gf->log2exp[gf_mod(gf, (uint16_t)(gf->exp2log[fb] + g[RS_NR - 1 - m]))]);
            }
        }
    }
    build_decode_tables(h, RS_NR);
}

/* Everything but the LFSR rows and encq, for a code of nr <= 32 roots: GF
 * tables, decode parameters, E' -> syndrome nibble tables, Chien rows, the
 * split kernels' GF image.  For nr < 32, E' sits in the first nr register
 * bytes (byte m = coefficient of x^(nr-1-m), zeros behind) and the tables
 * give S_0..S_(nr-1), zeros behind them. */
static void build_decode_tables(poporon_t *h, uint32_t nr)
{
    const poporon_rs_t *rs = h->rs;
    const poporon_gf_t *gf = rs->gf;
    RsDevTables &t = h->host_tab;
    for (uint32_t x = 0; x < 512; x++)
        t.exp2[x] = (uint8_t)gf->log2exp[x % 255];
    t.exp2[511] = 0; /* ZLOG sentinel of the correction kernel (no sum of two logs reaches 511) */
    for (uint32_t v = 0; v < 256; v++)
        t.log[v] = (uint8_t)gf->exp2log[v];

    RsCorrParams &p = h->corr;
    memset(&p, 0, sizeof(p));
    p.fcr = rs->first_consecutive_root;
    p.prim = rs->primitive_element;
    p.iprim = h->primitive_inverse;
    p.vfast = ((uint64_t)(p.fcr + nr - 1) * p.prim * 254u) < 32768u;
    p.nr = nr;

    /* E' -> syndrome nibble tables (rs_device.h) */
    auto gmul = [&](uint32_t x, uint32_t logc) -> uint8_t {
        return x == 0 ? 0 : (uint8_t)gf->log2exp[(gf->exp2log[x] + logc) % 255];
    };
    for (uint32_t m = 0; m < RS_NR; m++) {
        for (uint32_t n = 0; n < 2; n++) {
            for (uint32_t v = 0; v < 16; v++) {
                uint8_t rowb[RS_NR];
                for (uint32_t i = 0; i < RS_NR; i++) {
                    if (m >= nr || i >= nr) {
                        rowb[i] = 0;
                        continue;
                    }
                    const uint64_t e = (uint64_t)(nr - 1 - m) * p.prim * (p.fcr + i);
                    rowb[i] = gmul(v << (4 * n), (uint32_t)(e % 255));
                }
                memcpy(&t.synt[((m * 2 + n) * 2 + 0) * 16 + v], rowb, 16);
                memcpy(&t.synt[((m * 2 + n) * 2 + 1) * 16 + v], rowb + 16, 16);
            }
        }
    }
    /* Chien chunk rows: term j at 16 consecutive points */
    for (uint32_t j = 1; j <= 32; j++) {
        for (uint32_t e = 0; e < 256; e++) {
            uint8_t rowb[16];
            for (uint32_t b = 0; b < 16; b++)
                rowb[b] = e == 255 ? 0 : (uint8_t)gf->log2exp[(e + j * b) % 255];
            memcpy(&t.chien[(j - 1) * 256 + e], rowb, 16);
        }
    }
    /* the split kernels' GF table image (rs_device.h) */
    uint32_t *gfa = reinterpret_cast<uint32_t *>(t.gfa);
    for (uint32_t x = 0; x < 512; x++)
        for (uint32_t r = 0; r < 32; r++) {
            const uint32_t la = x < 256u ? (x ? (uint32_t)t.log[x] * 128u + 4u * r + 1u : 128u * RS_Z0 + 4u * r) : 0u;
            gfa[x * 32 + r] = ((uint32_t)t.exp2[x] << 8) | (la << 16);
        }
    uint32_t *gfc = reinterpret_cast<uint32_t *>(t.gfc);
    for (uint32_t x = 0; x < 512; x++)
        for (uint32_t r = 0; r < 32; r++) {
            const uint32_t v = x & 255u;
            gfc[x * 32 + r] = ((uint32_t)t.exp2[x] << 8) | ((v ? (uint32_t)t.log[v] * 128u : 0xFFFFu) << 16);
        }
    const char *fv = getenv("POPORON_AMD_FORCE_VERIFY");
    p.force_verify = (fv && fv[0] == '1') ? 1u : 0u;
    const char *dp = getenv("POPORON_AMD_DECODE_PATH");
    h->decode_path = !dp ? 0 : !strcmp(dp, "split") ? 1 : !strcmp(dp, "single") ? 2 : !strcmp(dp, "wave") ? 3 : 0;
}

/* General-parameter kernels: byte symbols (2 <= m <= 8) and 1 <= num_roots
 * < 2^m - 1 (at least one message byte); every field polynomial, fcr and
 * prim that poporon_create accepts. */
static bool params_generic(const poporon_t *h)
{
    const poporon_rs_t *rs = h->rs;
    const uint32_t m = rs->gf->symbol_size, nn = rs->gf->field_size;
    return m >= 2 && m <= 8 && rs->num_roots >= 1 && rs->num_roots < nn && rs->primitive_element != 0;
}

static void build_generic(poporon_t *h)
{
    const poporon_rs_t *rs = h->rs;
    const poporon_gf_t *gf = rs->gf;
    RsGenTables &t = h->gen_tab;
    const uint32_t nn = gf->field_size;
    memset(&t, 0, sizeof(t));
    for (uint32_t i = 0; i < 256; i++) {
        t.alog[i] = i <= nn ? (uint8_t)gf->log2exp[i] : 0;
        t.log[i] = i <= nn ? (uint8_t)gf->exp2log[i] : (uint8_t)nn;
    }
    for (uint32_t i = 0; i <= rs->num_roots; i++)
        t.gen[i] = (uint8_t)rs->generator_polynomial[i];
    /* lrow: the rows of rsg_lfsr_k (rs_generic.h) */
    for (uint32_t fb = 0; fb < 256; fb++) {
        const uint32_t v = fb & nn;
        for (uint32_t i = 0; i < rs->num_roots && v != 0; i++)
            t.lrow[fb * 256 + i] = (uint8_t)gf->log2exp[gf_mod(
                gf, (uint16_t)(gf->exp2log[v] + rs->generator_polynomial[rs->num_roots - 1 - i]))];
    }
    /* encq: the register after each byte of the message 1, 0, 0, ... -- the
     * steps of src/encode.c:120-143 as rsg_encode_k takes them (the
     * generator's logs used as they are) */
    {
        const uint32_t nr = rs->num_roots;
        const uint16_t *g = rs->generator_polynomial;
        memset(t.encq, 0xff, sizeof(t.encq));
        std::vector<uint8_t> reg(nr, 0);
        for (uint32_t d = 0; d < nn - nr; d++) {
            const uint32_t fb = gf->exp2log[(d == 0 ? 1u : 0u) ^ reg[0]];
            if (fb != nn)
                for (uint32_t j = 1; j < nr; j++)
                    reg[j] ^= (uint8_t)gf->log2exp[gf_mod(gf, (uint16_t)(fb + g[nr - j]))];
            for (uint32_t j = 0; j + 1 < nr; j++)
                reg[j] = reg[j + 1];
            reg[nr - 1] = fb != nn ? (uint8_t)gf->log2exp[gf_mod(gf, (uint16_t)(fb + g[0]))] : 0;
            for (uint32_t j = 0; j < nr; j++)
                t.encq[d * 256 + j] = reg[j] ? (uint8_t)gf->exp2log[reg[j]] : (uint8_t)0xff;
        }
    }
    RsGenParams &p = h->gen;
    memset(&p, 0, sizeof(p));
    p.m = gf->symbol_size;
    p.nn = nn;
    p.magic = (uint32_t)((1ull << 32) / nn) + 1u;
    p.fcr = rs->first_consecutive_root;
    p.prim = rs->primitive_element;
    p.iprim = h->primitive_inverse;
    p.nroots = rs->num_roots;
}

static bool params_supported(const poporon_t *h)
{
    const poporon_rs_t *rs = h->rs;
    if (rs->gf->symbol_size != 8 || rs->num_roots != RS_NR || rs->primitive_element == 0)
        return false;
    if (((uint32_t)rs->first_consecutive_root + RS_NR - 1) * rs->primitive_element + 254u >= 65536u)
        return false;
    /* distinct roots: then "remainder == 0" <=> "all syndromes are zero" */
    const uint32_t p = rs->primitive_element;
    if (p % 3 == 0 || p % 5 == 0 || p % 17 == 0)
        return false;
    for (uint32_t i = 0; i < RS_NR; i++) /* the LFSR remainder needs a generator without zero coefficients */
        if (rs->generator_polynomial[i] == rs->gf->field_size)
            return false;
    return true;
}

/* Codes with at most 32 roots encode on the RS(255,223) LFSR kernel with
 * g'(x) = g(x) x^(32 - nr) (rsk_encode_nr, rs_kernels.hip; 32 roots: the
 * codes the fast path leaves to the general kernels): the same steps as
 * src/encode.c:120-143 on the first nr register bytes, zeros behind them.
 * Symbols of m < 8 bits too: the register bytes stay below 2^m, so the
 * reference's feedback log[(d & nn) ^ p_0] is row (d ^ p_0) & nn, and the
 * rows of feedback bytes >= 2^m repeat those of their low m bits
 * (build_lfsr_rows).  Like the fast path it needs a generator without zero
 * coefficients (the reference's log-form LFSR reads a zero coefficient's log
 * literally). */
static bool params_lfsr_nr(const poporon_t *h)
{
    const poporon_rs_t *rs = h->rs;
    if (rs->gf->symbol_size > 8 || rs->num_roots == 0 || rs->num_roots > RS_NR || rs->primitive_element == 0)
        return false;
    for (uint32_t i = 0; i < rs->num_roots; i++)
        if (rs->generator_polynomial[i] == rs->gf->field_size)
            return false;
    return true;
}

/* Byte-symbol codes with 2 <= nr < 32 roots decode large error-mode batches
 * on the split kernels (rsk_syndrome_reset_nr .. rsk_apply_nr, the list on
 * the general kernel): the LFSR conditions above, distinct roots (prim
 * coprime to 255: "remainder zero" <=> "all syndromes zero") and the fast
 * path's exponent bound, as params_supported. */
static bool params_nrsplit(const poporon_t *h)
{
    const poporon_rs_t *rs = h->rs;
    if (!params_lfsr_nr(h) || rs->gf->symbol_size != 8 || rs->num_roots < 2 || rs->num_roots >= RS_NR)
        return false; /* GF(2^8) split kernels with npar < 32 (32 roots: the fast path's own codes) */
    const uint32_t p = rs->primitive_element;
    if (p % 3 == 0 || p % 5 == 0 || p % 17 == 0)
        return false;
    return ((uint32_t)rs->first_consecutive_root + rs->num_roots - 1) * p + 254u < 65536u;
}

/* rows of g'(x) = g(x) x^(32 - nr) in the LFSR kernel's interleaved layout:
 * row byte m = fb * g_(nr-1-m) for m < nr (src/encode.c:126-140), 0 past it;
 * feedback byte fb selects the row of fb & nn (m < 8: params_lfsr_nr) */
static void build_lfsr_rows(poporon_t *h)
{
    const poporon_rs_t *rs = h->rs;
    const poporon_gf_t *gf = rs->gf;
    const uint16_t *g = rs->generator_polynomial;
    const uint32_t nr = rs->num_roots;
    RsDevTables &t = h->host_tab;
    memset(&t, 0, sizeof(t));
    uint8_t row[32];
    for (uint32_t fb = 0; fb < 256; fb++) {
        const uint32_t v = fb & gf->field_size;
        for (uint32_t m = 0; m < 32; m++)
            row[m] = (v == 0 || m >= nr)
                         ? 0
                         : (uint8_t)gf->log2exp[gf_mod(gf, (uint16_t)(gf->exp2log[v] + g[nr - 1 - m]))];
        uint32_t il[8];
        for (uint32_t k = 0; k < 8; k++)
            il[k] = (uint32_t)row[k] | ((uint32_t)row[k + 8] << 8) | ((uint32_t)row[k + 16] << 16) |
                    ((uint32_t)row[k + 24] << 24);
        memcpy(&t.lfsr[fb * 2], il, 16);
        memcpy(&t.lfsr[fb * 2 + 1], il + 4, 16);
    }
    /* encq: parity (log form, 255 = zero, stride 32) of the message 1 followed
     * by d zeros, d < 255 - nr: the same LFSR steps (rs_enc1_k) */
    memset(t.encq, 255, sizeof(t.encq));
    uint8_t q[RS_NR];
    for (uint32_t m = 0; m < nr; m++) /* one step with feedback 1 */
        q[m] = (uint8_t)gf->log2exp[gf_mod(gf, g[nr - 1 - m])];
    for (uint32_t d = 0; d < 255u - nr; d++) {
        for (uint32_t m = 0; m < nr; m++)
            t.encq[d * RS_NR + m] = (uint8_t)gf->exp2log[q[m]];
        const uint32_t fb = q[0]; /* next step, input byte 0 */
        for (uint32_t m = 0; m < nr; m++) {
            const uint8_t sh = m + 1 < nr ? q[m + 1] : 0;
            q[m] = sh ^ (fb == 0 ? 0 : (uint8_t)gf->log2exp[gf_mod(gf, (uint16_t)(gf->exp2log[fb] + g[nr - 1 - m]))]);
        }
    }
}

/* ---- BCH handle: generator from minimal polynomials (src/bch.c:184-285) ---- */
static uint32_t bch_min_poly(const poporon_gf_t *gf, uint32_t e)
{
    uint16_t p[64];
    uint32_t deg = 0, c = e, out = 0;
    memset(p, 0, sizeof(p));
    p[0] = 1;
    do {
        const uint16_t root = gf->log2exp[c];
        for (int j = (int)deg; j >= 0; j--) {
            if (j + 1 < 64)
                p[j + 1] ^= p[j];
            p[j] = (p[j] && root) ? gf->log2exp[(gf->exp2log[p[j]] + gf->exp2log[root]) % gf->field_size] : 0;
        }
        deg++;
        c = (c * 2) % gf->field_size;
    } while (c != e);
    for (uint32_t i = 0; i <= deg && i < 32; i++)
        if (p[i] == 1)
            out |= 1u << i;
    return out;
}

static poporon_t *create_bch(const poporon_config_t *config)
{
    const uint32_t m = config->symbol_size, t = config->correction_capability;
    if (m < 3 || m > 16 || t < 1 || t > 16) /* src/bch.c:290-296 */
        return nullptr;
    poporon_gf_t *gf = poporon_gf_create(config->symbol_size, config->generator_polynomial);
    if (!gf)
        return nullptr;
    poporon_t *h = new (std::nothrow) _poporon_t();
    if (!h) {
        poporon_gf_destroy(gf);
        return nullptr;
    }
    h->fec_type = PPLN_FEC_BCH;
    h->rs = nullptr;
    h->bgf = gf;
    BchParams &b = h->bch;
    memset(&b, 0, sizeof(b));
    b.m = m;
    b.nn = gf->field_size;
    b.t = t;
    /* codewords of more than 31 bits overflow the reference's uint32 shifts
     * (undefined behaviour): the handle exists, its codec calls fail */
    h->bch_ok = m <= 5;
    if (h->bch_ok) {
        std::vector<uint8_t> used(b.nn + 1, 0);
        uint32_t gen = 1, gdeg = 0;
        for (uint32_t i = 1; i <= 2 * t; i++) {
            const uint32_t e = i % b.nn;
            if (used[e])
                continue;
            uint32_t c = e;
            do {
                used[c] = 1;
                c = (c * 2) % b.nn;
            } while (c != e);
            const uint32_t mp = bch_min_poly(gf, e);
            uint32_t prod = 0;
            for (uint32_t j = 0; j <= gdeg; j++)
                if (gen & (1u << j))
                    prod ^= mp << j;
            gen = prod;
            gdeg = 31u - (uint32_t)__builtin_clz(gen);
        }
        b.gen = gen;
        b.gdeg = gdeg;
        b.pbits = gdeg;
        b.k = b.nn - gdeg;
        b.dbytes = (b.k + 7) / 8;
        b.pbytes = (b.pbits + 7) / 8;
        for (uint32_t i = 0; i < 32; i++) {
            b.alog[i] = i <= b.nn ? (uint8_t)gf->log2exp[i] : 0;
            b.log[i] = i <= b.nn ? (uint8_t)gf->exp2log[i] : 0;
        }
    }
    return h;
}

EXPORT poporon_t *poporon_create(const poporon_config_t *config)
{
    if (!config)
        return nullptr;
    if (config->fec_type == PPLN_FEC_BCH)
        return create_bch(config);
    if (config->fec_type != PPLN_FEC_RS) {
        fail("LDPC is not provided by libpoporon_amd");
        return nullptr;
    }
    poporon_rs_t *rs = poporon_rs_create(config->symbol_size, config->generator_polynomial,
                                         config->first_consecutive_root, config->primitive_element, config->num_roots);
    if (!rs)
        return nullptr;
    if (config->primitive_element == 0) {
        poporon_rs_destroy(rs);
        return nullptr;
    }
    /* smallest 1 + j*field_size (uint16 arithmetic) divisible by prim, over prim */
    uint32_t tries = 0;
    uint16_t pi;
    for (pi = 1; (pi % config->primitive_element) != 0; pi = (uint16_t)(pi + rs->gf->field_size)) {
        if (++tries > (uint32_t)rs->gf->field_size * 2) {
            poporon_rs_destroy(rs);
            return nullptr;
        }
    }
    poporon_t *h = new (std::nothrow) _poporon_t();
    if (!h) {
        poporon_rs_destroy(rs);
        return nullptr;
    }
    h->fec_type = PPLN_FEC_RS;
    h->rs = rs;
    h->primitive_inverse = (uint16_t)(pi / config->primitive_element);
    h->erasure = config->erasure;
    h->ext_syndrome = config->syndrome;
    h->last_corrected = 0;
    h->fast = params_supported(h);
    h->generic = !h->fast && params_generic(h);
    h->lfsr_nr = h->generic && params_lfsr_nr(h);
    h->nrsplit = h->lfsr_nr && params_nrsplit(h);
    h->supported = h->fast || h->generic;
    {
        const char *gp = getenv("POPORON_AMD_GENERIC");
        h->gen_path = !gp ? 0 : !strcmp(gp, "lane") ? 1 : !strcmp(gp, "wave") ? 2 : 0;
    }
    if (h->fast)
        build_tables(h);
    if (h->generic)
        build_generic(h);
    if (h->lfsr_nr)
        build_lfsr_rows(h);
    if (h->nrsplit)
        build_decode_tables(h, rs->num_roots);
    return h;
}

/* The next request word of the single-call server (rs_serve_k): a new
 * sequence number, and never the word the server saw last -- it acts on a
 * change of the word only (14 bits of sequence wrap). */
static uint32_t srv_word(GpuCtx &g, uint32_t prev, uint32_t op, uint32_t size, uint32_t mode)
{
    uint32_t w;
    do
        w = ZC_REQ_WORD(++g.srv_seq, op, size, mode);
    while (w == prev);
    return w;
}

/* Scoped switch to the handle's device; restores the caller's device. */
struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

/* ------------------------------------------------------------------------ */
/* Handles per device: a batch call and other handles' single-call servers   */
/* ------------------------------------------------------------------------ */

/* A resident single-call server (rs_serve_k / rsgw_serve_k) holds one CU's
 * LDS; a persistent batch grid (rs_lfsr_k: one 128-160 KB workgroup per CU)
 * launched beside it waits for that CU until the server leaves (its idle
 * limit, 1 ms, or 0.5 s while its handle keeps calling).  A batch call stops
 * its own handle's server (srv_stop); the registry below makes the servers of
 * the other handles on the device leave too (yield_servers bumps their
 * ZC_YIELD word, which every server polls with its request word), and keeps
 * them from relaunching while the batch has not run (srv_may_launch): such a
 * single call is served by one launch instead (rs_dec1_k / rs_enc1_k /
 * rsgw_*_k), a kernel that ends on its own.  The reference's handles share
 * nothing (src/poporon.c, no globals); this keeps a handle's batch
 * throughput independent of another thread's single calls. */
#define MAX_DEVS 64
struct DevRegistry {
    std::mutex mu;
    std::vector<GpuCtx *> ctx;
};
static DevRegistry g_devs[MAX_DEVS];

static void dev_register(GpuCtx &g)
{
    if (g.registered || g.device < 0 || g.device >= MAX_DEVS)
        return;
    std::lock_guard<std::mutex> lk(g_devs[g.device].mu);
    g_devs[g.device].ctx.push_back(&g);
    g.registered = true;
}

static void dev_unregister(GpuCtx &g)
{
    if (!g.registered)
        return;
    DevRegistry &r = g_devs[g.device];
    std::lock_guard<std::mutex> lk(r.mu);
    r.ctx.erase(std::remove(r.ctx.begin(), r.ctx.end(), &g), r.ctx.end());
    g.registered = false;
}

/* batch_enter: with other handles on the device, mark this batch open and
 * ask their servers to leave */
static void yield_servers(GpuCtx &g)
{
    if (!g.registered)
        return;
    DevRegistry &r = g_devs[g.device];
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.ctx.size() < 2)
        return;
    g.batch_open = true;
    for (GpuCtx *x : r.ctx)
        if (x != &g && x->zc) {
            volatile uint32_t *y = reinterpret_cast<volatile uint32_t *>(x->zc + ZC_YIELD);
            *y = *y + 1u;
        }
}

/* the end of a batch call: its completion event behind its launches on
 * `stream` (synchronous calls: none) */
static void batch_exit(GpuCtx &g, hipStream_t stream, bool sync)
{
    if (!g.batch_open)
        return;
    DeviceGuard dg(g.device);
    std::lock_guard<std::mutex> lk(g_devs[g.device].mu);
    g.batch_open = false;
    if (sync)
        return;
    if (!g.batch_ev && hipEventCreateWithFlags(&g.batch_ev, hipEventDisableTiming) != hipSuccess) {
        g.batch_ev = nullptr;
        return;
    }
    g.batch_ev_live = hipEventRecord(g.batch_ev, stream) == hipSuccess;
}

struct BatchScope {
    GpuCtx &g;
    hipStream_t stream;
    bool sync;
    ~BatchScope() { batch_exit(g, stream, sync); }
};

/* Frees whatever the context holds, ready or not: a gpu_init that failed
 * half-way leaves a stream or tables behind, and they go here so that the
 * next call retries from scratch. */
static void gpu_release(GpuCtx &g)
{
    const int dev = g.device;
    const bool any = g.ready || g.stream || g.sstream || g.tab || g.gtab || g.rem || g.stage || g.hstage || g.zc ||
                     g.rem_done || g.registered || g.batch_ev ||
                     g.pipe[0].stream || g.pipe[1].stream || g.pipe[2].stream;
    if (!any || dev < 0) {
        g = GpuCtx();
        g.device = dev;
        return;
    }
    dev_unregister(g); /* no other handle touches g.zc or the batch state from here on */
    int prev = -1;
    (void)hipGetDevice(&prev);
    (void)hipSetDevice(dev);
    if (g.stream)
        (void)hipStreamSynchronize(g.stream);
    if (g.batch_ev)
        (void)hipEventDestroy(g.batch_ev);
    if (g.rem_done) {
        (void)hipEventSynchronize(g.rem_done);
        (void)hipEventDestroy(g.rem_done);
    }
    for (auto &t : g.pending) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    for (auto e : g.event_pool)
        (void)hipEventDestroy(e);
    (void)hipFree(g.tab);
    (void)hipFree(g.gtab);
    (void)hipFree(g.rem);
    (void)hipFree(g.stage);
    if (g.hstage)
        (void)hipHostFree(g.hstage);
    if (g.sstream) {
        if (g.zc && g.srv_on) { /* ask a live server to leave now rather than at its idle limit */
            volatile uint32_t *req = reinterpret_cast<volatile uint32_t *>(g.zc + ZC_REQ);
            *req = srv_word(g, *req, RS_SRV_STOP, 0u, 0u);
        }
        (void)hipStreamSynchronize(g.sstream);
        (void)hipStreamDestroy(g.sstream);
    }
    if (g.zc)
        (void)hipHostFree(g.zc);
    for (auto &ps : g.pipe) {
        if (ps.stream)
            (void)hipStreamSynchronize(ps.stream);
        (void)hipHostFree(ps.host);
        (void)hipFree(ps.dev);
        if (ps.done)
            (void)hipEventDestroy(ps.done);
        if (ps.stream)
            (void)hipStreamDestroy(ps.stream);
    }
    if (g.stream)
        (void)hipStreamDestroy(g.stream);
    if (prev >= 0)
        (void)hipSetDevice(prev);
    g = GpuCtx();
    g.device = dev; /* a handle stays bound to the device it was given */
}

EXPORT void poporon_destroy(poporon_t *h)
{
    if (!h)
        return;
    gpu_release(h->gpu);
    poporon_rs_destroy(h->rs);
    poporon_gf_destroy(h->bgf);
    delete h;
}

EXPORT poporon_fec_type_t poporon_get_fec_type(const poporon_t *h) { return h ? h->fec_type : PPLN_FEC_UNKNOWN; }
EXPORT uint32_t poporon_get_iterations_used(const poporon_t *) { return 0; }
/* src/poporon.c:322-362: BCH sizes are the byte images of the parity / data bits */
EXPORT size_t poporon_get_parity_size(const poporon_t *h)
{
    if (!h)
        return 0;
    if (h->fec_type == PPLN_FEC_BCH)
        return h->bch_ok ? h->bch.pbytes : 0;
    return h->rs->num_roots;
}
EXPORT size_t poporon_get_info_size(const poporon_t *h)
{
    if (!h)
        return 0;
    if (h->fec_type == PPLN_FEC_BCH)
        return h->bch_ok ? h->bch.dbytes : 0;
    return (size_t)(h->rs->gf->field_size - h->rs->num_roots);
}
EXPORT uint32_t poporon_version_id(void) { return (uint32_t)POPORON_VERSION_ID; }
EXPORT poporon_buildtime_t poporon_buildtime(void) { return (poporon_buildtime_t)POPORON_BUILDTIME; }

/* ------------------------------------------------------------------------ */
/* GPU context                                                              */
/* ------------------------------------------------------------------------ */

EXPORT int poporon_amd_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess)
        return 0;
    return n;
}

EXPORT bool poporon_amd_supported(const poporon_t *h) { return h && h->supported; }


EXPORT bool poporon_amd_set_device(poporon_t *h, int device)
{
    if (!h)
        return fail("NULL handle");
    if (h->gpu.ready && h->gpu.device != device)
        return fail("handle already bound to device %d", h->gpu.device);
    int n = poporon_amd_device_count();
    if (device < 0 || device >= n)
        return fail("device %d out of range (%d HIP devices)", device, n);
    h->gpu.device = device;
    return true;
}

static bool gpu_init_steps(poporon_t *h);

/* Lazily binds the handle to its device and uploads its tables.  A failure
 * part-way releases what was created, so a later call can retry. */
static bool gpu_init(poporon_t *h)
{
    if (h->gpu.ready)
        return true;
    if (gpu_init_steps(h))
        return true;
    const std::string msg = g_last_error;
    gpu_release(h->gpu);
    g_last_error = msg;
    return false;
}

/* the single-call server (below) leaves before a batch call on its handle:
 * while resident it holds a CU (and, with few hardware queues, may sit ahead of
 * the batch's dispatches) */
static bool srv_stop(poporon_t *h);

/* every batch entry point: the device context, and no live server of this
 * handle beside the batch's kernels */
static bool batch_enter(poporon_t *h)
{
    if (!gpu_init(h) || !srv_stop(h))
        return false;
    yield_servers(h->gpu);
    return true;
}

static bool gpu_init_steps(poporon_t *h)
{
    GpuCtx &g = h->gpu;
    if (h->fec_type == PPLN_FEC_BCH && !h->bch_ok)
        return fail("BCH codewords longer than 31 bits (symbol_size > 5) are not served");
    if (h->fec_type == PPLN_FEC_RS && !h->supported)
        return fail("RS parameters not served by the GPU kernels (need 2 <= symbol_size <= 8 and "
                    "1 <= num_roots < 2^symbol_size - 1)");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
        return fail("no HIP device available (%s); libpoporon_amd has no CPU fallback",
                    e != hipSuccess ? hipGetErrorString(e) : "0 devices");
    if (g.device < 0) {
        int cur = 0;
        HIP_OK(hipGetDevice(&cur));
        g.device = cur;
    }
    DeviceGuard dg(g.device);
    if (!dg.ok)
        return fail("hipSetDevice(%d) failed", g.device);
    hipDeviceProp_t prop;
    HIP_OK(hipGetDeviceProperties(&prop, g.device));
    g.num_cu = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    HIP_OK(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));
    HIP_OK(hipEventCreateWithFlags(&g.rem_done, hipEventDisableTiming));
    if (h->fec_type == PPLN_FEC_BCH) {
        /* parameters and tables go by value with every launch */
    } else if (h->fast) {
        HIP_OK(hipMalloc((void **)&g.tab, sizeof(RsDevTables)));
        HIP_OK(hipMemcpy(g.tab, &h->host_tab, sizeof(RsDevTables), hipMemcpyHostToDevice));
    } else {
        HIP_OK(hipMalloc((void **)&g.gtab, sizeof(RsGenTables)));
        HIP_OK(hipMemcpy(g.gtab, &h->gen_tab, sizeof(RsGenTables), hipMemcpyHostToDevice));
        if (h->lfsr_nr) { /* the LFSR rows of g(x) x^(32 - nr) (+ the split decode's tables: nrsplit) */
            HIP_OK(hipMalloc((void **)&g.tab, sizeof(RsDevTables)));
            HIP_OK(hipMemcpy(g.tab, &h->host_tab, sizeof(RsDevTables), hipMemcpyHostToDevice));
        }
    }
    g.ready = true;
    dev_register(g);
    return true;
}

static bool ensure_rem(poporon_t *h, size_t count)
{
    GpuCtx &g = h->gpu;
    if (g.rem_cap >= count)
        return true;
    size_t cap = std::max(count, (size_t)1024);
    if (g.rem) {
        /* the last reader of rem may run on any stream the caller chose */
        if (g.rem_pending)
            HIP_OK(hipEventSynchronize(g.rem_done));
        g.rem_pending = false;
        HIP_OK(hipStreamSynchronize(g.stream));
        HIP_OK(hipFree(g.rem));
        g.rem = nullptr;
        g.rem_cap = 0;
    }
    HIP_OK(hipMalloc((void **)&g.rem, rs_ws_bytes(cap)));
    g.rem_cap = cap;
    return true;
}

static bool ensure_stage(poporon_t *h, size_t bytes)
{
    GpuCtx &g = h->gpu;
    if (g.stage_cap >= bytes)
        return true;
    size_t cap = std::max(bytes, (size_t)4096);
    if (g.stage || g.hstage) {
        HIP_OK(hipStreamSynchronize(g.stream));
        HIP_OK(hipFree(g.stage));
        if (g.hstage)
            HIP_OK(hipHostFree(g.hstage));
        g.stage = nullptr;
        g.hstage = nullptr;
        g.stage_cap = 0;
    }
    HIP_OK(hipMalloc((void **)&g.stage, cap));
    HIP_OK(hipHostMalloc((void **)&g.hstage, cap, hipHostMallocDefault));
    g.stage_cap = cap;
    return true;
}

EXPORT bool poporon_amd_reserve(poporon_t *h, size_t max_count)
{
    if (!h)
        return fail("NULL handle");
    if (!gpu_init(h))
        return false;
    DeviceGuard dg(h->gpu.device);
    return ensure_rem(h, max_count);
}

/* parity bytes per codeword: num_roots (RS) or the BCH parity byte image */
static size_t par_bytes(const poporon_t *h)
{
    return h->fec_type == PPLN_FEC_BCH ? h->bch.pbytes : h->rs->num_roots;
}

/* largest decodable message size (RS: src/decode.c:418-429); BCH: no upper bound */
static size_t kmax(const poporon_t *h)
{
    return h->fec_type == PPLN_FEC_BCH ? (size_t)-1 : (size_t)h->rs->gf->field_size - h->rs->num_roots;
}

/* Encode sizes: the reference's uint16 byte counter never terminates past
 * 65535 (src/encode.c:121,125, quirk Q7: refused here); a BCH message must
 * hold the info byte image (src/encode.c:210-212). */
static bool check_encode_size(const poporon_t *h, size_t size)
{
    if (h->fec_type == PPLN_FEC_BCH && size < h->bch.dbytes)
        return fail("BCH encode size %zu < info byte image %u", size, (unsigned)h->bch.dbytes);
    if (size > 65535)
        return fail("size %zu > 65535 (the reference's uint16 byte counter never terminates)", size);
    return true;
}

static bool check_decode_size(const poporon_t *h, size_t size)
{
    if (h->fec_type == PPLN_FEC_BCH) /* src/decode.c:553-555, :598 */
        return size >= 1 && size >= h->bch.dbytes;
    /* src/decode.c:418-429: pad = nn - nroots - size must lie in [0, nn - nroots) */
    return size >= 1 && size <= kmax(h);
}

/* ------------------------------------------------------------------------ */
/* in-library kernel timing (HIP events on the launch stream)               */
/* ------------------------------------------------------------------------ */

static hipEvent_t take_event(GpuCtx &g)
{
    hipEvent_t e = nullptr;
    if (!g.event_pool.empty()) {
        e = g.event_pool.back();
        g.event_pool.pop_back();
    } else if (hipEventCreate(&e) != hipSuccess) {
        e = nullptr;
    }
    return e;
}

/* Time the launches of one stage when timing is on: the events ride on the
 * kernels' own dispatches (RS_LAUNCH, rs_device.h) */
thread_local RsLaunchTimer rs_launch_timer = {nullptr, nullptr, 0};

struct KernelTimer {
    GpuCtx &g;
    int kernel;
    hipEvent_t a = nullptr, b = nullptr;
    KernelTimer(GpuCtx &g_, int k, hipStream_t) : g(g_), kernel(k)
    {
        if (!g.timing || (a = take_event(g)) == nullptr)
            return;
        if ((b = take_event(g)) == nullptr) {
            g.event_pool.push_back(a);
            a = nullptr;
            return;
        }
        rs_launch_timer = {a, b, 0};
    }
    /* every call site ends a successful stage with done(true); the destructor
     * alone runs on an early error return (HIP_OK), when a launch may have
     * failed and never recorded its events: they go back to the pool unread */
    void done(bool launched = true)
    {
        if (!a)
            return;
        if (launched && rs_launch_timer.n > 0) {
            g.pending.push_back({kernel, a, b});
        } else { /* nothing (successfully) launched */
            g.event_pool.push_back(a);
            g.event_pool.push_back(b);
        }
        rs_launch_timer = {nullptr, nullptr, 0};
        a = b = nullptr;
    }
    ~KernelTimer() { done(false); }
};

/* Folds the finished stage timings into the totals.  An entry whose events
 * cannot be read is dropped (its events recycled) rather than left queued,
 * so one failed launch cannot wedge every later timing call. */
static bool drain_timing(GpuCtx &g)
{
    bool all = true;
    for (auto &t : g.pending) {
        float ms = 0.f;
        if (hipEventSynchronize(t.b) == hipSuccess && hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
            g.total_ms[t.kernel] += ms;
            g.launches[t.kernel] += 1;
        } else {
            all = false;
        }
        g.event_pool.push_back(t.a);
        g.event_pool.push_back(t.b);
    }
    g.pending.clear();
    if (!all) {
        (void)hipGetLastError();
        return fail("a timed kernel's events could not be read (launch failed?); entry dropped");
    }
    return true;
}

EXPORT bool poporon_amd_timing(poporon_t *h, int enable)
{
    if (!h)
        return fail("NULL handle");
    if (!gpu_init(h))
        return false;
    DeviceGuard dg(h->gpu.device);
    GpuCtx &g = h->gpu;
    if (!drain_timing(g))
        return false;
    for (int k = 0; k < NKERN; k++) {
        g.total_ms[k] = 0;
        g.launches[k] = 0;
    }
    g.timing = enable != 0;
    return true;
}

EXPORT bool poporon_amd_timing_read(poporon_t *h, int kernel, double *total_ms, uint64_t *launches)
{
    if (!h || kernel < 0 || kernel >= NKERN)
        return fail("bad handle or kernel id");
    if (!h->gpu.ready)
        return fail("no GPU work recorded");
    DeviceGuard dg(h->gpu.device);
    if (!drain_timing(h->gpu))
        return false;
    if (total_ms)
        *total_ms = h->gpu.total_ms[kernel];
    if (launches)
        *launches = h->gpu.launches[kernel];
    return true;
}

/* ------------------------------------------------------------------------ */
/* device batches                                                           */
/* ------------------------------------------------------------------------ */

/* The handle's syndrome workspace (rem) is written and read by launches on
 * whatever stream a call names.  Before a call overwrites it, its stream waits
 * for the last launch that read it if that ran on another stream (same stream:
 * already ordered); after its own last reader the call records rem_done. */
static bool rem_acquire(GpuCtx &g, hipStream_t s)
{
    if (g.rem_pending && g.rem_stream != s)
        HIP_OK(hipStreamWaitEvent(s, g.rem_done, 0));
    return true;
}

static bool rem_release(GpuCtx &g, hipStream_t s)
{
    HIP_OK(hipEventRecord(g.rem_done, s));
    g.rem_stream = s;
    g.rem_pending = true;
    return true;
}

/* general parameters: one codeword per 8..64 lanes (rsgw_*) or per lane
 * (rsg_*).  The wave kernels take single calls and batches below 16,384
 * codewords of every code, every large decode batch of codes of 15 symbols
 * or more (round 6: 8 / 16 / 32 lanes per codeword for codes of up to 31 /
 * 63 / 127 symbols, branch-free BM; 65,536 codewords of 2^m - 1 = 15 / 31 /
 * 63 / 127: 40 / 39 / 70 / 184 us against 80 / 84 / 213 / 745 us per lane,
 * profiles/r06_general_lat_{wave,lane}.log) and large encode batches of
 * 255-symbol codes; the per-lane kernels large decode batches of 3- and
 * 7-symbol codes (22 us vs 32 at m = 2) and large encode batches of shorter
 * codes with more than 32 roots (codes with up to 32 take the RS(255,223) LFSR
 * kernel, params_lfsr_nr) */
static bool gen_wave(const poporon_t *h, size_t count, bool encode, size_t size)
{
    const uint32_t nn = h->rs->gf->field_size;
    if (size < 1 || size + h->rs->num_roots > nn) /* the wave kernels hold one row of <= nn symbols */
        return false;
    if (h->gen_path)
        return h->gen_path == 2;
    return count < 16384 || (encode ? nn == 255u : nn >= 15u);
}

#define GEN_LFSR_MIN 1024 /* batch size from which codes of more than 32 roots encode on rsg_lfsr_k */

static bool launch_encode(poporon_t *h, const uint8_t *d_data, size_t ds, uint8_t *d_par, size_t ps, size_t size,
                          size_t count, hipStream_t s)
{
    KernelTimer t(h->gpu, POPORON_AMD_KERNEL_ENCODE, s);
    if (h->fec_type == PPLN_FEC_BCH) {
        HIP_OK(bchk_encode(&h->bch, d_data, ds, d_par, ps, count, h->gpu.num_cu, s));
    } else if (h->fast && count == 1 && size <= 223) { /* one codeword: 223 dependent LFSR steps are the latency */
        HIP_OK(rsk_encode1(h->gpu.tab, d_data, d_par, (uint32_t)size, nullptr, 0, s));
    } else if (h->fast) {
        HIP_OK(rsk_encode(h->gpu.tab, d_data, ds, d_par, ps, (uint32_t)size, count, h->gpu.num_cu, s));
    } else if (h->nrsplit && count == 1 && size <= 255u - h->rs->num_roots) {
        /* one codeword: the whole workgroup (rs_enc1_k reads exp2 / log, which
         * build_decode_tables fills only for nrsplit codes) */
        HIP_OK(rsk_encode1_nr(h->gpu.tab, d_data, d_par, (uint32_t)size, h->rs->num_roots, nullptr, 0u, s));
    } else if (h->lfsr_nr && !h->gen_path) { /* (POPORON_AMD_GENERIC forces the general kernels, as for decode) */
        HIP_OK(rsk_encode_nr(h->gpu.tab, d_data, ds, d_par, ps, (uint32_t)size, count, h->rs->num_roots,
                             h->gpu.num_cu, s));
    } else if (h->rs->num_roots > RS_NR && !h->gen_path && count >= GEN_LFSR_MIN) {
        /* the per-lane LFSR of 16 ceil(nr / 16) bytes (rsg_lfsr_k; smaller
         * batches on the wave kernel, whose codeword spreads over the wave:
         * 64 codewords 27-34 vs 34-41 us, 4,096 39-53 vs 51-53 -> 39-45,
         * 65,536 292-524 vs 43-52 us, profiles/r06_general_lat_auto_v2.log) */
        RsGenParams prm = h->gen;
        prm.size = (uint32_t)size;
        HIP_OK(rsg_lfsr_encode(h->gpu.gtab, &prm, d_data, ds, d_par, ps, count, h->gpu.num_cu, s));
    } else {
        RsGenParams prm = h->gen;
        prm.size = (uint32_t)size;
        if (gen_wave(h, count, true, size))
            HIP_OK(rsgw_encode(h->gpu.gtab, &prm, d_data, ds, d_par, ps, count, nullptr, 0u, h->gpu.num_cu, s));
        else
            HIP_OK(rsg_encode(h->gpu.gtab, &prm, d_data, ds, d_par, ps, count, h->gpu.num_cu, s));
    }
    t.done();
    return true;
}

/* batches from this size on take the split kernels (rs_fast.hip, six
 * launches, one codeword per lane); smaller ones one launch of rs_wave_k (one
 * codeword per wave).  Where they cross (16 errors, wall time per call,
 * profiles/r04_batchlat_*.log): 12,288 codewords 86 vs ~108 us, 16,384 107 vs
 * ~108, 32,768 196 vs ~110 */
#define SPLIT_MIN_COUNT 16384

/* the split error-mode decode of one sub-batch (rs_fast.hip); npar < 32: a
 * byte-symbol code of npar roots (h->nrsplit), its list on the general kernel */
static bool launch_split(poporon_t *h, const RsCorrParams &prm, const RsSplitWs &ws, uint8_t *d_data, size_t ds,
                         uint8_t *d_par, size_t ps, size_t size, size_t count, uint8_t *ok, uint8_t *corrected,
                         hipStream_t s, uint32_t npar = RS_NR, const uint16_t *ext = nullptr, size_t ext_stride = 0)
{
    GpuCtx &g = h->gpu;
    const bool nr = npar < RS_NR;
    {
        KernelTimer t(g, POPORON_AMD_KERNEL_REMAINDER, s);
        if (ext) /* external log-form syndromes (src/decode.c:446-464): converted, refusals to the list */
            HIP_OK(rsk_ext_syn(g.tab, ext, ext_stride, count, npar, ws.syn, ws.list, ws.nlist, s));
        else if (nr)
            HIP_OK(rsk_syndrome_reset_nr(g.tab, d_data, ds, d_par, ps, (uint32_t)size, count, ws.syn, ws.nlist, npar,
                                         g.num_cu, s));
        else
            HIP_OK(rsk_syndrome_reset(g.tab, d_data, ds, d_par, ps, (uint32_t)size, count, ws.syn, ws.nlist,
                                      g.num_cu, s));
        t.done();
    }
    {
        KernelTimer t(g, POPORON_AMD_KERNEL_BM, s);
        if (nr)
            HIP_OK(rsk_bm_nr(g.tab, &ws, count, npar, ok, corrected, g.num_cu, s));
        else
            HIP_OK(rsk_bm(g.tab, &ws, count, ok, corrected, g.num_cu, s));
        t.done();
    }
    {
        KernelTimer t(g, POPORON_AMD_KERNEL_CHIEN, s);
        HIP_OK(rsk_chien(g.tab, &prm, &ws, count, ok, corrected, g.num_cu, s));
        t.done();
    }
    {
        KernelTimer t(g, POPORON_AMD_KERNEL_FORNEY, s);
        HIP_OK(rsk_forney(g.tab, &prm, &ws, d_data, ds, d_par, ps, count, ok, corrected, g.num_cu, s));
        t.done();
    }
    {
        KernelTimer t(g, POPORON_AMD_KERNEL_APPLY, s);
        if (nr)
            HIP_OK(rsk_apply_nr(&prm, &ws, d_data, ds, d_par, ps, count, npar, s));
        else
            HIP_OK(rsk_apply(&prm, &ws, d_data, ds, d_par, ps, count, s));
        t.done();
    }
    {
        /* what the split kernels hand on: one codeword per wave (rs_wave_k) */
        KernelTimer t(g, POPORON_AMD_KERNEL_LIST, s);
        if (nr) {
            RsGenParams gp = h->gen;
            gp.size = (uint32_t)size;
            gp.pad = prm.pad;
            if (h->gen_path == 1)
                HIP_OK(rsg_decode_list(g.gtab, &gp, d_data, ds, d_par, ps, count, ws.list, ws.nlist, ext, ext_stride,
                                       nullptr, 0, nullptr, ok, corrected, g.num_cu, s));
            else
                HIP_OK(rsgw_decode(g.gtab, &gp, d_data, ds, d_par, ps, count, ext, ext_stride, nullptr, nullptr, 0,
                                   nullptr, ok, corrected, ws.list, ws.nlist, nullptr, 0u, g.num_cu, s));
        } else {
            HIP_OK(rsk_wave(g.tab, &prm, d_data, ds, d_par, ps, count, ws.list, ws.nlist, ext ? nullptr : ws.syn, ext,
                            ext_stride, nullptr, nullptr, 0, nullptr, ok, corrected, g.num_cu, s));
        }
        t.done();
    }
    return true;
}

/* rem / rem_cap: a workspace of rs_ws_bytes(rem_cap) bytes (rem_cap >= count)
 * owned by the caller; NULL: the handle's own */
static bool launch_decode(poporon_t *h, uint8_t *d_data, size_t ds, uint8_t *d_par, size_t ps, size_t size,
                          size_t count, const uint16_t *ext_syn, size_t ext_stride, const uint8_t *pos8,
                          const uint32_t *pos32, size_t pos_stride, const uint8_t *cnt, uint8_t *ok,
                          uint8_t *corrected, hipStream_t s, uint8_t *rem = nullptr, size_t rem_cap = 0)
{
    if (h->fec_type == PPLN_FEC_BCH) {
        if (ext_syn || pos8 || pos32)
            return fail("BCH has no erasure or external-syndrome decode");
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_CORRECT, s);
        HIP_OK(bchk_decode(&h->bch, d_data, ds, d_par, ps, count, ok, corrected, h->gpu.num_cu, s));
        t.done();
        return true;
    }
    if (h->nrsplit && count == 1 && h->decode_path == 0) {
        /* one codeword of a fewer-roots code: the whole reference decode on
         * one workgroup (rs_dec1_k with P.nr = num_roots; every mode) */
        RsCorrParams prm = h->corr;
        prm.size = (uint32_t)size;
        prm.pad = (int32_t)(h->rs->gf->field_size - h->rs->num_roots - size);
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_SINGLE, s);
        HIP_OK(rsk_decode1(h->gpu.tab, &prm, ext_syn ? 2u : (pos8 || pos32) ? 1u : 0u, d_data, d_par, pos8, pos32,
                           cnt, 1u, ext_syn, ok, corrected, nullptr, 0, s));
        t.done();
        return true;
    }
    if (h->nrsplit && !pos8 && !pos32 && h->corr.vfast && !h->corr.force_verify &&
        (h->decode_path == 1 || h->decode_path == 0)) {
        /* a byte-symbol code of fewer than 32 roots, errors only: the split
         * kernels with npar = num_roots, the list on the general kernel --
         * at every batch size, single calls included: the general kernel's
         * one lane per codeword takes ~1 ms whatever the count, the six
         * split launches ~0.1 ms from 1 to 65,536 codewords of RS(255,239)
         * (profiles/r05_nr_batchlat.log) */
        RsCorrParams prm = h->corr;
        prm.size = (uint32_t)size;
        prm.pad = (int32_t)(h->rs->gf->field_size - h->rs->num_roots - size);
        const bool shared = !rem;
        if (shared) {
            if (!ensure_rem(h, count) || !rem_acquire(h->gpu, s))
                return false;
            rem = h->gpu.rem;
            rem_cap = h->gpu.rem_cap;
        }
        const RsSplitWs ws = rs_ws_carve(rem, rem_cap ? rem_cap : count);
        if (!launch_split(h, prm, ws, d_data, ds, d_par, ps, size, count, ok, corrected, s, h->rs->num_roots, ext_syn,
                          ext_stride))
            return false;
        return !shared || rem_release(h->gpu, s);
    }
    if (h->nrsplit && pos8 && !ext_syn && h->corr.vfast && !h->corr.force_verify &&
        (h->decode_path == 1 || h->decode_path == 0) && pos_stride >= h->rs->num_roots && pos_stride % 4u == 0u &&
        (reinterpret_cast<uintptr_t>(pos8) & 3u) == 0u) {
        /* ... and its erasure batches (u8 slots in 4-byte aligned rows): the
         * errata kernels with npar = num_roots, the list on the general
         * kernel in erasure mode, the 32-entry record apply */
        const uint32_t nr = h->rs->num_roots;
        RsCorrParams prm = h->corr;
        prm.size = (uint32_t)size;
        prm.pad = (int32_t)(h->rs->gf->field_size - nr - size);
        GpuCtx &g = h->gpu;
        const bool shared = !rem;
        if (shared) {
            if (!ensure_rem(h, count) || !rem_acquire(g, s))
                return false;
            rem = g.rem;
            rem_cap = g.rem_cap;
        }
        const RsSplitWs ws = rs_ws_carve(rem, rem_cap ? rem_cap : count);
        {
            KernelTimer t(g, POPORON_AMD_KERNEL_REMAINDER, s);
            HIP_OK(rsk_syndrome_reset_nr(g.tab, d_data, ds, d_par, ps, (uint32_t)size, count, ws.syn, ws.nlist, nr,
                                         g.num_cu, s));
            t.done();
        }
        {
            KernelTimer t(g, POPORON_AMD_KERNEL_BM, s);
            HIP_OK(rsk_ebm_nr(g.tab, &prm, &ws, pos8, pos_stride, cnt, count, ok, corrected, nr, g.num_cu, s));
            t.done();
        }
        {
            KernelTimer t(g, POPORON_AMD_KERNEL_CHIEN, s);
            HIP_OK(rsk_chien32(g.tab, &prm, &ws, count, ok, corrected, 0u, g.num_cu, s));
            t.done();
        }
        {
            KernelTimer t(g, POPORON_AMD_KERNEL_FORNEY, s);
            HIP_OK(rsk_forney32_nr(g.tab, &prm, &ws, pos8, pos_stride, count, ok, corrected, nr, g.num_cu, s));
            t.done();
        }
        {
            /* the hand-off (meta RS_ST_LIST: the record apply passes them by) */
            KernelTimer t(g, POPORON_AMD_KERNEL_LIST, s);
            RsGenParams gp = h->gen;
            gp.size = (uint32_t)size;
            gp.pad = prm.pad;
            if (h->gen_path == 1)
                HIP_OK(rsg_decode_list(g.gtab, &gp, d_data, ds, d_par, ps, count, ws.list, ws.nlist, nullptr, 0, pos8,
                                       pos_stride, cnt, ok, corrected, g.num_cu, s));
            else
                HIP_OK(rsgw_decode(g.gtab, &gp, d_data, ds, d_par, ps, count, nullptr, 0, pos8, nullptr, pos_stride,
                                   cnt, ok, corrected, ws.list, ws.nlist, nullptr, 0u, g.num_cu, s));
            t.done();
        }
        {
            KernelTimer t(g, POPORON_AMD_KERNEL_APPLY, s);
            HIP_OK(rsk_apply_era_nr(&prm, ws.meta, ws.ext, d_data, ds, d_par, ps, count, nr, s));
            t.done();
        }
        return !shared || rem_release(g, s);
    }
    if (!h->fast) {
        RsGenParams prm = h->gen;
        prm.size = (uint32_t)size;
        prm.pad = (int32_t)(h->rs->gf->field_size - h->rs->num_roots - size);
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_CORRECT, s);
        if (gen_wave(h, count, false, size))
            HIP_OK(rsgw_decode(h->gpu.gtab, &prm, d_data, ds, d_par, ps, count, ext_syn, ext_stride, pos8, pos32,
                               pos_stride, cnt, ok, corrected, nullptr, nullptr, nullptr, 0u, h->gpu.num_cu, s));
        else
            HIP_OK(rsg_decode(h->gpu.gtab, &prm, d_data, ds, d_par, ps, count, ext_syn, ext_stride, pos8, pos32,
                              pos_stride, cnt, ok, corrected, h->gpu.num_cu, s));
        t.done();
        return true;
    }
    RsCorrParams prm = h->corr;
    prm.size = (uint32_t)size;
    prm.pad = (int32_t)(h->rs->gf->field_size - h->rs->num_roots - size);
    if (count == 1) { /* one codeword: one launch on one workgroup (rs_single.hip; it always runs the check) */
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_SINGLE, s);
        HIP_OK(rsk_decode1(h->gpu.tab, &prm, ext_syn ? 2u : (pos8 || pos32) ? 1u : 0u, d_data, d_par, pos8, pos32,
                           cnt, 1u, ext_syn, ok, corrected, nullptr, 0, s));
        t.done();
        return true;
    }
    /* a few thousand codewords: one codeword per wave, syndromes included,
     * one launch (the lane-per-codeword kernels would give each SIMD a few
     * waves, each a ~10^4-step serial chain) */
    if (h->decode_path == 3 || (h->decode_path == 0 && count < SPLIT_MIN_COUNT)) {
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_WAVE, s);
        HIP_OK(rsk_wave(h->gpu.tab, &prm, d_data, ds, d_par, ps, count, nullptr, nullptr, nullptr, ext_syn, ext_stride,
                        pos8, pos32, pos_stride, cnt, ok, corrected, h->gpu.num_cu, s));
        t.done();
        return true;
    }
    /* external syndromes of a large batch: the split kernels from converted
     * syndromes, refusals and what they hand on to rs_wave_k (which reads
     * the external syndromes itself) */
    const bool xsplit = ext_syn && !pos8 && !pos32 && prm.vfast && !prm.force_verify && h->decode_path != 2 &&
                        (h->decode_path == 1 || count >= SPLIT_MIN_COUNT);
    if (xsplit) {
        const bool own = !rem;
        if (own) {
            if (!ensure_rem(h, count) || !rem_acquire(h->gpu, s))
                return false;
            rem = h->gpu.rem;
            rem_cap = h->gpu.rem_cap;
        }
        const RsSplitWs ws = rs_ws_carve(rem, rem_cap ? rem_cap : count);
        if (!launch_split(h, prm, ws, d_data, ds, d_par, ps, size, count, ok, corrected, s, RS_NR, ext_syn,
                          ext_stride))
            return false;
        return !own || rem_release(h->gpu, s);
    }
    const bool shared = !rem && !ext_syn; /* the handle's workspace */
    if (shared) {
        if (!ensure_rem(h, count) || !rem_acquire(h->gpu, s))
            return false;
        rem = h->gpu.rem;
        rem_cap = h->gpu.rem_cap;
    }
    const bool split = !ext_syn && !pos8 && !pos32 && prm.vfast && !prm.force_verify &&
                       h->decode_path != 2 && (h->decode_path == 1 || count >= SPLIT_MIN_COUNT);
    if (split) {
        const RsSplitWs ws = rs_ws_carve(rem, rem_cap ? rem_cap : count);
        GpuCtx &g = h->gpu;
        /* (sub-batches of 2^19 codewords, to keep a sub-batch's bytes in the
         * Infinity Cache until the apply, measured slower: 0.84 vs 0.75 ms
         * per bench step) */
        if (!launch_split(h, prm, ws, d_data, ds, d_par, ps, size, count, ok, corrected, s))
            return false;
        return !shared || rem_release(g, s);
    }
    /* erasure batches: records (64 B per codeword in ws.ext) applied
     * block-wise (scattered byte read-modify-writes cost ~0.3 ms per 2^20
     * codewords with 32 erasures).  u8 slots: rs_era_bp_k for 32 sorted
     * erasures (prim 1), the errata kernels (rs_errata.hip) for every other
     * count with or without errors, the general kernel's list for what they
     * hand on; u32 slots: the general kernel for all */
    const bool esplit = !ext_syn && (pos8 || pos32) && prm.vfast && !prm.force_verify &&
                        h->decode_path != 2 && (h->decode_path == 1 || count >= SPLIT_MIN_COUNT);
    if (esplit) {
        const RsSplitWs ws = rs_ws_carve(rem, rem_cap ? rem_cap : count);
        GpuCtx &g = h->gpu;
        const uintptr_t pa = reinterpret_cast<uintptr_t>(pos8);
        const bool efast = pos8 && prm.prim == 1u && pos_stride % 16u == 0u && (pa & 15u) == 0u;
        const bool errata = pos8 && pos_stride >= RS_NR && pos_stride % 4u == 0u && (pa & 3u) == 0u;
        if (efast || errata) {
            {
                KernelTimer t(g, POPORON_AMD_KERNEL_REMAINDER, s);
                HIP_OK(rsk_syndrome_reset(g.tab, d_data, ds, d_par, ps, (uint32_t)size, count, ws.syn, ws.nlist,
                                          g.num_cu, s));
                t.done();
            }
            if (efast) {
                KernelTimer t(g, POPORON_AMD_KERNEL_ERASURE, s);
                HIP_OK(rsk_era(g.tab, &prm, &ws, pos8, pos_stride, cnt, count, ok, corrected, errata ? 1u : 0u,
                               g.num_cu, s));
                t.done();
            }
            if (errata) {
                const uint32_t only_pend = efast ? 1u : 0u;
                {
                    KernelTimer t(g, POPORON_AMD_KERNEL_BM, s);
                    HIP_OK(rsk_ebm(g.tab, &prm, &ws, pos8, pos_stride, cnt, count, ok, corrected, only_pend, g.num_cu,
                                   s));
                    t.done();
                }
                {
                    KernelTimer t(g, POPORON_AMD_KERNEL_CHIEN, s);
                    HIP_OK(rsk_chien32(g.tab, &prm, &ws, count, ok, corrected, only_pend, g.num_cu, s));
                    t.done();
                }
                {
                    KernelTimer t(g, POPORON_AMD_KERNEL_FORNEY, s);
                    HIP_OK(rsk_forney32(g.tab, &prm, &ws, pos8, pos_stride, count, ok, corrected, only_pend,
                                        g.num_cu, s));
                    t.done();
                }
            }
            {
                /* what those hand on: one codeword per wave, in place (their
                 * meta stays RS_ST_LIST: the block apply passes them by) */
                KernelTimer t(g, POPORON_AMD_KERNEL_LIST, s);
                HIP_OK(rsk_wave(g.tab, &prm, d_data, ds, d_par, ps, count, ws.list, ws.nlist, ws.syn, nullptr, 0,
                                pos8, nullptr, pos_stride, cnt, ok, corrected, g.num_cu, s));
                t.done();
            }
        } else {
            {
                KernelTimer t(g, POPORON_AMD_KERNEL_REMAINDER, s);
                HIP_OK(rsk_syndrome(g.tab, d_data, ds, d_par, ps, (uint32_t)size, count, ws.syn, g.num_cu, s));
                t.done();
            }
            KernelTimer t(g, POPORON_AMD_KERNEL_CORRECT, s);
            HIP_OK(rsk_correct_era_rec(g.tab, &prm, count, ws.syn, pos8, pos32, pos_stride, cnt, ok, corrected, ws.ext,
                                       ws.meta, g.num_cu, s));
            t.done();
        }
        {
            KernelTimer t(g, POPORON_AMD_KERNEL_APPLY, s);
            HIP_OK(rsk_apply_era(&prm, ws.meta, ws.ext, d_data, ds, d_par, ps, count, s));
            t.done();
        }
        return !shared || rem_release(g, s);
    }
    if (!ext_syn) {
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_REMAINDER, s);
        HIP_OK(rsk_syndrome(h->gpu.tab, d_data, ds, d_par, ps, (uint32_t)size, count, rem, h->gpu.num_cu, s));
        t.done();
    }
    KernelTimer t(h->gpu, POPORON_AMD_KERNEL_CORRECT, s);
    HIP_OK(rsk_correct(h->gpu.tab, &prm, d_data, ds, d_par, ps, count, rem, ext_syn, ext_stride, pos8, pos32,
                       pos_stride, cnt, ok, corrected, h->gpu.num_cu, s));
    t.done();
    return !shared || rem_release(h->gpu, s);
}

EXPORT bool poporon_check_batch_device(poporon_t *h, const uint8_t *d_data, size_t data_stride,
                                       const uint8_t *d_parity, size_t parity_stride, size_t size, size_t count,
                                       uint8_t *d_dirty, void *stream)
{
    if (!h || (count && (!d_data || !d_parity || !d_dirty)))
        return fail("NULL argument");
    if (h->fec_type != PPLN_FEC_RS)
        return fail("poporon_check_batch_device serves RS handles");
    if (!check_decode_size(h, size))
        return fail("size %zu outside [1, %u]", size, (unsigned)kmax(h));
    if (!batch_enter(h))
        return false;
    BatchScope bsc{h->gpu, (hipStream_t)stream, false};
    DeviceGuard dg(h->gpu.device);
    hipStream_t s = (hipStream_t)stream;
    KernelTimer t(h->gpu, POPORON_AMD_KERNEL_CHECK, s);
    if (h->fast) {
        HIP_OK(rsk_check(h->gpu.tab, d_data, data_stride, d_parity, parity_stride, (uint32_t)size, count, d_dirty,
                         h->gpu.num_cu, s));
    } else if (h->nrsplit) {
        HIP_OK(rsk_check_nr(h->gpu.tab, d_data, data_stride, d_parity, parity_stride, (uint32_t)size, count, d_dirty,
                            h->rs->num_roots, h->gpu.num_cu, s));
    } else {
        RsGenParams prm = h->gen;
        prm.size = (uint32_t)size;
        if (gen_wave(h, count, false, size))
            HIP_OK(rsgw_check(h->gpu.gtab, &prm, d_data, data_stride, d_parity, parity_stride, count, d_dirty,
                              nullptr, 0, h->gpu.num_cu, s));
        else
            HIP_OK(rsg_check(h->gpu.gtab, &prm, d_data, data_stride, d_parity, parity_stride, count, d_dirty,
                             nullptr, 0, h->gpu.num_cu, s));
    }
    t.done();
    return true;
}

EXPORT bool poporon_syndrome_batch_device(poporon_t *h, const uint8_t *d_data, size_t data_stride,
                                          const uint8_t *d_parity, size_t parity_stride, size_t size, size_t count,
                                          uint16_t *d_syndromes, size_t syndrome_stride, uint8_t *d_nonzero,
                                          void *stream)
{
    if (!h || (count && (!d_data || !d_parity || (!d_syndromes && !d_nonzero))))
        return fail("NULL argument");
    if (h->fec_type != PPLN_FEC_RS)
        return fail("poporon_syndrome_batch_device serves RS handles");
    if (d_syndromes && syndrome_stride < h->rs->num_roots)
        return fail("syndrome_stride < num_roots (%u)", (unsigned)h->rs->num_roots);
    if (!check_decode_size(h, size))
        return fail("size %zu outside [1, %u]", size, (unsigned)kmax(h));
    if (!batch_enter(h))
        return false;
    BatchScope bsc{h->gpu, (hipStream_t)stream, false};
    DeviceGuard dg(h->gpu.device);
    hipStream_t s = (hipStream_t)stream;
    if (h->nrsplit) { /* fewer roots: the LFSR kernel's npar syndromes, then their logs */
        if (!ensure_rem(h, count) || !rem_acquire(h->gpu, s))
            return false;
        {
            KernelTimer t(h->gpu, POPORON_AMD_KERNEL_REMAINDER, s);
            HIP_OK(rsk_syndrome_reset_nr(h->gpu.tab, d_data, data_stride, d_parity, parity_stride, (uint32_t)size,
                                         count, h->gpu.rem, nullptr, h->rs->num_roots, h->gpu.num_cu, s));
            t.done();
        }
        HIP_OK(rsk_syn_log_nr(h->gpu.tab, h->gpu.rem, count, d_syndromes, syndrome_stride, d_nonzero,
                              h->rs->num_roots, s));
        return rem_release(h->gpu, s);
    }
    if (!h->fast) {
        RsGenParams prm = h->gen;
        prm.size = (uint32_t)size;
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_REMAINDER, s);
        if (gen_wave(h, count, false, size))
            HIP_OK(rsgw_check(h->gpu.gtab, &prm, d_data, data_stride, d_parity, parity_stride, count, d_nonzero,
                              d_syndromes, syndrome_stride, h->gpu.num_cu, s));
        else
            HIP_OK(rsg_check(h->gpu.gtab, &prm, d_data, data_stride, d_parity, parity_stride, count, d_nonzero,
                             d_syndromes, syndrome_stride, h->gpu.num_cu, s));
        t.done();
        return true;
    }
    if (!ensure_rem(h, count) || !rem_acquire(h->gpu, s))
        return false;
    {
        KernelTimer t(h->gpu, POPORON_AMD_KERNEL_REMAINDER, s);
        HIP_OK(rsk_syndrome(h->gpu.tab, d_data, data_stride, d_parity, parity_stride, (uint32_t)size, count,
                            h->gpu.rem, h->gpu.num_cu, s));
        t.done();
    }
    HIP_OK(rsk_syn_log(h->gpu.tab, h->gpu.rem, count, d_syndromes, syndrome_stride, d_nonzero, s));
    return rem_release(h->gpu, s);
}

EXPORT bool poporon_encode_batch_device(poporon_t *h, const uint8_t *d_data, size_t data_stride, uint8_t *d_parity,
                                        size_t parity_stride, size_t size, size_t count, void *stream)
{
    if (!h || (count && (!d_data || !d_parity)))
        return fail("NULL argument");
    if (!check_encode_size(h, size))
        return false;
    if (!batch_enter(h))
        return false;
    BatchScope bsc{h->gpu, (hipStream_t)stream, false};
    DeviceGuard dg(h->gpu.device);
    return launch_encode(h, d_data, data_stride, d_parity, parity_stride, size, count, (hipStream_t)stream);
}

EXPORT bool poporon_decode_batch_device(poporon_t *h, uint8_t *d_data, size_t data_stride, uint8_t *d_parity,
                                        size_t parity_stride, size_t size, size_t count, const uint8_t *d_positions,
                                        size_t positions_stride, const uint8_t *d_counts, uint8_t *d_ok,
                                        uint8_t *d_corrected, void *stream)
{
    if (!h || (count && (!d_data || !d_parity || !d_ok)))
        return fail("NULL argument");
    if (d_positions && (h->fec_type != PPLN_FEC_RS || !d_counts || positions_stride < h->rs->num_roots))
        return fail("erasure batch needs an RS handle, counts and positions_stride >= num_roots");
    if (!check_decode_size(h, size))
        return fail("decode size %zu outside [1, %u]", size, (unsigned)kmax(h));
    if (!batch_enter(h))
        return false;
    BatchScope bsc{h->gpu, (hipStream_t)stream, false};
    DeviceGuard dg(h->gpu.device);
    return launch_decode(h, d_data, data_stride, d_parity, parity_stride, size, count, nullptr, 0, d_positions,
                         nullptr, positions_stride, d_counts, d_ok, d_corrected, (hipStream_t)stream);
}

EXPORT bool poporon_decode_batch_syndrome_device(poporon_t *h, uint8_t *d_data, size_t data_stride,
                                                 uint8_t *d_parity, size_t parity_stride, size_t size, size_t count,
                                                 const uint16_t *d_syndromes, size_t syndrome_stride, uint8_t *d_ok,
                                                 uint8_t *d_corrected, void *stream)
{
    if (!h || (count && (!d_data || !d_parity || !d_ok || !d_syndromes)))
        return fail("NULL argument");
    if (h->fec_type != PPLN_FEC_RS)
        return fail("external-syndrome decode serves RS handles");
    if (syndrome_stride < h->rs->num_roots)
        return fail("syndrome_stride < num_roots (%u)", (unsigned)h->rs->num_roots);
    if (!check_decode_size(h, size))
        return fail("decode size %zu outside [1, %u]", size, (unsigned)kmax(h));
    if (!batch_enter(h))
        return false;
    BatchScope bsc{h->gpu, (hipStream_t)stream, false};
    DeviceGuard dg(h->gpu.device);
    return launch_decode(h, d_data, data_stride, d_parity, parity_stride, size, count, d_syndromes, syndrome_stride,
                         nullptr, nullptr, 0, nullptr, d_ok, d_corrected, (hipStream_t)stream);
}

/* ------------------------------------------------------------------------ */
/* host batches: staged through device memory in chunks                     */
/* ------------------------------------------------------------------------ */

/*
 * Host batches are streamed through PIPE_SLOTS slots, each with its own HIP
 * stream, pinned host buffer and device buffer.  Chunk i goes to slot
 * i % PIPE_SLOTS: its rows are gathered into pinned memory (CPU threads),
 * copied in, processed and copied back asynchronously; the slot's results are
 * scattered to the caller's arrays only when the slot is needed again (or at
 * the end).  So the CPU gather of chunk i+1, the H2D copy of chunk i+1, the
 * kernels of chunk i and the D2H copy of chunk i-1 overlap.
 */
static const size_t kPipeChunk = 1u << 18; /* codewords per chunk */

/* row copy dst[c*dw .. +w) = src[c*sw .. +w) for c < count, split over CPU threads */
static void copy_rows(uint8_t *dst, size_t dw, const uint8_t *src, size_t sw, size_t w, size_t count)
{
    auto run = [=](size_t a, size_t b) {
        if (dw == w && sw == w) {
            memcpy(dst + a * w, src + a * w, (b - a) * w);
            return;
        }
        for (size_t c = a; c < b; c++)
            memcpy(dst + c * dw, src + c * sw, w);
    };
    const size_t bytes = w * count;
    unsigned nt = std::thread::hardware_concurrency();
    nt = std::max(1u, std::min(nt, 16u));
    if (bytes < (4u << 20) || nt == 1) {
        run(0, count);
        return;
    }
    std::vector<std::thread> th;
    const size_t per = (count + nt - 1) / nt;
    for (unsigned t = 1; t < nt; t++) {
        const size_t a = std::min(count, t * per), b = std::min(count, a + per);
        if (a < b)
            th.emplace_back(run, a, b);
    }
    run(0, std::min(count, per));
    for (auto &x : th)
        x.join();
}

static bool pipe_slot(poporon_t *h, GpuCtx::PipeSlot &ps, size_t bytes)
{
    if (!ps.stream)
        HIP_OK(hipStreamCreateWithFlags(&ps.stream, hipStreamNonBlocking));
    if (!ps.done)
        HIP_OK(hipEventCreateWithFlags(&ps.done, hipEventDisableTiming));
    if (ps.cap >= bytes)
        return true;
    HIP_OK(hipStreamSynchronize(ps.stream));
    (void)hipHostFree(ps.host);
    (void)hipFree(ps.dev);
    ps.host = nullptr;
    ps.dev = nullptr;
    ps.cap = 0;
    HIP_OK(hipHostMalloc((void **)&ps.host, bytes, hipHostMallocDefault));
    HIP_OK(hipMalloc((void **)&ps.dev, bytes));
    ps.cap = bytes;
    return true;
}

/* wait for every slot (after an error: nothing may still be in flight into
 * the pinned buffers) */
static void pipe_drain(GpuCtx &g)
{
    for (auto &ps : g.pipe) {
        if (ps.stream)
            (void)hipStreamSynchronize(ps.stream);
        ps.busy = false;
    }
}

EXPORT bool poporon_encode_batch(poporon_t *h, const uint8_t *data, size_t data_stride, uint8_t *parity,
                                 size_t parity_stride, size_t size, size_t count)
{
    if (!h || (count && (!data || !parity)))
        return fail("NULL argument");
    if (!check_encode_size(h, size))
        return false;
    if (!batch_enter(h))
        return false;
    BatchScope bsc{h->gpu, nullptr, true};
    DeviceGuard dg(h->gpu.device);
    GpuCtx &g = h->gpu;
    const size_t nr = par_bytes(h);
    const size_t chunk = std::max<size_t>(1, std::min(count, kPipeChunk));
    for (auto &ps : g.pipe)
        if (!pipe_slot(h, ps, chunk * (size + nr) + 64))
            return false;
    /* parity of the slot's chunk -> caller */
    auto finish = [&](GpuCtx::PipeSlot &ps) -> bool {
        if (!ps.busy)
            return true;
        ps.busy = false;
        HIP_OK(hipEventSynchronize(ps.done));
        copy_rows(parity + ps.c0 * parity_stride, parity_stride, ps.host + ps.n * size, nr, nr, ps.n);
        return true;
    };
    bool ok = true;
    size_t i = 0;
    for (size_t c0 = 0; ok && c0 < count; c0 += chunk, i++) {
        GpuCtx::PipeSlot &ps = g.pipe[i % PIPE_SLOTS];
        if (!(ok = finish(ps)))
            break;
        const size_t n = std::min(chunk, count - c0);
        uint8_t *hd = ps.host, *dd = ps.dev, *dp = ps.dev + n * size;
        copy_rows(hd, size, data + c0 * data_stride, data_stride, size, n);
        ok = hipMemcpyAsync(dd, hd, n * size, hipMemcpyHostToDevice, ps.stream) == hipSuccess &&
             launch_encode(h, dd, size, dp, nr, size, n, ps.stream) &&
             hipMemcpyAsync(hd + n * size, dp, n * nr, hipMemcpyDeviceToHost, ps.stream) == hipSuccess &&
             hipEventRecord(ps.done, ps.stream) == hipSuccess;
        ps.busy = true;
        ps.c0 = c0;
        ps.n = n;
    }
    for (size_t k = 0; ok && k < PIPE_SLOTS; k++) /* oldest first */
        ok = finish(g.pipe[(i + k) % PIPE_SLOTS]);
    if (!ok) {
        const std::string msg = g_last_error.empty() ? std::string("HIP failure in the host pipeline") : g_last_error;
        pipe_drain(g);
        return fail("%s", msg.c_str());
    }
    return true;
}

EXPORT bool poporon_decode_batch(poporon_t *h, uint8_t *data, size_t data_stride, uint8_t *parity,
                                 size_t parity_stride, size_t size, size_t count, const uint8_t *positions,
                                 size_t positions_stride, const uint8_t *counts, uint8_t *ok, uint8_t *corrected)
{
    if (!h || (count && (!data || !parity || !ok)))
        return fail("NULL argument");
    if (positions && (h->fec_type != PPLN_FEC_RS || !counts || positions_stride < h->rs->num_roots))
        return fail("erasure batch needs an RS handle, counts and positions_stride >= num_roots");
    if (!check_decode_size(h, size))
        return fail("decode size %zu outside [1, %u]", size, (unsigned)kmax(h));
    if (!batch_enter(h))
        return false;
    BatchScope bsc{h->gpu, nullptr, true};
    DeviceGuard dg(h->gpu.device);
    GpuCtx &g = h->gpu;
    const size_t nr = par_bytes(h);
    const size_t w = size + nr;
    const size_t chunk = std::max<size_t>(1, std::min(count, kPipeChunk));
    /* slot layout: [codewords w*n | ok n | cor n | positions nr*n | counts n | decode workspace (device)] */
    const size_t per = w + 2 + (positions ? nr + 1 : 0);
    /* parity right after the data in rows of equal stride: move whole rows */
    const bool rows = parity == data + size && parity_stride == data_stride;
    for (auto &ps : g.pipe)
        if (!pipe_slot(h, ps, chunk * per + 512 + rs_ws_bytes(chunk)))
            return false;
    auto finish = [&](GpuCtx::PipeSlot &ps) -> bool {
        if (!ps.busy)
            return true;
        ps.busy = false;
        HIP_OK(hipEventSynchronize(ps.done));
        const size_t n = ps.n;
        if (rows) { /* wire layout: whole codeword rows */
            copy_rows(data + ps.c0 * data_stride, data_stride, ps.host, w, w, n);
        } else {
            copy_rows(data + ps.c0 * data_stride, data_stride, ps.host, w, size, n);
            copy_rows(parity + ps.c0 * parity_stride, parity_stride, ps.host + size, w, nr, n);
        }
        memcpy(ok + ps.c0, ps.host + n * w, n);
        if (corrected)
            memcpy(corrected + ps.c0, ps.host + n * w + n, n);
        return true;
    };
    bool good = true;
    size_t i = 0;
    for (size_t c0 = 0; good && c0 < count; c0 += chunk, i++) {
        GpuCtx::PipeSlot &ps = g.pipe[i % PIPE_SLOTS];
        if (!(good = finish(ps)))
            break;
        const size_t n = std::min(chunk, count - c0);
        uint8_t *hc = ps.host, *dc = ps.dev;
        /* positions 16-byte aligned: the 32-erasure kernel reads them as uint4 */
        const size_t o_ok = n * w, o_cor = o_ok + n, o_pos = (o_cor + n + 15) & ~(size_t)15,
                     o_cnt = o_pos + (positions ? n * nr : 0);
        const size_t o_rem = (o_cnt + (positions ? n : 0) + 255) & ~(size_t)255;
        /* codeword rows [data | parity] */
        if (rows) {
            copy_rows(hc, w, data + c0 * data_stride, data_stride, w, n);
        } else {
            copy_rows(hc, w, data + c0 * data_stride, data_stride, size, n);
            copy_rows(hc + size, w, parity + c0 * parity_stride, parity_stride, nr, n);
        }
        size_t in_bytes = n * w;
        if (positions) {
            copy_rows(hc + o_pos, nr, positions + c0 * positions_stride, positions_stride, nr, n);
            memcpy(hc + o_cnt, counts + c0, n);
        }
        good = hipMemcpyAsync(dc, hc, in_bytes, hipMemcpyHostToDevice, ps.stream) == hipSuccess &&
               (!positions || hipMemcpyAsync(dc + o_pos, hc + o_pos, n * nr + n, hipMemcpyHostToDevice,
                                             ps.stream) == hipSuccess) &&
               launch_decode(h, dc, w, dc + size, w, size, n, nullptr, 0, positions ? dc + o_pos : nullptr, nullptr,
                             nr, positions ? dc + o_cnt : nullptr, dc + o_ok, dc + o_cor, ps.stream, dc + o_rem,
                             n) &&
               hipMemcpyAsync(hc, dc, n * w + 2 * n, hipMemcpyDeviceToHost, ps.stream) == hipSuccess &&
               hipEventRecord(ps.done, ps.stream) == hipSuccess;
        ps.busy = true;
        ps.c0 = c0;
        ps.n = n;
    }
    for (size_t k = 0; good && k < PIPE_SLOTS; k++)
        good = finish(g.pipe[(i + k) % PIPE_SLOTS]);
    if (!good) {
        const std::string msg = g_last_error.empty() ? std::string("HIP failure in the host pipeline") : g_last_error;
        pipe_drain(g);
        return fail("%s", msg.c_str());
    }
    return true;
}

/* ------------------------------------------------------------------------ */
/* multi-GPU: one handle per device, contiguous codeword ranges             */
/* ------------------------------------------------------------------------ */

/*
 * Codewords are independent: a batch is split into
 * contiguous ranges, device i taking [count*i/G, count*(i+1)/G), and no data
 * crosses between devices.  Each device has its own handle (tables,
 * workspace, streams); the host entry points run one host thread per device,
 * each driving its handle's pinned pipeline over its range, so the devices'
 * PCIe links and kernels work concurrently.
 */
struct _poporon_multi_t {
    std::vector<poporon_t *> h;
};

EXPORT bool poporon_amd_multi_range(size_t count, size_t parts, size_t part, size_t *first, size_t *n)
{
    if (parts == 0 || part >= parts || !first || !n)
        return fail("bad partition arguments");
    /* 128-bit products: count * part may exceed 64 bits for huge counts */
    const size_t a = (size_t)(((unsigned __int128)count * part) / parts);
    const size_t b = (size_t)(((unsigned __int128)count * (part + 1)) / parts);
    *first = a;
    *n = b - a;
    return true;
}

EXPORT void poporon_amd_multi_destroy(poporon_multi_t *m)
{
    if (!m)
        return;
    for (auto *p : m->h)
        poporon_destroy(p);
    delete m;
}

EXPORT poporon_multi_t *poporon_amd_multi_create(const poporon_config_t *config, const int *devices,
                                                 size_t num_devices)
{
    if (!config)
        return nullptr;
    std::vector<int> devs;
    if (devices) {
        devs.assign(devices, devices + num_devices);
    } else {
        const int n = poporon_amd_device_count();
        for (int d = 0; d < n; d++)
            devs.push_back(d);
    }
    if (devs.empty()) {
        fail("no HIP device for the multi-GPU handle");
        return nullptr;
    }
    poporon_multi_t *m = new (std::nothrow) _poporon_multi_t();
    if (!m)
        return nullptr;
    /* a device may be listed more than once: its handles are independent
     * (own tables, workspace, streams and host threads) and share that GPU --
     * e.g. two host pipelines per device, or the G > 1 split exercised on a
     * one-GPU machine (tests/test_gpu_fullsize.py) */
    for (size_t i = 0; i < devs.size(); i++) {
        poporon_t *p = poporon_create(config);
        if (!p || !poporon_amd_set_device(p, devs[i]) || !gpu_init(p)) {
            const std::string msg = g_last_error;
            poporon_destroy(p);
            poporon_amd_multi_destroy(m);
            fail("device %d: %s", devs[i], msg.c_str());
            return nullptr;
        }
        m->h.push_back(p);
    }
    return m;
}

EXPORT size_t poporon_amd_multi_device_count(const poporon_multi_t *m) { return m ? m->h.size() : 0; }

EXPORT poporon_t *poporon_amd_multi_handle(poporon_multi_t *m, size_t index)
{
    return (m && index < m->h.size()) ? m->h[index] : nullptr;
}

/* run f(i, first, n) for every device's range, one host thread per device;
 * the first failure's message is kept */
template <class F>
static bool multi_run(poporon_multi_t *m, size_t count, F &&f)
{
    const size_t G = m->h.size();
    std::vector<std::string> err(G);
    std::vector<char> okv(G, 1);
    std::vector<std::thread> th;
    auto one = [&](size_t i) {
        size_t first = 0, n = 0;
        poporon_amd_multi_range(count, G, i, &first, &n);
        if (n && !f(i, first, n)) {
            okv[i] = 0;
            err[i] = g_last_error;
        }
    };
    for (size_t i = 1; i < G; i++)
        th.emplace_back(one, i);
    one(0);
    for (auto &t : th)
        t.join();
    for (size_t i = 0; i < G; i++)
        if (!okv[i])
            return fail("device %zu: %s", i, err[i].c_str());
    return true;
}

EXPORT bool poporon_encode_batch_multi(poporon_multi_t *m, const uint8_t *data, size_t data_stride, uint8_t *parity,
                                       size_t parity_stride, size_t size, size_t count)
{
    if (!m || (count && (!data || !parity)))
        return fail("NULL argument");
    return multi_run(m, count, [&](size_t i, size_t c0, size_t n) {
        return poporon_encode_batch(m->h[i], data + c0 * data_stride, data_stride, parity + c0 * parity_stride,
                                    parity_stride, size, n);
    });
}

EXPORT bool poporon_decode_batch_multi(poporon_multi_t *m, uint8_t *data, size_t data_stride, uint8_t *parity,
                                       size_t parity_stride, size_t size, size_t count, const uint8_t *positions,
                                       size_t positions_stride, const uint8_t *counts, uint8_t *ok,
                                       uint8_t *corrected)
{
    if (!m || (count && (!data || !parity || !ok)))
        return fail("NULL argument");
    return multi_run(m, count, [&](size_t i, size_t c0, size_t n) {
        return poporon_decode_batch(m->h[i], data + c0 * data_stride, data_stride, parity + c0 * parity_stride,
                                    parity_stride, size, n, positions ? positions + c0 * positions_stride : nullptr,
                                    positions_stride, counts ? counts + c0 : nullptr, ok + c0,
                                    corrected ? corrected + c0 : nullptr);
    });
}

/* Device-resident shards: device i's range (poporon_amd_multi_range) sits at
 * the i-th pointer of each array, in that device's memory; enqueued on
 * streams[i] (streams may be NULL: each device's null stream).  Returns once
 * every device's work is enqueued. */
EXPORT bool poporon_encode_batch_multi_device(poporon_multi_t *m, const uint8_t *const *d_data, size_t data_stride,
                                              uint8_t *const *d_parity, size_t parity_stride, size_t size,
                                              size_t count, void *const *streams)
{
    if (!m || (count && (!d_data || !d_parity)))
        return fail("NULL argument");
    return multi_run(m, count, [&](size_t i, size_t, size_t n) {
        return poporon_encode_batch_device(m->h[i], d_data[i], data_stride, d_parity[i], parity_stride, size, n,
                                           streams ? streams[i] : nullptr);
    });
}

EXPORT bool poporon_decode_batch_multi_device(poporon_multi_t *m, uint8_t *const *d_data, size_t data_stride,
                                              uint8_t *const *d_parity, size_t parity_stride, size_t size,
                                              size_t count, const uint8_t *const *d_positions,
                                              size_t positions_stride, const uint8_t *const *d_counts,
                                              uint8_t *const *d_ok, uint8_t *const *d_corrected, void *const *streams)
{
    if (!m || (count && (!d_data || !d_parity || !d_ok)))
        return fail("NULL argument");
    return multi_run(m, count, [&](size_t i, size_t, size_t n) {
        return poporon_decode_batch_device(m->h[i], d_data[i], data_stride, d_parity[i], parity_stride, size, n,
                                           d_positions ? d_positions[i] : nullptr, positions_stride,
                                           d_counts ? d_counts[i] : nullptr, d_ok[i],
                                           d_corrected ? d_corrected[i] : nullptr, streams ? streams[i] : nullptr);
    });
}

/* ------------------------------------------------------------------------ */
/* single-codeword API (the reference's entry points): a batch of one       */
/* ------------------------------------------------------------------------ */

/* the coherent host buffer of the single-call paths (GpuCtx::zc, layout
 * ZC_* in rs_device.h); false if the device cannot address it (then the copy
 * paths run) */
static bool ensure_zc(GpuCtx &g)
{
    if (!g.zc) {
        void *dp = nullptr;
        uint8_t *hp = nullptr;
        if (hipHostMalloc((void **)&hp, ZC_BYTES, hipHostMallocCoherent) == hipSuccess &&
            hipHostGetDevicePointer(&dp, hp, 0) == hipSuccess) {
            memset(hp, 0, ZC_BYTES);
            g.zc_dev = (uint8_t *)dp;
        } else {
            (void)hipGetLastError();
        }
        if (hp) { /* published under the registry lock: yield_servers writes other handles' buffers */
            if (g.registered) {
                std::lock_guard<std::mutex> lk(g_devs[g.device].mu);
                g.zc = hp;
            } else {
                g.zc = hp;
            }
        }
    }
    return g.zc_dev != nullptr;
}

/* Next completion word of a single-call launch (never 0), with ZC_FLAG
 * cleared first: the server answers with request words from its own counter
 * (srv_seq), so the word it left there could equal the next zc_seq and
 * zc_wait would return before this launch wrote anything */
static uint32_t zc_arm(GpuCtx &g)
{
    *reinterpret_cast<volatile uint32_t *>(g.zc + ZC_FLAG) = 0u;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    uint32_t s = ++g.zc_seq;
    if (s == 0u)
        s = ++g.zc_seq;
    return s;
}

/* Wait for a single-call kernel's completion word (it stores `seq` at
 * ZC_FLAG with a system-scope release after every result): polling host
 * memory costs the caller ~1 us after the kernel ends, a stream
 * synchronisation several.  The stream is queried now and then so that a
 * failed launch cannot leave the caller spinning. */
static bool zc_wait(GpuCtx &g, uint32_t seq)
{
    const volatile uint32_t *f = reinterpret_cast<const volatile uint32_t *>(g.zc + ZC_FLAG);
    for (uint32_t spin = 1;; ++spin) {
        if (*f == seq) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return true;
        }
        if ((spin & 4095u) == 0u) {
            const hipError_t e = hipStreamQuery(g.stream);
            if (e == hipSuccess) {
                if (*f == seq) {
                    std::atomic_thread_fence(std::memory_order_acquire);
                    return true;
                }
                return fail("single-codeword kernel ended without its completion word");
            }
            if (e != hipErrorNotReady)
                return fail("HIP error %d (%s) in a single-codeword call", (int)e, hipGetErrorString(e));
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
}

/* The single-call server (rs_serve_k, rs_single.hip): a resident workgroup
 * that polls the handle's coherent buffer, so a poporon_encode /
 * poporon_decode call is a few posted PCIe writes and reads instead of a
 * kernel launch.  It leaves by itself after SRV_IDLE_TICKS without a request
 * (so a stream or device synchronisation waits at most that long for it) or
 * SRV_MAX_TICKS in all; the next call then launches it again.
 * POPORON_AMD_SERVE=0 turns it off (one launch per call, rs_enc1_k /
 * rs_dec1_k). */
#define SRV_IDLE_TICKS 100000ull  /* 1 ms of s_memrealtime (100 MHz) */
#define SRV_MAX_TICKS 50000000ull /* 0.5 s */

static bool serve_enabled()
{
    static const bool on = [] {
        const char *e = getenv("POPORON_AMD_SERVE");
        return !(e && e[0] == '0');
    }();
    return on;
}

/* Launch a server for the handle unless a batch of another handle on the
 * device may still be running (then -1: the caller serves this request with
 * one launch); 1 launched, 0 error.  Under the registry lock, so that a
 * batch_enter either sees this server (and bumps its yield word) or is seen
 * here. */
static int srv_launch(poporon_t *h, uint32_t last)
{
    GpuCtx &g = h->gpu;
    if (!g.sstream)
        HIP_OK(hipStreamCreateWithFlags(&g.sstream, hipStreamNonBlocking));
    std::unique_lock<std::mutex> lk;
    if (g.registered)
        lk = std::unique_lock<std::mutex>(g_devs[g.device].mu);
    if (g.registered)
        for (GpuCtx *x : g_devs[g.device].ctx) {
            if (x == &g)
                continue;
            if (x->batch_open)
                return -1;
            if (x->batch_ev_live) {
                const hipError_t q = hipEventQuery(x->batch_ev);
                if (q == hipErrorNotReady)
                    return -1;
                x->batch_ev_live = false;
            }
        }
    const uint32_t yv = *reinterpret_cast<volatile uint32_t *>(g.zc + ZC_YIELD);
    const uint32_t id = g.srv_id + 1u;
    if (h->fast || h->nrsplit) {
        RsCorrParams prm = h->corr;
        HIP_OK(rsk_serve(g.tab, &prm, g.zc_dev, last, id, yv, SRV_IDLE_TICKS, SRV_MAX_TICKS, g.sstream));
    } else { /* general parameters: one wave, GZ_* payload (rs_generic.hip rsgw_serve_k) */
        RsGenParams prm = h->gen;
        HIP_OK(rsgw_serve(g.gtab, &prm, g.zc_dev, last, id, yv, SRV_IDLE_TICKS, SRV_MAX_TICKS, g.sstream));
    }
    g.srv_id = id;
    g.srv_on = true;
    return 1;
}

/* One request through the server; the payload is in g.zc already.  A server
 * that left before it saw the request (idle limit, lifetime, yield) has
 * stored its id to ZC_EXITED without serving it: launch a new one for it.
 * 1 served, 0 error, -1 not served (another handle's batch may be running,
 * srv_launch): the caller launches the request's kernel instead. */
static int srv_call(poporon_t *h, uint32_t op, uint32_t size, uint32_t mode)
{
    GpuCtx &g = h->gpu;
    volatile uint32_t *z32 = reinterpret_cast<volatile uint32_t *>(g.zc);
    /* the request word differs from the last one the server saw */
    const uint32_t prev = z32[ZC_REQ / 4], word = srv_word(g, prev, op, size, mode);
    z32[ZC_FLAG / 4] = 0u; /* the server answers with the request word (never 0: op >= 1) */
    std::atomic_thread_fence(std::memory_order_release); /* the payload before the request word */
    z32[ZC_REQ / 4] = word;
    if (!g.srv_on) {
        const int l = srv_launch(h, prev);
        if (l <= 0)
            return l; /* the request word stays unserved: the next server starts past it */
    }
    const volatile uint32_t *f = z32 + ZC_FLAG / 4, *ex = z32 + ZC_EXITED / 4;
    for (uint32_t spin = 1;; ++spin) {
        if (*f == word) {
            std::atomic_thread_fence(std::memory_order_acquire);
            return true;
        }
        if (*ex == g.srv_id) { /* the server has left */
            std::atomic_thread_fence(std::memory_order_acquire);
            if (*f == word) {
                std::atomic_thread_fence(std::memory_order_acquire);
                return true;
            }
            g.srv_on = false;
            const int l = srv_launch(h, prev);
            if (l <= 0)
                return l;
            continue;
        }
        if ((spin & 4095u) == 0u) {
            const hipError_t e = hipStreamQuery(g.sstream);
            if (e == hipSuccess && *ex != g.srv_id && *f != word) {
                g.srv_on = false;
                return fail("single-call server ended without serving or leaving its exit word");
            }
            if (e != hipSuccess && e != hipErrorNotReady) {
                g.srv_on = false;
                return fail("HIP error %d (%s) in the single-call server", (int)e, hipGetErrorString(e));
            }
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
}

/* A live server of this handle leaves now (a stop request, then its exit
 * word: one PCIe round trip).  Batch calls come here first (batch_enter): a
 * resident server holds one CU's LDS, so one workgroup of a persistent batch
 * grid would wait for its idle limit, and with GPU_MAX_HW_QUEUES below the
 * streams in use its dispatch can share a hardware queue with the batch's.
 * The next single call launches a new server. */
#define SRV_STOP_DEADLINE_S 10
static bool srv_stop(poporon_t *h)
{
    GpuCtx &g = h->gpu;
    if (!g.srv_on || !g.zc)
        return true;
    volatile uint32_t *z32 = reinterpret_cast<volatile uint32_t *>(g.zc);
    const uint32_t prev = z32[ZC_REQ / 4];
    std::atomic_thread_fence(std::memory_order_release);
    z32[ZC_REQ / 4] = srv_word(g, prev, RS_SRV_STOP, 0u, 0u);
    const volatile uint32_t *ex = z32 + ZC_EXITED / 4;
    /* a queued server sees the stop request as soon as it runs; past
     * SRV_STOP_DEADLINE_S (the GPU busy with other work for that long, or
     * hung) the batch call fails instead of spinning on */
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 1; *ex != g.srv_id; ++spin) {
        if ((spin & 4095u) == 0u) {
            const hipError_t e = hipStreamQuery(g.sstream);
            if (e == hipSuccess && *ex != g.srv_id) {
                g.srv_on = false;
                return fail("single-call server ended without its exit word");
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(SRV_STOP_DEADLINE_S))
                return fail("single-call server did not leave within %d s of a stop request", SRV_STOP_DEADLINE_S);
            if (e != hipSuccess && e != hipErrorNotReady) {
                g.srv_on = false;
                return fail("HIP error %d (%s) in the single-call server", (int)e, hipGetErrorString(e));
            }
        }
#if defined(__x86_64__)
        __builtin_ia32_pause();
#endif
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    g.srv_on = false;
    return true;
}

EXPORT bool poporon_encode(poporon_t *h, uint8_t *data, size_t size, uint8_t *parity)
{
    if (!h || !data || !parity)
        return false;
    if (h->fec_type == PPLN_FEC_BCH && size < h->bch.dbytes) /* src/encode.c:210-212 */
        return false;
    if (h->fec_type != PPLN_FEC_RS && h->fec_type != PPLN_FEC_BCH)
        return false;
    if (size > 65535) /* the reference's uint16 counter loops forever here (quirk Q7) */
        return fail("size %zu > 65535", size);
    if (!gpu_init(h))
        return false;
    DeviceGuard dg(h->gpu.device);
    GpuCtx &g = h->gpu;
    const size_t nr = par_bytes(h);
    /* one RS codeword: rs_enc1_k reads the message from and writes the parity
     * to coherent host memory and signals its completion word there (one
     * launch, no copies, no stream synchronisation) */
    /* (codes with fewer roots, h->nrsplit, the same way: their encq rows, P.nr) */
    if (h->fec_type == PPLN_FEC_RS && (h->fast || h->nrsplit) && size >= 1 && size <= kmax(h) && ensure_zc(g)) {
        memcpy(g.zc + ZC_DATA, data, size);
        const int sv = serve_enabled() && !g.timing ? srv_call(h, RS_SRV_ENCODE, (uint32_t)size, 0u) : -1;
        if (sv == 0)
            return false;
        if (sv < 0) {
            const uint32_t seq = zc_arm(g);
            KernelTimer t(g, POPORON_AMD_KERNEL_ENCODE, g.stream);
            HIP_OK(rsk_encode1_nr(g.tab, g.zc_dev + ZC_DATA, g.zc_dev + ZC_PAR, (uint32_t)size, (uint32_t)nr,
                                  reinterpret_cast<uint32_t *>(g.zc_dev + ZC_FLAG), seq, g.stream));
            t.done();
            if (!zc_wait(g, seq))
                return false;
        }
        memcpy(parity, g.zc + ZC_PAR, nr);
        return true;
    }
    /* general parameters: rsgw_encode_k on coherent host memory, the same way */
    if (h->fec_type == PPLN_FEC_RS && h->generic && gen_wave(h, 1, true, size) && ensure_zc(g)) {
        memcpy(g.zc + GZ_DATA, data, size);
        const int sv = serve_enabled() && !g.timing ? srv_call(h, RS_SRV_ENCODE, (uint32_t)size, 0u) : -1;
        if (sv == 0)
            return false;
        if (sv < 0) {
            RsGenParams prm = h->gen;
            prm.size = (uint32_t)size;
            const uint32_t seq = zc_arm(g);
            KernelTimer t(g, POPORON_AMD_KERNEL_ENCODE, g.stream);
            HIP_OK(rsgw_encode(g.gtab, &prm, g.zc_dev + GZ_DATA, size, g.zc_dev + GZ_PAR, nr, 1,
                               reinterpret_cast<uint32_t *>(g.zc_dev + ZC_FLAG), seq, g.num_cu, g.stream));
            t.done();
            if (!zc_wait(g, seq))
                return false;
        }
        memcpy(parity, g.zc + GZ_PAR, nr);
        return true;
    }
    const size_t off_p = (size + 15) & ~(size_t)15;
    if (!ensure_stage(h, off_p + nr + 16))
        return false;
    /* pinned mirror: one H2D copy in, one D2H copy out */
    if (size) {
        memcpy(g.hstage, data, size);
        HIP_OK(hipMemcpyAsync(g.stage, g.hstage, size, hipMemcpyHostToDevice, g.stream));
    }
    if (!launch_encode(h, g.stage, size, g.stage + off_p, nr, size, 1, g.stream))
        return false;
    HIP_OK(hipMemcpyAsync(g.hstage + off_p, g.stage + off_p, nr, hipMemcpyDeviceToHost, g.stream));
    HIP_OK(hipStreamSynchronize(g.stream));
    memcpy(parity, g.hstage + off_p, nr);
    return true;
}

/* src/decode.c:542-590: data bytes and corrected_num are written on success only */
static bool bch_decode_one(poporon_t *h, uint8_t *data, size_t size, uint8_t *parity, size_t *corrected_num)
{
    if (size < h->bch.dbytes)
        return false;
    if (!gpu_init(h))
        return false;
    DeviceGuard dg(h->gpu.device);
    GpuCtx &g = h->gpu;
    const size_t db = h->bch.dbytes, pb = h->bch.pbytes;
    if (!ensure_stage(h, db + pb + 2 + 16))
        return false;
    uint8_t *dd = g.stage, *dp = g.stage + db, *dok = dp + pb;
    if (db)
        HIP_OK(hipMemcpyAsync(dd, data, db, hipMemcpyHostToDevice, g.stream));
    if (pb)
        HIP_OK(hipMemcpyAsync(dp, parity, pb, hipMemcpyHostToDevice, g.stream));
    if (!launch_decode(h, dd, db, dp, pb, db, 1, nullptr, 0, nullptr, nullptr, 0, nullptr, dok, dok + 1, g.stream))
        return false;
    uint8_t res[2];
    uint8_t out[4];
    HIP_OK(hipMemcpyAsync(res, dok, 2, hipMemcpyDeviceToHost, g.stream));
    if (db)
        HIP_OK(hipMemcpyAsync(out, dd, db, hipMemcpyDeviceToHost, g.stream));
    HIP_OK(hipStreamSynchronize(g.stream));
    if (!res[0])
        return false;
    memcpy(data, out, db);
    if (corrected_num)
        *corrected_num = res[1];
    return true;
}

/* One RS codeword on the device: false only for a device-side failure (no
 * usable GPU, a HIP error); the decode outcome goes to *success / *fixed. */
static bool rs_decode_one(poporon_t *h, uint8_t *data, size_t size, uint8_t *parity, bool *success_out,
                          size_t *fixed_out)
{
    size_t fixed = 0;
    bool success = false;
    if (!gpu_init(h))
        return false;
    {
        DeviceGuard dg(h->gpu.device);
        GpuCtx &g = h->gpu;
        const size_t nr = h->rs->num_roots;
        if ((h->fast || h->nrsplit) && ensure_zc(g)) {
            /* rs_dec1_k: the whole decode of one codeword in one launch, reading
             * the codeword, the erasure slots or the external syndromes from
             * coherent host memory and writing back the corrected bytes, ok and
             * corrected_num, then its completion word */
            uint8_t *z = g.zc;
            memcpy(z + ZC_DATA, data, size);
            memcpy(z + ZC_PAR, parity, nr);
            uint32_t mode = 0;
            if (h->ext_syndrome) {
                mode = 2; /* values > 255 are refused by the kernel (out-of-table in the reference) */
                memcpy(z + ZC_EXT, h->ext_syndrome, nr * sizeof(uint16_t));
            } else if (h->erasure) {
                mode = 1;
                const poporon_erasure_t *e = h->erasure;
                /* the reference reads slots by root ordinal (quirks Q2/Q3): nr
                 * slots, those past the list's capacity read as 0; the count as
                 * it is (past num_roots: refused for a dirty codeword, Q5) */
                uint32_t *pos = reinterpret_cast<uint32_t *>(z + ZC_POS);
                const size_t have = std::min<size_t>(e->capacity, nr);
                memcpy(pos, e->erasure_positions, have * sizeof(uint32_t));
                memset(pos + have, 0, (nr - have) * sizeof(uint32_t));
                *reinterpret_cast<uint32_t *>(z + ZC_CNT) = e->erasure_count;
            }
            RsCorrParams prm = h->corr;
            prm.size = (uint32_t)size;
            prm.pad = (int32_t)(h->rs->gf->field_size - h->rs->num_roots - size);
            uint8_t *zd = g.zc_dev;
            const int sv = serve_enabled() && !g.timing && prm.pad == (int32_t)(RS_NN - nr - size)
                               ? srv_call(h, RS_SRV_DECODE, (uint32_t)size, mode)
                               : -1;
            if (sv == 0)
                return false;
            if (sv < 0) {
                const uint32_t seq = zc_arm(g);
                KernelTimer t(g, POPORON_AMD_KERNEL_SINGLE, g.stream);
                HIP_OK(rsk_decode1(g.tab, &prm, mode, zd + ZC_DATA, zd + ZC_PAR, nullptr,
                                   reinterpret_cast<const uint32_t *>(zd + ZC_POS), zd + ZC_CNT, 4u,
                                   reinterpret_cast<const uint16_t *>(zd + ZC_EXT), zd + ZC_OK, zd + ZC_COR,
                                   reinterpret_cast<uint32_t *>(zd + ZC_FLAG), seq, g.stream));
                t.done();
                if (!zc_wait(g, seq))
                    return false;
            }
            memcpy(data, z + ZC_DATA, size);
            memcpy(parity, z + ZC_PAR, nr);
            success = z[ZC_OK] != 0;
            fixed = z[ZC_COR];
        } else if (gen_wave(h, 1, false, size) && ensure_zc(g)) {
            /* general parameters, one wave (rsgw_decode_k): the row, the slots
             * or the external syndromes read from coherent host memory, the
             * corrected bytes, ok and corrected_num written back there, then
             * the completion word (no copies, no stream synchronisation) */
            const uint32_t nn = h->rs->gf->field_size;
            uint8_t *z = g.zc, *zd = g.zc_dev;
            memcpy(z + GZ_DATA, data, size);
            memcpy(z + GZ_PAR, parity, nr);
            const uint16_t *ext = nullptr;
            const uint32_t *pos32 = nullptr;
            const uint8_t *cnt = nullptr;
            bool refuse = false;
            if (h->ext_syndrome) {
                for (size_t i = 0; i < nr; i++)
                    refuse |= h->ext_syndrome[i] > nn; /* out-of-table index in the reference */
                memcpy(z + GZ_EXT, h->ext_syndrome, nr * sizeof(uint16_t));
                ext = reinterpret_cast<const uint16_t *>(zd + GZ_EXT);
            } else if (h->erasure) {
                const poporon_erasure_t *e = h->erasure;
                uint32_t *pos = reinterpret_cast<uint32_t *>(z + GZ_POS);
                const size_t have = std::min<size_t>(e->capacity, nr); /* stale slots read as the reference (Q2/Q3) */
                memcpy(pos, e->erasure_positions, have * sizeof(uint32_t));
                memset(pos + have, 0, (nr - have) * sizeof(uint32_t));
                z[GZ_CNT] = (uint8_t)std::min<uint32_t>(e->erasure_count, 255u); /* past nr: refused if dirty (Q5) */
                pos32 = reinterpret_cast<const uint32_t *>(zd + GZ_POS);
                cnt = zd + GZ_CNT;
            }
            if (refuse) {
                fail("external syndrome > field size: undefined in the reference, refused");
            } else {
                const int sv = serve_enabled() && !g.timing
                                   ? srv_call(h, RS_SRV_DECODE, (uint32_t)size, ext ? 2u : pos32 ? 1u : 0u)
                                   : -1;
                if (sv == 0)
                    return false;
                if (sv < 0) {
                    RsGenParams prm = h->gen;
                    prm.size = (uint32_t)size;
                    prm.pad = (int32_t)(nn - nr - size);
                    const uint32_t seq = zc_arm(g);
                    KernelTimer t(g, POPORON_AMD_KERNEL_CORRECT, g.stream);
                    HIP_OK(rsgw_decode(g.gtab, &prm, zd + GZ_DATA, size, zd + GZ_PAR, nr, 1, ext, nr, nullptr, pos32,
                                       nr, cnt, zd + GZ_OK, zd + GZ_COR, nullptr, nullptr,
                                       reinterpret_cast<uint32_t *>(zd + ZC_FLAG), seq, g.num_cu, g.stream));
                    t.done();
                    if (!zc_wait(g, seq))
                        return false;
                }
                memcpy(data, z + GZ_DATA, size);
                memcpy(parity, z + GZ_PAR, nr);
                success = z[GZ_OK] != 0;
                fixed = z[GZ_COR];
            }
        } else {
            /* general parameters (rs_generic.hip): everything through the pinned
             * mirror, one H2D copy of [data | parity | ok | cor | pad | syndromes
             * (nr x u16) or slots (nr x u32) + count], the kernel, one D2H copy of
             * [data | parity | ok | cor] */
            const size_t off_p = size, off_ok = size + nr, off_cor = off_ok + 1;
            const size_t off_x = (off_cor + 1 + 15) & ~(size_t)15;
            if (!ensure_stage(h, off_x + nr * 4 + 16))
                return false;
            uint8_t *hs = g.hstage;
            const uint16_t *ext = nullptr;
            const uint32_t *pos32 = nullptr;
            const uint8_t *pos8 = nullptr;
            const uint8_t *cnt = nullptr;
            bool refuse = false;
            size_t in_bytes = off_cor + 1;
            memcpy(hs, data, size);
            memcpy(hs + off_p, parity, nr);
            if (h->ext_syndrome) {
                for (size_t i = 0; i < nr; i++)
                    refuse |= h->ext_syndrome[i] > h->rs->gf->field_size; /* out-of-table index in the reference */
                memcpy(hs + off_x, h->ext_syndrome, nr * sizeof(uint16_t));
                in_bytes = off_x + nr * sizeof(uint16_t);
                ext = (const uint16_t *)(g.stage + off_x);
            } else if (h->erasure) {
                const poporon_erasure_t *e = h->erasure;
                memset(hs + off_x, 0, nr * 4);
                memcpy(hs + off_x, e->erasure_positions, std::min<size_t>(e->capacity, nr) * sizeof(uint32_t));
                /* counts past num_roots (quirk Q5) reach the kernel clamped to 255:
                 * refused there only for a dirty codeword */
                hs[off_x + nr * 4] = (uint8_t)std::min<uint32_t>(e->erasure_count, 255u);
                in_bytes = off_x + nr * 4 + 1;
                pos32 = (const uint32_t *)(g.stage + off_x);
                cnt = g.stage + off_x + nr * 4;
                /* a fewer-roots code whose nr slots (the count's and the stale
                 * ones the reference reads, Q2) all fit a byte below 255: u8
                 * slots, so the errata kernels take it (launch_decode) */
                const uint32_t *pv = reinterpret_cast<const uint32_t *>(hs + off_x);
                bool small = h->nrsplit;
                for (size_t i = 0; i < nr && small; i++)
                    small = pv[i] < 255u;
                if (small) {
                    uint8_t sl[RS_NR];
                    for (size_t i = 0; i < nr; i++)
                        sl[i] = (uint8_t)pv[i];
                    memset(hs + off_x, 0, nr * 4);
                    memcpy(hs + off_x, sl, nr); /* a row of nr u8 slots, 4-byte aligned, stride nr * 4 */
                    pos32 = nullptr;
                    pos8 = g.stage + off_x;
                }
            }
            if (refuse) {
                fail("external syndrome > field size: undefined in the reference, refused");
            } else {
                HIP_OK(hipMemcpyAsync(g.stage, hs, in_bytes, hipMemcpyHostToDevice, g.stream));
                if (!launch_decode(h, g.stage, size, g.stage + off_p, nr, size, 1, ext, nr, pos8, pos32,
                                   pos8 ? nr * 4 : nr, cnt, g.stage + off_ok, g.stage + off_cor, g.stream))
                    return false;
                HIP_OK(hipMemcpyAsync(hs, g.stage, off_cor + 1, hipMemcpyDeviceToHost, g.stream));
                HIP_OK(hipStreamSynchronize(g.stream));
                memcpy(data, hs, size);
                memcpy(parity, hs + off_p, nr);
                success = hs[off_ok] != 0;
                fixed = hs[off_cor];
            }
        }
    }
    *success_out = success;
    *fixed_out = fixed;
    return true;
}

EXPORT bool poporon_decode(poporon_t *h, uint8_t *data, size_t size, uint8_t *parity, size_t *corrected_num)
{
    if (!h || !data || !parity || !size)
        return false;
    if (h->fec_type == PPLN_FEC_BCH)
        return bch_decode_one(h, data, size, parity, corrected_num);
    if (h->fec_type != PPLN_FEC_RS)
        return false;
    size_t fixed = 0;
    bool success = false;
    if (check_decode_size(h, size) && !rs_decode_one(h, data, size, parity, &success, &fixed)) {
        /* no usable device / a HIP failure: not a decode outcome.  The
         * reference never reports more than num_roots corrections, so the
         * sentinel tells this apart from "uncorrectable" (false, count 0..32);
         * poporon_amd_last_error() says what failed */
        h->last_corrected = POPORON_AMD_DEVICE_ERROR;
        if (corrected_num)
            *corrected_num = POPORON_AMD_DEVICE_ERROR;
        return false;
    }
    h->last_corrected = fixed;
    if (corrected_num)
        *corrected_num = fixed;
    return success;
}
