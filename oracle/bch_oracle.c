/*
 * bch_oracle.c -- CPU restatement of libpoporon's binary BCH codec.
 *
 * TEST INFRASTRUCTURE ONLY (see rs_oracle.h for the rules).  Restates, for
 * codewords that fit a uint32 (codeword length 2^m - 1 <= 31):
 *   generator from minimal polynomials   src/bch.c:184-285
 *   encode (systematic, binary division) src/bch.c:359-384
 *   decode (syndromes, BM, Chien, check) src/bch.c:25-165, :386-436
 *   byte packing of poporon_encode/decode src/encode.c:199-233,
 *                                         src/decode.c:542-590
 * Parity status: pinned by tests/golden/bch_golden.npz (tools/gen_golden_bch.py,
 * from the compiled reference) and, where oracle/_ref exists, checked against
 * the reference directly.
 */
#include <string.h>

#include "rs_oracle.h"

#define BCH_POLY 64 /* BCH_MAX_POLY, src/bch.c:12 */
#define BCH_T 16    /* BCH_MAX_T */

struct oracle_bch_s {
    uint32_t m, nn;        /* nn = 2^m - 1 (field size, also the codeword length) */
    uint32_t t;            /* correction capability */
    uint32_t k, pbits;     /* data bits, parity bits */
    uint32_t gen, gdeg;    /* binary generator */
    uint16_t alog[65536], log[65536];
};

size_t oracle_bch_sizeof(void) { return sizeof(oracle_bch_t); }

/* minimal polynomial of alpha^e as a binary word: product of (x + alpha^c)
 * over the conjugates c = e, 2e, 4e, ... (src/bch.c:184-220) */
static uint32_t min_poly(const oracle_bch_t *b, uint32_t e)
{
    uint16_t p[BCH_POLY];
    uint32_t deg = 0, c = e, out = 0, i;
    int j;
    memset(p, 0, sizeof(p));
    p[0] = 1;
    do {
        const uint16_t root = b->alog[c];
        for (j = (int)deg; j >= 0; j--) {
            if (j + 1 < BCH_POLY)
                p[j + 1] ^= p[j];
            p[j] = (p[j] && root) ? b->alog[(b->log[p[j]] + b->log[root]) % b->nn] : 0;
        }
        deg++;
        c = (c * 2) % b->nn;
    } while (c != e);
    for (i = 0; i <= deg; i++)
        if (p[i] == 1)
            out |= 1u << i;
    return out;
}

static int deg_binary(uint32_t v)
{
    int i;
    if (!v)
        return -1;
    for (i = 31; i >= 0; i--)
        if (v & (1u << i))
            return i;
    return 0;
}

/* Returns 0 on success, -1 where poporon_bch_create returns NULL, -2 for
 * parameters it accepts but whose codewords do not fit 31 bits. */
int oracle_bch_init(oracle_bch_t *b, uint8_t m, uint16_t poly, uint8_t t)
{
    uint32_t i, v, gen = 1, gdeg = 0;
    uint8_t used[65536];
    if (m < 3 || m > 16 || t < 1 || t > BCH_T)
        return -1;
    memset(b, 0, sizeof(*b));
    b->m = m;
    b->nn = (uint8_t)((1u << m) - 1); /* uint8 field_size, as the GF struct */
    b->t = t;
    b->log[0] = (uint16_t)b->nn;
    b->alog[b->nn] = 0;
    v = 1;
    for (i = 0; i < b->nn; i++) {
        b->log[v] = (uint16_t)i;
        b->alog[i] = (uint16_t)v;
        v <<= 1;
        if (v & (1u << m))
            v ^= poly;
        v &= b->nn;
    }
    if (v != 1)
        return -1;
    if (m > 5)
        return -2;
    memset(used, 0, sizeof(used));
    for (i = 1; i <= 2u * t; i++) { /* src/bch.c:241-262 */
        const uint32_t e = i % b->nn;
        uint32_t c = e, mp, j, prod = 0;
        if (used[e])
            continue;
        do {
            used[c] = 1;
            c = (c * 2) % b->nn;
        } while (c != e);
        mp = min_poly(b, e);
        for (j = 0; j <= gdeg; j++)
            if (gen & (1u << j))
                prod ^= mp << j;
        gen = prod;
        gdeg = (uint32_t)deg_binary(gen);
    }
    b->gen = gen;
    b->gdeg = gdeg;
    b->pbits = gdeg;
    b->k = b->nn - gdeg;
    return 0;
}

uint32_t oracle_bch_data_bits(const oracle_bch_t *b) { return b->k; }
uint32_t oracle_bch_parity_bits(const oracle_bch_t *b) { return b->pbits; }

/* src/bch.c:359-384 */
uint32_t oracle_bch_encode_word(const oracle_bch_t *b, uint32_t data)
{
    const uint32_t sh = data << b->pbits;
    uint32_t r = sh;
    int i;
    for (i = (int)b->nn - 1; i >= (int)b->gdeg; i--)
        if (r & (1u << i))
            r ^= b->gen << (i - (int)b->gdeg);
    return sh ^ r;
}

/* src/bch.c:25-50 */
static int syndromes(const oracle_bch_t *b, uint32_t cw, uint16_t *s)
{
    uint32_t i, j;
    int nz = 0;
    for (i = 0; i < 2 * b->t; i++) {
        s[i] = 0;
        for (j = 0; j < b->nn; j++)
            if (cw & (1u << j))
                s[i] ^= b->alog[((i + 1) * j) % b->nn];
        nz |= s[i] != 0;
    }
    return nz;
}

/* src/bch.c:52-75 */
static uint16_t poly_eval(const oracle_bch_t *b, const uint16_t *p, int deg, uint16_t x)
{
    uint16_t sum = 0, lx;
    int i;
    if (x == 0)
        return p[0];
    lx = b->log[x];
    for (i = 0; i <= deg; i++)
        if (p[i])
            sum ^= b->alog[(b->log[p[i]] + (lx * (uint32_t)i) % b->nn) % b->nn];
    return sum;
}

/* src/bch.c:77-141: returns the final error count; loc gets the locator */
static int berlekamp(const oracle_bch_t *b, const uint16_t *s, uint16_t *loc)
{
    uint16_t cur[BCH_POLY], prev[BCH_POLY], tmp[BCH_POLY], pd = 1, d;
    int ec = 0, shift = 1, it, i;
    memset(cur, 0, sizeof(cur));
    memset(prev, 0, sizeof(prev));
    cur[0] = prev[0] = 1;
    for (it = 0; it < (int)(2 * b->t); it++) {
        d = s[it];
        for (i = 1; i <= ec; i++)
            if (cur[i] && s[it - i])
                d ^= b->alog[(b->log[cur[i]] + b->log[s[it - i]]) % b->nn];
        if (d == 0) {
            shift++;
            continue;
        }
        {
            const uint16_t mult = b->alog[(b->nn - b->log[pd] + b->log[d]) % b->nn];
            const int grow = 2 * ec <= it;
            if (grow)
                memcpy(tmp, cur, sizeof(tmp));
            for (i = 0; i < BCH_POLY - shift; i++)
                if (prev[i])
                    cur[i + shift] ^= b->alog[(b->log[prev[i]] + b->log[mult]) % b->nn];
            if (grow) {
                memcpy(prev, tmp, sizeof(prev));
                ec = it + 1 - ec;
                pd = d;
                shift = 1;
            } else {
                shift++;
            }
        }
    }
    memcpy(loc, cur, sizeof(cur));
    return ec;
}

/* src/bch.c:386-436.  Returns 1/0; *out = corrected word (received on failure),
 * *nerr = errors fixed (0 on failure). */
int oracle_bch_decode_word(const oracle_bch_t *b, uint32_t rx, uint32_t *out, int32_t *nerr)
{
    uint16_t s[BCH_POLY], loc[BCH_POLY], pos[BCH_T];
    int ec, found = 0, i;
    uint32_t fixed;
    rx &= (1u << b->nn) - 1u;
    *out = rx;
    *nerr = 0;
    memset(s, 0, sizeof(s));
    if (!syndromes(b, rx, s))
        return 1;
    ec = berlekamp(b, s, loc);
    if (ec > (int)b->t)
        return 0;
    for (i = 0; i < (int)b->nn; i++) { /* Chien, src/bch.c:143-165 */
        const uint16_t ainv = b->alog[(b->nn - (uint32_t)i) % b->nn];
        if (poly_eval(b, loc, ec, ainv) == 0) {
            pos[found++] = (uint16_t)i;
            if (found >= ec)
                break;
        }
    }
    if (found != ec)
        return 0;
    fixed = rx;
    for (i = 0; i < found; i++)
        fixed ^= 1u << pos[i];
    if (syndromes(b, fixed, s))
        return 0;
    *out = fixed;
    *nerr = found;
    return 1;
}

/* poporon_encode for BCH (src/encode.c:199-233): big-endian data bytes in,
 * big-endian parity bytes out.  Returns 1/0. */
int oracle_bch_encode(const oracle_bch_t *b, const uint8_t *data, size_t size, uint8_t *parity)
{
    const uint32_t db = (b->k + 7) / 8, pb = (b->pbits + 7) / 8;
    uint32_t dv = 0, cw, pv, i;
    if (size < db)
        return 0;
    for (i = 0; i < db && i < 4; i++)
        dv |= (uint32_t)data[i] << (8 * (db - 1 - i));
    if (b->k < 32)
        dv &= (1u << b->k) - 1u;
    cw = oracle_bch_encode_word(b, dv);
    pv = cw & ((1u << b->pbits) - 1u);
    memset(parity, 0, pb);
    for (i = 0; i < pb && i < 4; i++)
        parity[pb - 1 - i] = (uint8_t)(pv >> (8 * i));
    return 1;
}

/* poporon_decode for BCH (src/decode.c:542-590): data bytes rewritten on
 * success only; *corrected written on success only (as the reference). */
int oracle_bch_decode(const oracle_bch_t *b, uint8_t *data, size_t size, const uint8_t *parity, size_t *corrected)
{
    const uint32_t db = (b->k + 7) / 8, pb = (b->pbits + 7) / 8;
    uint32_t dv = 0, pv = 0, out, cd, i;
    int32_t ne;
    if (size < db || size == 0)
        return 0;
    for (i = 0; i < db && i < 4; i++)
        dv |= (uint32_t)data[i] << (8 * (db - 1 - i));
    if (b->k < 32)
        dv &= (1u << b->k) - 1u;
    for (i = 0; i < pb && i < 4; i++)
        pv |= (uint32_t)parity[i] << (8 * (pb - 1 - i));
    if (b->pbits < 32)
        pv &= (1u << b->pbits) - 1u;
    if (!oracle_bch_decode_word(b, (dv << b->pbits) | pv, &out, &ne))
        return 0;
    cd = (out >> b->pbits) & ((1u << b->k) - 1u);
    for (i = 0; i < db && i < 4; i++)
        data[db - 1 - i] = (uint8_t)(cd >> (8 * i));
    if (corrected)
        *corrected = ne > 0 ? (size_t)ne : 0;
    return 1;
}
