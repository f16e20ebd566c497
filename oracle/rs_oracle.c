/*
 * rs_oracle.c -- CPU restatement of libpoporon's RS(n,k) path over GF(2^m).
 *
 * TEST INFRASTRUCTURE ONLY (see rs_oracle.h).  Written from the behavioural
 * description in SURVEY.md Appendix A and a reading of the reference; nothing
 * here is linked into libpoporon_amd.  Integer widths are chosen to reproduce
 * the reference's truncations (uint8 field_size, uint16 gf_mod argument,
 * int16 loop/location variables) so that even the out-of-capacity behaviour
 * (miscorrections, failure points, corrected_num on failure) matches.
 */
#include "rs_oracle.h"

#include <pthread.h>
#include <string.h>

size_t oracle_rs_sizeof(void) { return sizeof(oracle_rs_t); }

/* src/internal/common.h:102-110: fold v modulo 2^m-1; the argument is a
 * uint16 and the result a uint8 in the reference. */
uint16_t oracle_gf_mod(const oracle_rs_t *rs, uint32_t v)
{
    uint16_t x = (uint16_t)v;
    const uint8_t fs = (uint8_t)rs->nn;
    while (x >= fs) {
        x = (uint16_t)(x - fs);
        x = (uint16_t)((x >> rs->m) + (x & fs));
    }
    return (uint8_t)x;
}

#define MOD(v) oracle_gf_mod(rs, (uint32_t)(v))

/* src/gf.c:29-86 (tables), src/rs.c:29-82 (generator), src/poporon.c:78-93
 * (primitive inverse). */
int oracle_rs_init(oracle_rs_t *rs, uint8_t m, uint16_t gfpoly, uint16_t fcr, uint16_t prim, uint16_t nroots)
{
    uint16_t e, v, step, root;
    uint32_t tries;
    uint16_t g[ORACLE_MAX_ROOTS + 1];

    if (m < 1 || m > 16 || nroots > ORACLE_MAX_ROOTS)
        return -1;
    memset(rs, 0, sizeof(*rs));
    rs->m = m;
    rs->nn = (uint8_t)((1u << m) - 1); /* struct field is uint8_t */
    rs->gfpoly = gfpoly;
    rs->fcr = fcr;
    rs->prim = prim;
    rs->nroots = nroots;

    /* antilog / log tables: walk the powers of x modulo gfpoly */
    rs->log[0] = rs->nn;
    rs->alog[rs->nn] = 0;
    v = 1;
    for (step = 0; step < (uint8_t)rs->nn; step++) {
        rs->log[v] = step;
        rs->alog[step] = v;
        v = (uint16_t)(v << 1);
        if (v & (1u << m))
            v ^= gfpoly;
        v &= (uint8_t)rs->nn;
    }
    if (v != rs->alog[0])
        return -1; /* gfpoly not primitive */

    /* generator: product of (x - alpha^(prim*(fcr+i))), built in place */
    g[0] = 1;
    root = (uint16_t)(fcr * prim);
    for (step = 0; step < nroots; step++, root = (uint16_t)(root + prim)) {
        g[step + 1] = 1;
        for (e = step; e > 0; e--)
            g[e] = g[e] ? (uint16_t)(g[e - 1] ^ rs->alog[MOD(rs->log[g[e]] + root)]) : g[e - 1];
        g[0] = rs->alog[MOD(rs->log[g[0]] + root)];
    }
    for (step = 0; step <= nroots; step++)
        rs->genpoly[step] = rs->log[g[step]];

    /* smallest 1 + j*nn (uint16 arithmetic) divisible by prim, over prim */
    if (prim == 0)
        return -1;
    tries = 0;
    for (v = 1; (v % prim) != 0; v = (uint16_t)(v + (uint8_t)rs->nn))
        if (++tries > (uint32_t)(uint8_t)rs->nn * 2)
            return -1;
    rs->iprim = (uint16_t)(v / prim);
    return 0;
}

/* src/encode.c:120-143: systematic LFSR, parity[0] is the highest-degree
 * remainder coefficient.  The reference's uint16 byte counter never
 * terminates for size > 65535; the restatement stops there instead. */
void oracle_rs_encode(const oracle_rs_t *rs, const uint8_t *data, size_t size, uint8_t *parity)
{
    const uint16_t nr = rs->nroots, A0 = (uint8_t)rs->nn;
    size_t b;
    uint16_t t, fb;

    memset(parity, 0, nr);
    if (size > 65535)
        size = 65535;
    for (b = 0; b < size; b++) {
        fb = rs->log[(uint16_t)((data[b] & A0) ^ parity[0])];
        if (fb != A0)
            for (t = 1; t < nr; t++)
                parity[t] ^= (uint8_t)rs->alog[MOD(fb + rs->genpoly[nr - t])];
        memmove(parity, parity + 1, (size_t)(nr - 1));
        parity[nr - 1] = (fb != A0) ? (uint8_t)rs->alog[MOD(fb + rs->genpoly[0])] : 0;
    }
}

/* src/decode.c:375-415: Horner per root over data then parity; a zero
 * accumulator skips the multiply.  Output in log form. */
int oracle_rs_syndrome(const oracle_rs_t *rs, const uint8_t *data, size_t size, const uint8_t *parity,
                       uint16_t *syn)
{
    const uint16_t nr = rs->nroots, A0 = (uint8_t)rs->nn;
    uint16_t s, flag = 0;
    size_t b;
    int r;

    for (r = 0; r < nr; r++)
        syn[r] = data[0] & A0;
    for (b = 1; b < size + nr; b++) {
        const uint16_t in = (b < size ? data[b] : parity[b - size]) & A0;
        for (r = 0; r < nr; r++) {
            s = syn[r];
            syn[r] = s ? (uint16_t)(in ^ rs->alog[MOD(rs->log[s] + (rs->fcr + r) * rs->prim)]) : in;
        }
    }
    for (r = 0; r < nr; r++) {
        flag |= syn[r];
        syn[r] = rs->log[syn[r]];
    }
    return flag != 0;
}

/*
 * src/decode.c:17-230 (error_correction_u8): erasure locator, Berlekamp-
 * Massey, Chien, Omega, Forney, re-syndrome check, apply.  eras_apply selects
 * the erasure-list apply rule (:211-214) versus the location rule (:215-227).
 */
static int correct(const oracle_rs_t *rs, uint8_t *data, size_t size, uint8_t *parity, const uint16_t *S,
                   uint32_t ne, const uint32_t *pos, int eras_apply, int16_t pad, size_t *corrected)
{
    const uint16_t nr = rs->nroots;
    const uint16_t A0 = (uint8_t)rs->nn;
    uint16_t lam[ORACLE_MAX_ROOTS + 1], B[ORACLE_MAX_ROOTS + 1], T[ORACLE_MAX_ROOTS + 1];
    uint16_t reg[ORACLE_MAX_ROOTS + 1], omega[ORACLE_MAX_ROOTS + 1];
    uint16_t roots[ORACLE_MAX_ROOTS + 1], locs[ORACLE_MAX_ROOTS + 1], mag[ORACLE_MAX_ROOTS + 1];
    uint32_t r, L;
    uint16_t deg, cnt, disc, acc, num, num2, den;
    int16_t i, j, k;

    /* erasure locator prod (1 + X_l x), X_l = alpha^(prim*(nn-1-(pos+pad))) */
    memset(lam, 0, sizeof(uint16_t) * (nr + 1u));
    lam[0] = 1;
    if (ne > 0) {
        lam[1] = rs->alog[MOD(rs->prim * ((uint32_t)(uint8_t)rs->nn - 1u - (pos[0] + (uint32_t)(int32_t)pad)))];
        for (i = 1; (uint32_t)i < ne; i++) {
            const uint8_t xl =
                (uint8_t)MOD(rs->prim * ((uint32_t)(uint8_t)rs->nn - 1u - (pos[i] + (uint32_t)(int32_t)pad)));
            for (j = (int16_t)(i + 1); j > 0; j--) {
                const uint16_t lg = rs->log[lam[j - 1]];
                if (lg != A0)
                    lam[j] ^= rs->alog[MOD(xl + lg)];
            }
        }
    }
    for (i = 0; i <= (int16_t)nr; i++)
        B[i] = rs->log[lam[i]];

    /* Berlekamp-Massey, r = ne+1 .. nroots */
    r = ne;
    L = ne;
    while (++r <= nr) {
        disc = 0;
        for (i = 0; (uint32_t)i < r; i++)
            if (lam[i] != 0 && S[r - (uint32_t)i - 1] != A0)
                disc ^= rs->alog[MOD(rs->log[lam[i]] + S[r - (uint32_t)i - 1])];
        disc = rs->log[disc];
        if (disc == A0) {
            memmove(B + 1, B, sizeof(uint16_t) * nr);
            B[0] = A0;
            continue;
        }
        T[0] = lam[0];
        for (i = 0; i < (int16_t)nr; i++)
            T[i + 1] = (B[i] != A0) ? (uint16_t)(lam[i + 1] ^ rs->alog[MOD(disc + B[i])]) : lam[i + 1];
        if (2 * L <= r + ne - 1) {
            L = r + ne - L;
            for (i = 0; i <= (int16_t)nr; i++)
                B[i] = (lam[i] == 0) ? A0 : MOD(rs->log[lam[i]] - disc + A0);
        } else {
            memmove(B + 1, B, sizeof(uint16_t) * nr);
            B[0] = A0;
        }
        memcpy(lam, T, sizeof(uint16_t) * (nr + 1u));
    }

    /* locator to log form, degree */
    deg = 0;
    for (i = 0; i <= (int16_t)nr; i++) {
        lam[i] = rs->log[lam[i]];
        if (lam[i] != A0)
            deg = (uint16_t)i;
    }
    if (deg == 0)
        return 0;

    /* Chien search over alpha^1 .. alpha^nn, ascending */
    memcpy(reg + 1, lam + 1, sizeof(uint16_t) * nr);
    cnt = 0;
    for (i = 1, k = (int16_t)(rs->iprim - 1); i <= (int16_t)(uint8_t)rs->nn;
         i++, k = (int16_t)MOD((int32_t)k + rs->iprim)) {
        acc = 1;
        for (j = (int16_t)deg; j > 0; j--) {
            if (reg[j] != A0) {
                reg[j] = MOD(reg[j] + j);
                acc ^= rs->alog[reg[j]];
            }
        }
        if (acc != 0)
            continue;
        if (k < pad)
            return 0;
        roots[cnt] = (uint16_t)i;
        locs[cnt] = (uint16_t)k;
        if (++cnt == deg)
            break;
    }
    if (cnt != deg)
        return 0;

    /* Omega = S * Lambda truncated to deg terms, log form */
    for (i = 0; i <= (int16_t)(deg - 1); i++) {
        acc = 0;
        for (j = i; j >= 0; j--)
            if (S[i - j] != A0 && lam[j] != A0)
                acc ^= rs->alog[MOD(S[i - j] + lam[j])];
        omega[i] = rs->log[acc];
    }

    /* Forney; corrected counts nonzero numerators (also on later failure) */
    *corrected = 0;
    for (j = (int16_t)(cnt - 1); j >= 0; j--) {
        num = 0;
        for (i = (int16_t)(deg - 1); i >= 0; i--)
            if (omega[i] != A0)
                num ^= rs->alog[MOD(omega[i] + i * roots[j])];
        if (num == 0) {
            mag[j] = 0;
            continue;
        }
        num2 = rs->alog[MOD(roots[j] * (rs->fcr - 1) + (uint8_t)rs->nn)];
        den = 0;
        for (i = (int16_t)((deg < nr - 1 ? deg : nr - 1) & ~1); i >= 0; i -= 2)
            if (lam[i + 1] != A0)
                den ^= rs->alog[MOD(lam[i + 1] + i * roots[j])];
        mag[j] = rs->alog[MOD(rs->log[num] + rs->log[num2] + (uint8_t)rs->nn - rs->log[den])];
        (*corrected)++;
    }

    /* the error pattern must reproduce every syndrome */
    for (i = 0; i < (int16_t)nr; i++) {
        acc = 0;
        for (j = 0; j < (int16_t)cnt; j++) {
            if (mag[j] == 0)
                continue;
            k = (int16_t)((rs->fcr + i) * rs->prim * ((uint8_t)rs->nn - locs[j] - 1));
            acc ^= rs->alog[MOD(rs->log[mag[j]] + k)];
        }
        if (acc != rs->alog[S[i]])
            return 0;
    }

    if (eras_apply) {
        /* quirk Q1/Q2: magnitude j (ascending location) goes to list slot j.
         * Slots outside data[] are undefined behaviour in the reference;
         * here they address parity (p < size+nroots) or are dropped. */
        for (i = 0; i < (int16_t)cnt; i++) {
            const uint32_t p = pos[i];
            if (p < size)
                data[p] ^= (uint8_t)mag[i];
            else if (p < size + nr)
                parity[p - size] ^= (uint8_t)mag[i];
        }
    } else {
        for (i = 0; i < (int16_t)cnt; i++) {
            const int32_t p = (int32_t)locs[i] - (int32_t)pad;
            if (p >= 0 && p < (int32_t)size)
                data[p] ^= (uint8_t)mag[i];
            else if (p >= (int32_t)size && p < (int32_t)(size + nr))
                parity[p - (int32_t)size] ^= (uint8_t)mag[i];
            else
                return 0;
        }
    }
    return 1;
}

/* src/decode.c:418-429: int16 truncation of nn - nroots - size. */
static int16_t padding(const oracle_rs_t *rs, size_t size)
{
    const int16_t p = (int16_t)(uint16_t)((size_t)(uint8_t)rs->nn - rs->nroots - size);
    if (p < 0 || p >= (int)(uint8_t)rs->nn - (int)rs->nroots)
        return -1;
    return p;
}

/* src/decode.c:431-487 plus the argument checks of src/decode.c:596-600. */
int oracle_rs_decode(const oracle_rs_t *rs, uint8_t *data, size_t size, uint8_t *parity, int eras_mode,
                     const uint32_t *eras_pos, uint32_t eras_count, const uint16_t *ext_syn, size_t *corrected)
{
    uint16_t S[ORACLE_MAX_ROOTS + 1];
    size_t fixed = 0;
    int ok = 0, r;
    int16_t pad;

    if (!data || !parity || !size)
        return 0;
    pad = padding(rs, size);
    if (pad < 0)
        goto out;
    if (ext_syn) {
        int any = 0;
        for (r = 0; r < rs->nroots; r++)
            any |= ext_syn[r] != (uint8_t)rs->nn;
        ok = !any || correct(rs, data, size, parity, ext_syn, 0, NULL, 0, pad, &fixed);
        goto out;
    }
    if (eras_mode) {
        if (eras_count > rs->nroots) /* UB in the reference (quirk Q5) */
            goto out;
        ok = !oracle_rs_syndrome(rs, data, size, parity, S) ||
             correct(rs, data, size, parity, S, eras_count, eras_pos, 1, pad, &fixed);
        goto out;
    }
    ok = !oracle_rs_syndrome(rs, data, size, parity, S) || correct(rs, data, size, parity, S, 0, NULL, 0, pad, &fixed);
out:
    if (corrected)
        *corrected = fixed;
    return ok;
}

void oracle_rs_encode_batch(const oracle_rs_t *rs, const uint8_t *data, size_t data_stride, uint8_t *parity,
                            size_t parity_stride, size_t size, size_t count)
{
    size_t c;
    for (c = 0; c < count; c++)
        oracle_rs_encode(rs, data + c * data_stride, size, parity + c * parity_stride);
}

void oracle_rs_decode_batch(const oracle_rs_t *rs, uint8_t *data, size_t data_stride, uint8_t *parity,
                            size_t parity_stride, size_t size, size_t count, int eras_mode, const uint32_t *eras_pos,
                            size_t eras_stride, const uint32_t *eras_count, uint8_t *ok, uint32_t *corrected)
{
    size_t c, fixed;
    for (c = 0; c < count; c++) {
        fixed = 0;
        ok[c] = (uint8_t)oracle_rs_decode(rs, data + c * data_stride, size, parity + c * parity_stride, eras_mode,
                                          eras_mode ? eras_pos + c * eras_stride : NULL,
                                          eras_mode ? eras_count[c] : 0, NULL, &fixed);
        corrected[c] = (uint32_t)fixed;
    }
}

typedef struct {
    const oracle_rs_t *rs;
    uint8_t *data, *parity;
    size_t ds, ps, size, count;
    int eras_mode;
    const uint32_t *eras_pos, *eras_count;
    size_t es;
    uint8_t *ok;
    uint32_t *corrected;
    int decode;
} slice_t;

static void *run_slice(void *arg)
{
    slice_t *s = (slice_t *)arg;
    if (s->decode)
        oracle_rs_decode_batch(s->rs, s->data, s->ds, s->parity, s->ps, s->size, s->count, s->eras_mode, s->eras_pos,
                               s->es, s->eras_count, s->ok, s->corrected);
    else
        oracle_rs_encode_batch(s->rs, s->data, s->ds, s->parity, s->ps, s->size, s->count);
    return NULL;
}

static void run_mt(slice_t base, int nthreads)
{
    pthread_t th[256];
    slice_t sl[256];
    size_t per, c0 = 0;
    int t;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    per = (base.count + (size_t)nthreads - 1) / (size_t)nthreads;
    for (t = 0; t < nthreads; t++) {
        sl[t] = base;
        sl[t].count = c0 < base.count ? (base.count - c0 < per ? base.count - c0 : per) : 0;
        sl[t].data = base.data + c0 * base.ds;
        sl[t].parity = base.parity + c0 * base.ps;
        if (base.decode) {
            sl[t].ok = base.ok + c0;
            sl[t].corrected = base.corrected + c0;
            if (base.eras_mode) {
                sl[t].eras_pos = base.eras_pos + c0 * base.es;
                sl[t].eras_count = base.eras_count + c0;
            }
        }
        c0 += sl[t].count;
        pthread_create(&th[t], NULL, run_slice, &sl[t]);
    }
    for (t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
}

void oracle_rs_encode_batch_mt(const oracle_rs_t *rs, const uint8_t *data, size_t data_stride, uint8_t *parity,
                               size_t parity_stride, size_t size, size_t count, int nthreads)
{
    slice_t s;
    memset(&s, 0, sizeof(s));
    s.rs = rs;
    s.data = (uint8_t *)data;
    s.parity = parity;
    s.ds = data_stride;
    s.ps = parity_stride;
    s.size = size;
    s.count = count;
    run_mt(s, nthreads);
}

void oracle_rs_decode_batch_mt(const oracle_rs_t *rs, uint8_t *data, size_t data_stride, uint8_t *parity,
                               size_t parity_stride, size_t size, size_t count, int eras_mode,
                               const uint32_t *eras_pos, size_t eras_stride, const uint32_t *eras_count, uint8_t *ok,
                               uint32_t *corrected, int nthreads)
{
    slice_t s;
    memset(&s, 0, sizeof(s));
    s.rs = rs;
    s.data = data;
    s.parity = parity;
    s.ds = data_stride;
    s.ps = parity_stride;
    s.size = size;
    s.count = count;
    s.eras_mode = eras_mode;
    s.eras_pos = eras_pos;
    s.es = eras_stride;
    s.eras_count = eras_count;
    s.ok = ok;
    s.corrected = corrected;
    s.decode = 1;
    run_mt(s, nthreads);
}
