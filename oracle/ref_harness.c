/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY: multi-threaded driver for the
 * REAL reference (libpoporon compiled from /root/reference/src into
 * oracle/_ref by oracle/Makefile).  bench.py's cpu_baseline leg times it.
 *
 * Each thread owns one poporon handle (the reference handle is not
 * reentrant, src/internal/common.h:62-72) and loops the reference's public
 * single-codeword API over a contiguous slice, exactly as an application
 * would (README.md:63-101).
 */
#include <poporon.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>

typedef struct {
    uint8_t *data, *parity;
    size_t ds, ps, size, count;
    uint8_t *ok, *cor;
    int decode;
} job_t;

static void *run(void *arg)
{
    job_t *j = (job_t *)arg;
    poporon_config_t *cfg = poporon_config_rs_default();
    poporon_t *h = poporon_create(cfg);
    poporon_config_destroy(cfg);
    for (size_t c = 0; c < j->count; c++) {
        if (j->decode) {
            size_t n = 0;
            j->ok[c] = poporon_decode(h, j->data + c * j->ds, j->size, j->parity + c * j->ps, &n);
            j->cor[c] = (uint8_t)n;
        } else {
            poporon_encode(h, j->data + c * j->ds, j->size, j->parity + c * j->ps);
        }
    }
    poporon_destroy(h);
    return NULL;
}

static void run_all(job_t base, int nthreads)
{
    pthread_t th[256];
    job_t jb[256];
    size_t per, c0 = 0;
    int t;
    if (nthreads < 1)
        nthreads = 1;
    if (nthreads > 256)
        nthreads = 256;
    per = (base.count + (size_t)nthreads - 1) / (size_t)nthreads;
    for (t = 0; t < nthreads; t++) {
        jb[t] = base;
        jb[t].count = c0 < base.count ? (base.count - c0 < per ? base.count - c0 : per) : 0;
        jb[t].data = base.data + c0 * base.ds;
        jb[t].parity = base.parity + c0 * base.ps;
        if (base.decode) {
            jb[t].ok = base.ok + c0;
            jb[t].cor = base.cor + c0;
        }
        c0 += jb[t].count;
        pthread_create(&th[t], NULL, run, &jb[t]);
    }
    for (t = 0; t < nthreads; t++)
        pthread_join(th[t], NULL);
}

void refbench_encode(uint8_t *data, size_t ds, uint8_t *parity, size_t ps, size_t size, size_t count, int nthreads)
{
    job_t j = {data, parity, ds, ps, size, count, NULL, NULL, 0};
    run_all(j, nthreads);
}

void refbench_decode(uint8_t *data, size_t ds, uint8_t *parity, size_t ps, size_t size, size_t count, uint8_t *ok,
                     uint8_t *cor, int nthreads)
{
    job_t j = {data, parity, ds, ps, size, count, ok, cor, 1};
    run_all(j, nthreads);
}
