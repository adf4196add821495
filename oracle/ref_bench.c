/*
 * ref_bench.c — CPU-baseline harness around the REFERENCE reader.
 * TEST/BENCH INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg).
 *
 * Linked against oracle/_ref/libzseek_ref.so, i.e. /root/reference/src/*.c
 * compiled by oracle/Makefile against liblz4 1.9.3 / libzstd 1.4.9.  It times
 * exactly the reference hot path: T independent reader handles
 * (zseek_reader_open_full over an in-memory pread callback), each looping
 * zseek_pread over a disjoint, frame-aligned slice of the decompressed range,
 * as BASELINE.md §3 prescribes.
 *
 * Exported (C ABI, loaded with ctypes):
 *   int ref_bench_run(img, img_len, threads, d_begin, d_end, align, req,
 *                     cache_size, out, &seconds, &bytes, errbuf)
 *   out == NULL  -> decode into a per-thread scratch buffer (timing);
 *   out != NULL  -> decoded bytes of [d_begin, d_end) land in out (checking).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "zseek.h"

typedef struct {
    const uint8_t *img;
    size_t len;
} mem_file_t;

static ssize_t mem_pread(void *data, size_t size, size_t offset,
                         void *user_data, void *call_data)
{
    (void)call_data;
    const mem_file_t *f = user_data;
    if (offset >= f->len)
        return 0;
    size_t n = f->len - offset < size ? f->len - offset : size;
    memcpy(data, f->img + offset, n);
    return (ssize_t)n;
}

static ssize_t mem_fsize(void *user_data, void *call_data)
{
    (void)call_data;
    return (ssize_t)((const mem_file_t *)user_data)->len;
}

typedef struct {
    mem_file_t file;
    zseek_reader_t *reader;
    uint64_t begin, end;
    size_t req;
    uint8_t *out;   /* NULL -> scratch */
    uint8_t *scratch;
    pthread_barrier_t *bar;
    int ok;
    uint64_t bytes;
    char err[ZSEEK_ERRBUF_SIZE];
} job_t;

static void *worker(void *arg)
{
    job_t *j = arg;
    pthread_barrier_wait(j->bar);
    uint64_t off = j->begin;
    j->ok = 1;
    while (off < j->end) {
        size_t want = j->end - off < j->req ? (size_t)(j->end - off) : j->req;
        uint8_t *dst = j->out ? j->out + (off - j->begin) : j->scratch;
        ssize_t r = zseek_pread(j->reader, dst, want, off, NULL, j->err);
        if (r <= 0) {
            j->ok = 0;
            break;
        }
        off += (uint64_t)r;
        j->bytes += (uint64_t)r;
    }
    pthread_barrier_wait(j->bar);
    return NULL;
}

__attribute__((visibility("default")))
int ref_bench_run(const uint8_t *img, size_t img_len, int threads,
                  uint64_t d_begin, uint64_t d_end, uint64_t align, size_t req,
                  size_t cache_size, uint8_t *out, double *seconds,
                  uint64_t *bytes, char *errbuf)
{
    if (threads < 1 || d_end < d_begin || req == 0 || align == 0)
        return -1;
    job_t *jobs = calloc((size_t)threads, sizeof(job_t));
    pthread_t *tids = calloc((size_t)threads, sizeof(pthread_t));
    pthread_barrier_t bar;
    pthread_barrier_init(&bar, NULL, (unsigned)threads + 1);
    uint64_t span = d_end - d_begin;
    uint64_t per = (span / (uint64_t)threads + align - 1) / align * align;
    int rc = 0;
    for (int t = 0; t < threads; t++) {
        job_t *j = &jobs[t];
        j->file.img = img;
        j->file.len = img_len;
        zseek_read_file_t uf = {&j->file, mem_pread, mem_fsize};
        j->reader = zseek_reader_open_full(uf, cache_size, NULL, j->err);
        if (!j->reader) {
            rc = -1;
            if (errbuf)
                memcpy(errbuf, j->err, ZSEEK_ERRBUF_SIZE);
        }
        j->begin = d_begin + (uint64_t)t * per;
        if (j->begin > d_end)
            j->begin = d_end;
        j->end = j->begin + per > d_end ? d_end : j->begin + per;
        j->req = req;
        j->out = out ? out + (j->begin - d_begin) : NULL;
        j->scratch = out ? NULL : malloc(req);
        j->bar = &bar;
    }
    if (rc == 0) {
        for (int t = 0; t < threads; t++)
            pthread_create(&tids[t], NULL, worker, &jobs[t]);
        struct timespec t0, t1;
        pthread_barrier_wait(&bar);
        clock_gettime(CLOCK_MONOTONIC, &t0);
        pthread_barrier_wait(&bar);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        for (int t = 0; t < threads; t++)
            pthread_join(tids[t], NULL);
        *seconds = (double)(t1.tv_sec - t0.tv_sec) +
                   1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
        uint64_t total = 0;
        for (int t = 0; t < threads; t++) {
            total += jobs[t].bytes;
            if (!jobs[t].ok && jobs[t].begin < jobs[t].end) {
                rc = -1;
                if (errbuf)
                    memcpy(errbuf, jobs[t].err, ZSEEK_ERRBUF_SIZE);
            }
        }
        *bytes = total;
    }
    for (int t = 0; t < threads; t++) {
        zseek_reader_close(jobs[t].reader, NULL, NULL);
        free(jobs[t].scratch);
    }
    pthread_barrier_destroy(&bar);
    free(tids);
    free(jobs);
    return rc;
}
