/*
 * zseek.h — public C API of the MI355X-native libzseek.
 *
 * Drop-in for the reference's header (/root/reference/src/zseek.h): the same
 * types, enum values, struct layouts and the same 11 exported functions with
 * the same signatures, argument meaning, return conventions and error-buffer
 * behaviour.  A program built against the reference header links and runs
 * against libzseek_amd/lib/libzseek.so unchanged.
 *
 * What differs is underneath zseek_pread: every seek-table frame the
 * requested range covers is decoded by one HIP grid on the GPU (see
 * include/zseek_hip.h and DESIGN.md), so one call may return the whole
 * multi-frame range instead of at most one frame.  Callers already loop on
 * short reads (the reference returns at most one frame per call), so this is
 * contract-compatible.
 */
#ifndef ZSEEK_H
#define ZSEEK_H

#include <stdbool.h>
#include <stddef.h>
#include <stdio.h>

#include <sched.h>
#include <sys/types.h>

#define ZSEEK_EXPORT __attribute__((visibility("default")))

/* Size of the caller-provided error message buffer (ref zseek.h:36). */
#define ZSEEK_ERRBUF_SIZE 80

#ifdef __cplusplus
extern "C" {
#endif

/* Write @size bytes of @data; true on success (ref zseek.h:55-56). */
typedef bool (*zseek_write_t)(const void *data, size_t size, void *user_data,
                              void *call_data);

/* User file for the writer (ref zseek.h:61-66). */
typedef struct {
    void *user_data;
    zseek_write_t write;
} zseek_write_file_t;

/* Read up to @size bytes at @offset into @data; bytes read (short at EOF) or
 * <0 on error (ref zseek.h:88-89). */
typedef ssize_t (*zseek_pread_t)(void *data, size_t size, size_t offset,
                                 void *user_data, void *call_data);

/* File size in bytes or <0 on error (ref zseek.h:104). */
typedef ssize_t (*zseek_fsize_t)(void *user_data, void *call_data);

/* User file for the reader (ref zseek.h:109-116). */
typedef struct {
    void *user_data;
    zseek_pread_t pread;
    zseek_fsize_t fsize;
} zseek_read_file_t;

/* Codec of a file (ref zseek.h:121-124). */
typedef enum {
    ZSEEK_ZSTD = 0,
    ZSEEK_LZ4,
} zseek_compression_type_t;

/* zstd writer controls (ref zseek.h:129-140). */
typedef struct {
    int nb_workers;
    size_t cpusetsize;
    cpu_set_t *cpuset;
    int compression_level;
    int strategy;
} zseek_zstd_param_t;

/* lz4 writer controls (ref zseek.h:145-148). */
typedef struct {
    int compression_level;
} zseek_lz4_param_t;

/* Writer controls (ref zseek.h:153-159). */
typedef struct {
    zseek_compression_type_t type;
    union {
        zseek_zstd_param_t zstd_params;
        zseek_lz4_param_t lz4_params;
    } params;
} zseek_compression_param_t;

typedef struct zseek_writer zseek_writer_t;
typedef struct zseek_reader zseek_reader_t;

/* Writer statistics (ref zseek.h:174-185). */
typedef struct {
    size_t seek_table_size;
    size_t seek_table_memory;
    size_t frames;
    size_t compressed_size;
    size_t buffer_size;
} zseek_writer_stats_t;

/* Reader statistics (ref zseek.h:190-203).  cache_memory / buffer_size
 * report this implementation's host memory (decoded-frame LRU, pinned
 * staging); GPU buffers are reported by zsk_reader_gpu_stats(). */
typedef struct {
    size_t seek_table_memory;
    size_t frames;
    size_t decompressed_size;
    size_t cache_memory;
    size_t cached_frames;
    size_t buffer_size;
} zseek_reader_stats_t;

/* --- writer (ref zseek.h:225-316) ---------------------------------------- */
ZSEEK_EXPORT zseek_writer_t *zseek_writer_open_full(zseek_write_file_t user_file,
    zseek_compression_param_t *zsp, size_t min_frame_size, void *call_data,
    char errbuf[ZSEEK_ERRBUF_SIZE]);
ZSEEK_EXPORT zseek_writer_t *zseek_writer_open(FILE *cfile,
    zseek_compression_param_t *zsp, size_t min_frame_size, void *call_data,
    char errbuf[ZSEEK_ERRBUF_SIZE]);
ZSEEK_EXPORT bool zseek_writer_close(zseek_writer_t *writer, void *call_data,
    char errbuf[ZSEEK_ERRBUF_SIZE]);
ZSEEK_EXPORT bool zseek_write(zseek_writer_t *writer, const void *buf,
    size_t len, void *call_data, char errbuf[ZSEEK_ERRBUF_SIZE]);
ZSEEK_EXPORT bool zseek_writer_stats(zseek_writer_t *writer,
    zseek_writer_stats_t *stats, char errbuf[ZSEEK_ERRBUF_SIZE]);

/* --- reader (ref zseek.h:335-443) ---------------------------------------- */
/* Open a seekable LZ4/zstd file; @cache_size = max decoded frames kept. */
ZSEEK_EXPORT zseek_reader_t *zseek_reader_open_full(zseek_read_file_t user_file,
    size_t cache_size, void *call_data, char errbuf[ZSEEK_ERRBUF_SIZE]);
ZSEEK_EXPORT zseek_reader_t *zseek_reader_open(FILE *cfile, size_t cache_size,
    void *call_data, char errbuf[ZSEEK_ERRBUF_SIZE]);
/* Always frees @reader; false (+errbuf) if something failed on the way. */
ZSEEK_EXPORT bool zseek_reader_close(zseek_reader_t *reader, void *call_data,
    char errbuf[ZSEEK_ERRBUF_SIZE]);
/* Decompressed bytes [offset, offset+count) into host @buf.  Returns N >= 0
 * bytes (0 at/after EOF; may be short) or -1 (+errbuf).  A NULL reader
 * returns 0 with "invalid reader", as the reference does. */
ZSEEK_EXPORT ssize_t zseek_pread(zseek_reader_t *reader, void *buf, size_t count,
    size_t offset, void *call_data, char errbuf[ZSEEK_ERRBUF_SIZE]);
ZSEEK_EXPORT ssize_t zseek_read(zseek_reader_t *reader, void *buf, size_t count,
    void *call_data, char errbuf[ZSEEK_ERRBUF_SIZE]);
ZSEEK_EXPORT bool zseek_reader_stats(zseek_reader_t *reader,
    zseek_reader_stats_t *stats, char errbuf[ZSEEK_ERRBUF_SIZE]);

#ifdef __cplusplus
}
#endif

#endif /* ZSEEK_H */
