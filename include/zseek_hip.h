/*
 * zseek_hip.h — GPU extensions of the MI355X-native libzseek (C ABI).
 *
 * Plain pointers and sizes only (no HIP or torch types): device pointers are
 * hipMalloc'd (or torch-allocated) memory on the reader's device, and a
 * stream is a hipStream_t passed as void* (NULL = the library's own stream).
 *
 * Reference interfaces these replace / extend:
 *   zsk_lz4_decode_frames  — the per-frame LZ4F_decompress loop of
 *                            /root/reference/src/decompress.c:752-773 (and
 *                            :627-664 for the no-cache variant), batched over
 *                            every frame of a request in one grid.
 *   zsk_zstd_decode_frames — ZSTD_decompressDCtx (decompress.c:537) /
 *                            ZSTD_decompressStream (:414-454), batched the
 *                            same way.
 *   zsk_reader_frames      — the seek-table accessors frame_offset_c/d and
 *                            frame_size_c/d, seek_table.c:204-226.
 *   zsk_pread_device       — zseek_pread (decompress.c:806-824) with the
 *                            decoded bytes left in device memory.
 *   zsk_verify_frame_checksums — the seek table's per-frame checksum,
 *                            parsed by seek_table.c:95-97 and never checked
 *                            there, checked on the GPU.
 *   zsk_lz4_compress_frames, zsk_writer_set_gpu_compress — the writer's
 *                            per-frame LZ4F_compressFrame call
 *                            (compress.c:750 direct frames, :483 buffered
 *                            ones; prefs compress.c:203-207), batched over
 *                            frames of <= 4 MiB in one grid.
 */
#ifndef ZSEEK_HIP_H
#define ZSEEK_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "zseek.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One seek-table frame of a device batch. */
typedef struct {
    uint64_t c_off;   /* compressed frame start in d_comp                  */
    uint64_t d_off;   /* decoded frame start in d_out                      */
    uint32_t c_size;  /* compressed size (seek-table cSize)                */
    uint32_t d_size;  /* decoded size (seek-table dSize); the frame writes */
                      /* exactly [d_off, d_off + d_size) of d_out          */
} zsk_frame_desc_t;

/* Per-frame status codes written to d_status (low 16 bits).  Values 1..19
 * follow liblz4's LZ4F error numbering (see zsk_status_string). */
#define ZSK_OK 0
#define ZSK_ERR_DST_OVERFLOW 100  /* frame decodes past its dSize        */
#define ZSK_ERR_SHORT_FRAME 101   /* frame decodes to less than dSize    */
#define ZSK_ERR_TRUNCATED 102     /* compressed frame ends mid-block     */
#define ZSK_STATUS_DIRECT 0x10000 /* liblz4 would have used its direct path */
#define ZSK_STATUS_BLOCK 0x20000  /* the failure is inside an LZ4 block   */
/* bits 24-25: LZ4 block size id - 4 of a frame that failed in a block */

/*
 * Decode @nframes independent LZ4 frames on the GPU, asynchronously on
 * @stream.  @d_desc, @d_comp, @d_out, @d_status are device pointers;
 * @d_comp must stay readable up to the 4-byte boundary after the last
 * compressed byte.  Each frame writes only its own [d_off, d_off+d_size).
 * Returns 0 if the launch was queued, -1 otherwise.
 */
ZSEEK_EXPORT int zsk_lz4_decode_frames(const zsk_frame_desc_t *d_desc,
    uint32_t nframes, const void *d_comp, void *d_out, int32_t *d_status,
    void *stream);

/*
 * Decode @nframes independent zstd frames (each seek-table entry: the zstd
 * frames and skippable frames it holds, as ZSTD_decompressDCtx decodes them)
 * on the GPU, on @stream.  Same descriptors and per-frame status as
 * zsk_lz4_decode_frames; a failed frame's status is ZSK_STATUS_ZSTD | the
 * ZSTD_ErrorCode libzstd 1.4.9 reports for it.  The call synchronizes
 * @stream once, after the planning kernel (a frame's sequence count sizes its
 * scratch), and returns with the decode queued.  Returns 0 or -1.
 */
ZSEEK_EXPORT int zsk_zstd_decode_frames(const zsk_frame_desc_t *d_desc,
    uint32_t nframes, const void *d_comp, void *d_out, int32_t *d_status,
    void *stream);
#define ZSK_STATUS_ZSTD 0x4000000 /* zstd frame failure: low bits = ZSTD_ErrorCode */

/* Human-readable name of a frame status (LZ4F-style "ERROR_..." names for
 * LZ4 frames, ZSTD_getErrorName strings for zstd frames). */
ZSEEK_EXPORT const char *zsk_status_string(int32_t status);

/*
 * zsk_lz4_decode_frames with one of the library's production decoders forced
 * for every frame (testing, tooling): ZSK_DECODER_AUTO is the library's own
 * choice (= zsk_lz4_decode_frames); WAVE the wave-per-frame decoder; LEAN,
 * SCAN and CHUNK the two-phase decoder with that parse kernel for every frame;
 * BLOCK the two-phase decoder's block route (one parse lane per LZ4 block of
 * each multi-block frame, the chunk parse for the rest) at any batch size.
 * Returns -1 for an unknown decoder.
 */
#define ZSK_DECODER_AUTO 0
#define ZSK_DECODER_WAVE 1
#define ZSK_DECODER_LEAN 2
#define ZSK_DECODER_SCAN 3
#define ZSK_DECODER_CHUNK 4
#define ZSK_DECODER_BLOCK 5
/* the one-frame route (every frame through the chunk parse reading it staged
 * in LDS), the library's own choice for batches of <= 64 frames, forced at
 * any size */
#define ZSK_DECODER_ONE 6
ZSEEK_EXPORT int zsk_lz4_decode_frames_ex(const zsk_frame_desc_t *d_desc,
    uint32_t nframes, const void *d_comp, void *d_out, int32_t *d_status,
    void *stream, int decoder);

/* Name of the dominant HIP kernel zsk_lz4_decode_frames launches for a
 * batch of nframes frames (as it appears in a rocprofv3 kernel trace,
 * without namespace), for tooling: the two-phase decoder's execute,
 * seq_exec_kernel, unless the environment forces the
 * wave-per-frame decoder (env ZSEEK_HIP_KERNEL=wave forces it). */
ZSEEK_EXPORT const char *zsk_lz4_kernel_name(uint32_t nframes);

/* Name of the parse kernel the two-phase decoder runs for a frame of
 * @c_size compressed bytes in a batch of @nframes frames (lz4_lean_kernel,
 * lz4_scan_kernel or lz4_chunk_kernel; lz4_wave_kernel for small batches):
 * the library's routing, exposed so tools attribute time and traffic to the
 * kernel that actually runs. */
ZSEEK_EXPORT const char *zsk_lz4_parse_kernel_name(uint32_t nframes, uint32_t c_size);

/* Measurement hook: while on, every two-phase decode launch records HIP
 * events between its stages (plan, parse, execute, hand-off) on its stream,
 * and a zstd launch also around each chunk's kernels on the streams they run
 * on.  zsk_kernel_timing(on) switches it and clears the records;
 * zsk_kernel_times(ms, cap) waits for the recorded launches and writes, per
 * slot, the MEDIAN milliseconds over them into ms[0..min(cap,8)): [0..3] the
 * stages; [4..7] (zstd launches, summed over the launch's chunks)
 * zstd_frame_kernel, zstd_seq_kernel, zstd_huf_kernel and seq_exec_kernel
 * (the zstd literal-source execute).  Returns the
 * number of launches recorded.  Not on any decode path's critical path. */
ZSEEK_EXPORT int zsk_kernel_timing(int on);
ZSEEK_EXPORT int zsk_kernel_times(double *ms, int cap);

/* Number of frames of an open reader and its seek table as prefix sums:
 * c_off/d_off receive n+1 entries each (either may be NULL). */
ZSEEK_EXPORT ssize_t zsk_reader_frames(zseek_reader_t *reader,
    uint64_t *c_off, uint64_t *d_off);

/* Codec of an open reader (ZSEEK_LZ4 / ZSEEK_ZSTD), -1 for NULL. */
ZSEEK_EXPORT int zsk_reader_type(zseek_reader_t *reader);

/*
 * zseek_pread into device memory @d_buf (on the reader's device): decoded
 * bytes [offset, offset+count) are produced on the GPU and never cross PCIe.
 * Same return convention as zseek_pread.  Synchronous.
 */
ZSEEK_EXPORT ssize_t zsk_pread_device(zseek_reader_t *reader, void *d_buf,
    size_t count, size_t offset, void *call_data,
    char errbuf[ZSEEK_ERRBUF_SIZE]);

/* GPU-side counters of a reader.  zsk_reader_gpu_stats fills the fields
 * through `device` (the struct's layout before copy_threads / io_parts were
 * added, so a caller built against that header is never written past its
 * struct); zsk_reader_gpu_stats_ex(reader, stats, sizeof *stats) fills the
 * first @size bytes of the current layout (at most its size). */
typedef struct {
    uint64_t batches;          /* decode grids launched                 */
    uint64_t frames_decoded;   /* frames decoded on the GPU             */
    uint64_t bytes_decoded;    /* decoded bytes produced on the GPU     */
    uint64_t bytes_uploaded;   /* compressed bytes copied host->device  */
    uint64_t device_memory;    /* device bytes held by the reader       */
    int device;                /* HIP device ordinal, -1 before first use */
    int copy_threads;          /* host copy / pread pool threads (usable CPUs - 2, 2..16) */
    int io_parts;              /* concurrent pread callbacks a batch uses: min(io_threads, copy_threads / 2) */
} zsk_gpu_stats_t;

ZSEEK_EXPORT bool zsk_reader_gpu_stats(zseek_reader_t *reader,
    zsk_gpu_stats_t *stats);
ZSEEK_EXPORT bool zsk_reader_gpu_stats_ex(zseek_reader_t *reader,
    zsk_gpu_stats_t *stats, size_t size);

/* Largest decoded span one batch grid covers (bytes, default 64 MiB; env
 * ZSEEK_HIP_BATCH_BYTES overrides at open).  A read runs as a pipeline of
 * such batches (the user pread of one, the upload / decode / download of
 * the next and the copy into the caller's buffer of a third overlap); its
 * first batch is at most 4 MiB. */
ZSEEK_EXPORT bool zsk_reader_set_batch_bytes(zseek_reader_t *reader,
    size_t bytes);

/*
 * Seek-table frame checksums.  The seekable format's optional per-frame
 * checksum (descriptor bit 7; 12-byte entries cSize, dSize, checksum,
 * seek_table.c:95-97 / writer :392-396) is the low 32 bits of XXH64(seed 0)
 * of the frame's decoded bytes; the reference parses it and never checks it.
 *
 * zsk_verify_frame_checksums: for every frame whose d_status is ZSK_OK, hash
 * d_out[d_off, d_off + d_size) on the GPU and set its status to
 * ZSK_ERR_SEEK_CHECKSUM when the low 32 bits differ from d_checksums[f]
 * (device array, one u32 per frame).  Asynchronous on @stream; 0 or -1.
 */
#define ZSK_ERR_SEEK_CHECKSUM 104
ZSEEK_EXPORT int zsk_verify_frame_checksums(const zsk_frame_desc_t *d_desc,
    uint32_t nframes, const void *d_out, const uint32_t *d_checksums,
    int32_t *d_status, void *stream);

/* Make a reader check the seek-table checksum of every frame it decodes
 * (files whose seek table carries them).  Default off, as the reference; env
 * ZSEEK_VERIFY_CHECKSUMS=1 at open turns it on.  A mismatching frame fails
 * like a corrupt one: a short read, then -1 and "...: frame checksum
 * mismatch".  false for a NULL reader. */
ZSEEK_EXPORT bool zsk_reader_set_verify_checksums(zseek_reader_t *reader,
    bool on);

/*
 * Allow up to @n concurrent calls of the reader's pread callback (on
 * disjoint ranges of >= 4 MiB of one batch's compressed span).  Default 1,
 * the reference's contract: it calls pread under the reader's lock, one call
 * at a time, and its default FILE* callback is not safe to call concurrently.
 * Only for callbacks that are (an in-memory image, pread(2) on a descriptor).
 * The calls run on the library's host pool, at most half of it at once (the
 * rest keeps copying decoded batches out): zsk_gpu_stats_t.io_parts.
 * Env ZSEEK_IO_THREADS at open.  false for a NULL reader or n outside 1..64.
 */
ZSEEK_EXPORT bool zsk_reader_set_io_threads(zseek_reader_t *reader, int n);

/*
 * The devices a reader decodes on: one decode pipeline ("lane") per entry; a
 * multi-frame read is split into contiguous frame ranges by decoded bytes,
 * one per lane, decoded concurrently (host destinations: each lane copies its
 * part into the caller's buffer; zsk_pread_device: each lane copies its part
 * into the destination, peer-to-peer from another device).  A device may
 * repeat (several pipelines on one GPU).  Default: env ZSEEK_HIP_DEVICES
 * ("0,1,2,3") at the first read, else ZSEEK_HIP_DEVICE, else the calling
 * thread's current device.  false for a NULL reader or an invalid device.
 * zsk_reader_devices writes up to @cap entries and returns the count (0
 * before the first read has picked the default).
 */
ZSEEK_EXPORT bool zsk_reader_set_devices(zseek_reader_t *reader,
    const int *devices, int n);
ZSEEK_EXPORT int zsk_reader_devices(zseek_reader_t *reader, int *devices,
    int cap);

/*
 * LZ4 frame compression, byte-identical to the reference
 * writer's frames: LZ4F_compressFrame(level, autoFlush = 1, 64 KiB blocks) of
 * liblz4 1.9.3, as compress.c:737-786 / :463-518 call it.  One frame per
 * descriptor, src_size <= ZSK_LZ4_COMPRESS_MAX_FRAME (one independent block
 * up to 64 KiB, linked 64 KiB blocks above; larger frames are refused with
 * c_size 0).  ZSK_COMPRESS_CONTENT_SIZE = the writer's contentSize != 0 case
 * (a buffered frame flushed by end_frame_lz4, compress.c:472): the header
 * then carries the frame's size.
 */
typedef struct {
    uint64_t src_off;   /* frame input start in d_src                        */
    uint64_t dst_off;   /* output slot start in d_dst: 16-byte aligned, at    */
                        /* least ZSK_LZ4_COMPRESS_BOUND(src_size) bytes       */
    uint32_t src_size;  /* <= ZSK_LZ4_COMPRESS_MAX_FRAME                      */
    uint32_t flags;     /* ZSK_COMPRESS_CONTENT_SIZE                          */
} zsk_compress_desc_t;
#define ZSK_COMPRESS_CONTENT_SIZE 1u
#define ZSK_LZ4_COMPRESS_MAX_FRAME (1u << 22)
#define ZSK_LZ4_COMPRESS_BOUND(n) \
    ((((uint64_t)(n)) + 4 * (((uint64_t)(n)) >> 16) + 24 + 15) & ~(uint64_t)15)

/* Device scratch bytes zsk_lz4_compress_frames needs for @nframes frames
 * (a 64 KiB table of position + input-word entries per frame); size scratch
 * with this call, not from the comment. */
ZSEEK_EXPORT size_t zsk_lz4_compress_scratch_size(uint32_t nframes);

/*
 * Compress @nframes frames on the GPU, asynchronously on @stream: frame f's
 * bytes d_src[src_off, src_off + src_size) become one LZ4 frame written at
 * d_dst + dst_off, its size in d_csize[f] (0 for a refused descriptor).
 * @level is the writer's compressionLevel (< 3: liblz4's fast encoder,
 * acceleration 1 - level for negative levels; HC levels return -1).
 * @d_scratch holds zsk_lz4_compress_scratch_size(nframes) bytes.  All
 * pointers are device pointers.  Returns 0 if queued, -1 otherwise.
 */
ZSEEK_EXPORT int zsk_lz4_compress_frames(const zsk_compress_desc_t *d_desc,
    uint32_t nframes, const void *d_src, void *d_dst, uint32_t *d_csize,
    int level, void *d_scratch, void *stream);

/*
 * Writer GPU mode: an LZ4 writer's frames of <= 4 MiB are compressed on the
 * GPU (zsk_lz4_compress_frames, on the calling thread's current device) in
 * batches of @batch_bytes input bytes (0: 1 GiB; (size_t)-1: GPU mode off,
 * after writing what is queued).  The file is byte-identical to host
 * compression.  Frames are written and logged when their batch is compressed:
 * when it fills, when a frame the GPU does not take (> 4 MiB) arrives, at
 * zseek_writer_stats and at zseek_writer_close; each write callback gets the
 * call_data of the zseek_write that produced the frame.  Deferred writes:
 * zseek_write returns true once its frame is QUEUED, so a compression or
 * write-callback failure of a queued frame is reported by the later call
 * that flushes (zseek_write, zseek_writer_stats or zseek_writer_close), not
 * by the zseek_write that queued it, and the writer then stays failed: every
 * later call, close included, returns false.  Staging is allocated at the
 * first queued frame and grows with the queue; frames per batch are capped
 * so the compressor's scratch (64 KiB per frame) stays within @batch_bytes.
 * Env ZSEEK_GPU_COMPRESS=1
 * (or a batch size in bytes) at open turns it on.  false for NULL, a zstd
 * writer, an HC level (>= 3) or no HIP device.
 */
ZSEEK_EXPORT bool zsk_writer_set_gpu_compress(zseek_writer_t *writer, size_t batch_bytes);

#ifdef __cplusplus
}
#endif

#endif /* ZSEEK_HIP_H */
