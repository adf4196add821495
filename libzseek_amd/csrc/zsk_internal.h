// zsk_internal.h — shared between the host reader and the HIP kernels.
// Not installed; the public C ABI lives in include/zseek.h and
// include/zseek_hip.h.
#ifndef ZSK_INTERNAL_H
#define ZSK_INTERNAL_H

#include <stdint.h>

#include <hip/hip_runtime_api.h>

namespace zsk {

// One seek-table frame of a batch (layout shared with zsk_frame_desc_t in
// include/zseek_hip.h).
struct FrameDesc {
    uint64_t c_off;    // compressed frame offset in the batch's input span
    uint64_t d_off;    // decoded frame offset in the batch's output span
    uint32_t c_size;   // seek-table cSize
    uint32_t d_size;   // seek-table dSize
};
static_assert(sizeof(FrameDesc) == 24, "FrameDesc is part of the C ABI");

// Per-frame status.  Low 16 bits: liblz4 LZ4F error code numbering
// (lz4frame.h LZ4F_LIST_ERRORS, 0 = OK) or one of the zseek-specific codes
// >= 100.  Bit 16: the failing block would have been decoded by liblz4
// straight into the destination (its "direct" path, which reports
// ERROR_GENERIC) — used to reproduce the reference's error strings.
enum : int32_t {
    ST_OK = 0,
    ST_GENERIC = 1,
    ST_MAXBLOCK = 2,
    ST_VERSION = 6,
    ST_BLOCK_CHECKSUM = 7,
    ST_RESERVED = 8,
    ST_HDR_INCOMPLETE = 12,
    ST_FRAME_TYPE = 13,
    ST_FRAME_SIZE = 14,
    ST_DECOMPRESS_FAILED = 16,
    ST_HDR_CHECKSUM = 17,
    ST_CONTENT_CHECKSUM = 18,
    ST_DST_OVERFLOW = 100,   // frame decodes to more than its seek-table dSize
    ST_SHORT_FRAME = 101,    // frame decodes to less than its seek-table dSize
    ST_TRUNCATED = 102,      // compressed frame ends mid-block
    ST_UNSUPPORTED = 103,
    ST_SEEK_CHECKSUM = 104,  // decoded frame's XXH64 low 32 bits != its seek-table checksum
    ST_NOT_RUN = 0x7fff,     // status slot never written (launch failed)
    ST_BLOCK_ERR = 200,      // internal: block-level parse failure
    ST_DIRECT_FLAG = 0x10000,
    ST_BLOCK_FAIL_FLAG = 0x20000,   // failure inside an LZ4 block (fail_at valid)
    ST_BSID_SHIFT = 24,             // bits 24-25: block size id - 4 of the frame
    ST_ZSTD_FLAG = 0x4000000,       // zstd frame failure: low bits = ZSTD_ErrorCode
};

inline uint32_t status_max_block(int32_t st)
{
    return 1u << (8 + 2 * (((st >> ST_BSID_SHIFT) & 3) + 4));
}

// Name of the dominant kernel launch_lz4_frames uses for nframes frames
// (execute kernel of the two-phase decoder, or the wave kernel), for matching
// profiler output.
const char *lz4_kernel_name(uint32_t nframes);

// Production decoders a batch can be forced through (tests; ROUTE_AUTO is the
// library's own choice).  LEAN / SCAN / CHUNK: the two-phase decoder with that
// parse for every frame.
// BLOCK: every multi-block-capable frame through the block route below (any
// batch size, no job minimum).
// ONE: the one-frame route (batches of <= kOneMaxFrames frames under AUTO):
// every frame takes the chunk parse, reading the frame staged whole in LDS
// (one frame per workgroup); no plan scan, no lean / scan launches.
enum : int { ROUTE_AUTO = 0, ROUTE_WAVE = 1, ROUTE_LEAN = 2, ROUTE_SCAN = 3, ROUTE_CHUNK = 4, ROUTE_BLOCK = 5,
             ROUTE_ONE = 6 };
constexpr uint32_t kOneMaxFrames = 64;

// Launch the LZ4 frame decoder over nframes frames (asynchronous on stream).
// d_fail_at (optional) receives, per frame, the output offset of the block
// whose decode failed.  tune: tuning builds only (0 = production kernels).
int launch_lz4_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                      uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at,
                      hipStream_t stream, int route = ROUTE_AUTO, int tune = 0);

// Scratch of the two-phase decoder (lz4_split.hip): per-frame item slot
// offsets and counts, and the items themselves (one u32 per LZ4 sequence).
// Block route (big multi-block frames): the block plan walks
// each eligible frame's block headers and gives every LZ4 block a job; the
// lean parse takes one lane per job at the output offset the block would
// start at if every block before it decodes to the frame's maximum block size
// (what LZ4F writers produce); the chunk parse accepts a frame whose jobs all
// parsed cleanly at those offsets and re-parses any other; the execute reads
// an accepted frame's items block by block.
struct BlockJob {
    uint32_t f;          // frame, or kNoJob: a slot no lane parses
    uint32_t hpos;       // block header, frame-relative
    uint32_t stop;       // the next header (hpos + 4 + block size)
    uint32_t slot_off;   // the job's item slots, relative to rec_base[f]
    uint32_t slot_cap;
    uint32_t info;       // block size id | independent blocks << 8
    uint32_t bop;        // speculative output offset (job index x max block)
    uint32_t pad;
};
struct BlockRes {
    uint32_t n;    // items
    uint32_t op;   // output offset the block ended at
    int32_t st;    // ST_OK: parsed up to `stop`, every rule checked
    uint32_t pad;
};
static_assert(sizeof(BlockJob) == 32 && sizeof(BlockRes) == 16, "block job layout");
constexpr uint32_t kNoJob = 0xFFFFFFFFu;
constexpr uint32_t kMaxBlockJobs = 64;   // blocks per frame the route takes

struct SplitScratch {
    uint64_t *rec_base = nullptr;   // [frames_cap]
    uint32_t *nitems = nullptr;     // [frames_cap]
    uint64_t *items = nullptr;      // [items_cap], 8-byte items
    uint64_t *total = nullptr;      // host-mapped: item slots the last plan needed
    uint32_t *redo = nullptr;      // device flag: frames out of order, slots by scan
    uint32_t frames_cap = 0;
    uint64_t items_cap = 0;
    // block route (allocated on first use)
    uint32_t *bfirst = nullptr;     // [bframes_cap] first job of frame f, or kNoJob
    uint32_t *bcount = nullptr;     // [bframes_cap]
    uint32_t *njobs = nullptr;      // device counter
    BlockJob *jobs = nullptr;       // [jobs_cap]
    BlockRes *jres = nullptr;       // [jobs_cap]
    uint32_t bframes_cap = 0, jobs_cap = 0;
    // the one-frame route's block-parallel execute: each job's phase-A
    // origins (64 Ki u16) and taint bits (2 Ki words), allocated on first use
    uint16_t *borg = nullptr;       // [borg_cap][65536]
    uint32_t *btaint = nullptr;     // [borg_cap][2048]
    uint32_t borg_cap = 0;
};

// Item slots frame descriptors need (host-side mirror of the plan kernel).
uint64_t split_items_needed(const FrameDesc *h_desc, uint32_t n);
// Grow scratch to at least (frames, items); stream-ordered.  0 on success.
int split_scratch_reserve(SplitScratch *s, uint32_t frames, uint64_t items, hipStream_t stream);
void split_scratch_free(SplitScratch *s);

// Parse routing of the two-phase decoder: frames of >= chunk_min compressed
// bytes take lz4_chunk_kernel, of [lean_min, chunk_min) lz4_lean_kernel,
// shorter ones lz4_scan_kernel.
struct ParseRoute {
    uint32_t chunk_min, lean_min;
};
ParseRoute parse_route(uint32_t nframes, int route);
// The parse kernel a frame of c_size compressed bytes takes in a batch of
// nframes (what a kernel trace shows), for tooling.
const char *parse_kernel_name(uint32_t nframes, uint32_t c_size, int route = ROUTE_AUTO);

// stop_last: the batch's last frame is executed only until it has produced
// that many bytes (its status still covers the whole frame; the reader's
// no-cache requests ending inside it).
// Two-phase decoder with caller-owned scratch (must cover nframes and the
// frames' item slots; frames that do not fit are decoded by the wave kernel).
// stages: bitmask 1 plan, 2 parse, 4 execute, 8 hand-offs (tuning builds
// time subsets).
// A lone frame's results straight into the reader's pinned buffers from the
// one-frame route's execute (no download kernel, no launch behind it): its
// status and fail_at to h_status[0..1], decoded bytes [h_from, h_from +
// h_len) to h_out (16-aligned, 15 bytes of slack), then `seq` to h_flag --
// the device mappings of the slot's buffers (download_flagged's word).
struct HostPost {
    uint32_t *h_status = nullptr;
    uint8_t *h_out = nullptr;
    uint32_t h_from = 0, h_len = 0;
    uint32_t *h_flag = nullptr;
    uint32_t seq = 0;
};
int launch_lz4_split(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at,
                     hipStream_t stream, SplitScratch *s, int route = ROUTE_AUTO, int stages = 15,
                     int tune = 0, uint32_t stop_last = 0xFFFFFFFFu, uint32_t max_dsize = 0xFFFFFFFFu,
                     const HostPost *post = nullptr, bool *posted = nullptr, bool in_order = false);
// (in_order: the caller laid the frames out in order in d_comp -- the
// one-frame route's chunk parse then does the plan's work, no plan launch.
// max_dsize: the batch's largest decoded frame when the caller knows it --
// the one-frame route then skips the wave execute for frames of <= 64 KiB.
// post: a one-frame batch's results to the host from its execute, when the
// batch takes that route (*posted = true; else the caller downloads))

// Item slots of a frame in the split decoder's scratch.  An item is 8 bytes;
// a sequence takes one (two when extended), a stored block two.  LZ4 data
// spends >= 3 compressed bytes per sequence and typically 8-25; one slot per
// 8 compressed bytes (+32) covers all but pathological frames, which do not
// fit and are decoded by the wave kernel instead (parse reports ST_NOT_RUN).
__host__ __device__ __forceinline__ uint32_t slots_of(uint32_t c_size)
{
    return (c_size / 8 + 32 + 3) & ~3u;
}

// Decoder selection (env ZSEEK_HIP_KERNEL = split | wave; default auto).
enum : int { ENGINE_AUTO = 0, ENGINE_SPLIT, ENGINE_WAVE };

// Per-stage launch timing: stages [plan, parse, execute, hand-off]; marks
// 0..4 are the boundaries, recorded as HIP events on the launch's stream
// while enabled.  Slots kTimedStages.. are per-kernel spans a launch sums
// over its chunks (zstd: frame, sequence, Huffman and execute kernels, each
// on the stream it runs on): kernel_span_begin returns the begin event
// (null when timing is off), kernel_span_end closes it.
constexpr int kTimedStages = 4;
constexpr int kTimedSlots = 8;
enum : int { SPAN_ZFRAME = 4, SPAN_ZSEQ = 5, SPAN_ZHUF = 6, SPAN_ZEXEC = 7 };
void stage_mark(int boundary, hipStream_t stream);
hipEvent_t kernel_span_begin(hipStream_t stream);
void kernel_span_end(int slot, hipEvent_t begin, hipStream_t stream);

// HIP streams and events of reader slots and writers: created on the current
// device (low = the lowest stream priority), destroyed drained at release;
// env ZSEEK_HIP_POOL=1 recycles them process-wide instead (round 3's
// workaround for a heap corruption whose cause was elsewhere).
hipError_t hip_stream_get(hipStream_t *s, bool low);
void hip_stream_put(hipStream_t s);
hipError_t hip_event_get(hipEvent_t *e);
void hip_event_put(hipEvent_t e);
int kernel_timing(int on);
int kernel_times(double *ms, int cap);
int lz4_engine();
int lz4_pick_engine(uint32_t nframes);   // never ENGINE_AUTO

// Execute phase (seq_exec.hip): one wave per frame, linear per-wave LDS
// stage, DPP scans, piece descriptors.  version: tuning builds only (0 = the
// production kernel).
// With `blk` (the block route's scratch), frames with a job list read their
// items job by job.
int launch_seq_exec(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items,
                    const uint32_t *nitems, const int32_t *d_status, hipStream_t stream,
                    int version = 0, const SplitScratch *blk = nullptr, uint32_t stop_last = 0xFFFFFFFFu,
                    uint32_t min_dsize = 0);
// The one-frame route's execute (seq_exec.hip): one frame of <= 64 KiB
// decoded per 1,024-thread workgroup, output staged whole in LDS; bigger
// frames are left to launch_seq_exec(..., min_dsize = 65537).  handoff: the
// kernel also decodes its frames the parse left ST_NOT_RUN (the wave
// decoder), so no hand-off pass is needed for them.
int launch_seq_exec_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                           const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                           int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t stop_last,
                           bool handoff, const uint8_t *lit = nullptr, const HostPost *post = nullptr);
// ... and its frames of more than 64 KiB (the one-frame route's big frames):
// one per workgroup through a sliding 64 KiB window, items job by job for a
// frame the block route accepted (blk, may be null); handoff as above.
int launch_seq_exec_big(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                        const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                        int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t stop_last,
                        bool handoff, const SplitScratch *blk, uint32_t skip_jobs = 0);
// ... the frames the block route accepted whose jobs are all below
// blk->borg_cap (the origin scratch), block-parallel: a workgroup per job of
// blk (a grid of `jobs`), then launch_seq_exec_big(..., blk->borg_cap) for
// the rest (seq_exec.hip, seq_exec_blocks_kernel).
int launch_seq_exec_blocks(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                           const uint64_t *rec_base, const uint64_t *items, hipStream_t stream, uint32_t stop_last,
                           const SplitScratch *blk, uint32_t jobs);
int launch_seq_exec_seg(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out,
                        const uint64_t *rec_base, const uint64_t *items, const uint32_t *nitems,
                        const int32_t *d_status, hipStream_t stream, const SplitScratch *blk);

// Execute phase over items whose literal runs come from a literal scratch
// laid out like the output (zstd): frame f's literals at lit + d_off[f].
// one: the one-frame route's execute (a workgroup per frame of <= 64 KiB;
// max_dsize, the batch's largest frame, says whether a wave kernel for bigger
// ones is needed too).
int launch_seq_exec_lit(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *lit,
                        uint8_t *d_out, const uint64_t *rec_base, const uint64_t *items,
                        const uint32_t *nitems, int32_t *d_status, hipStream_t stream, bool one = false,
                        uint32_t max_dsize = 0xFFFFFFFFu, uint32_t stop_last = 0xFFFFFFFFu);

// zstd decoder (zstd_decode.hip): plan (item bounds -> rec_base[0..n]) and
// decode (frame kernel -> items + literal scratch, execute, checksums).
struct ZstdScratch {
    uint32_t *bound = nullptr;     // per-frame item bound
    uint32_t *bblk = nullptr;      // per-frame block count (plan)
    uint64_t *rec_base = nullptr;  // n + 1 item slot offsets
    uint64_t *blk_base = nullptr;  // n + 1 block slot offsets
    uint32_t *nitems = nullptr;
    uint64_t *ck = nullptr;        // per-frame checksum request
    uint32_t *stop = nullptr;      // per-frame op index the sequence replay stopped at
    uint8_t *lit = nullptr;        // literal scratch (output-sized + 64)
    uint64_t *items = nullptr;
    uint8_t *ops = nullptr;        // per-frame op lists (4 per block + 4), 32 B each
    uint8_t *hjobs = nullptr;      // Huffman stream jobs, 4 per block, 32 B each
    uint8_t *slots = nullptr;      // per-block decoding tables (kZSlot bytes each)
    uint8_t *hbad = nullptr;       // per Huffman stream: 1 = corrupt
    // [0] item total, [1] output extent, [2] blocks, [3] largest frame (d_size), [4 + k] blk_base
    // at chunk boundary k (zstd_decode.hip: the decode runs in chunks); past
    // those, zstd_one_kernel's finished-workgroup counter (zero between launches)
    uint64_t *d_total = nullptr;
    uint64_t *total = nullptr;     // pinned host copy of d_total
    uint64_t *h_plan = nullptr;    // pinned: a host plan's rec_base then blk_base (zstd_decode_frames_host)
    uint64_t h_plan_cap = 0;       //   (u64 entries)
    uint64_t *d_plan = nullptr;    // its device copy (one upload), 2 (kOneMaxFrames + 1) entries
    hipStream_t side = nullptr;    // the Huffman kernel's stream (beside the sequence replay)
    hipStream_t sq = nullptr;      // the sequence kernel's stream
    static constexpr int kChunks = 8;   // most chunks a decode runs in
    hipEvent_t ev_f[kChunks] = {}, ev_s[kChunks] = {}, ev_h[kChunks] = {};   // per chunk: frame / seq / Huffman done
    int side_dev = -1;   // the device the side set belongs to (pooled, zstd_decode.hip)
    uint32_t frames_cap = 0;
    uint64_t lit_cap = 0, items_cap = 0, blocks_cap = 0, ops_cap = 0;
};
int zstd_scratch_reserve(ZstdScratch *s, uint32_t frames, uint64_t out_bytes, uint64_t items,
                         uint64_t blocks, hipStream_t stream);
void zstd_scratch_free(ZstdScratch *s);
// Teardown in three steps for an owner with streams of its own: the
// scratch's memory (after draining its streams; streams and events kept),
// then its streams, then (zstd_scratch_free) its events -- memory goes while
// every stream that used it exists, streams before the events recorded on
// them
void zstd_scratch_release_memory(ZstdScratch *s);
void zstd_scratch_drop_streams(ZstdScratch *s);
int launch_zstd_plan(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     ZstdScratch *s, hipStream_t stream);
// d_fail_at (optional): per failed frame, the output offset of its failing
// block's start (its end for the end-of-frame checks); the execute still
// writes the bytes before it.
// stop_last: the batch's last frame executed only up to that many bytes (a
// no-cache read's end; its checksum then not checked); cks false: no frame
// carries a content checksum (a host plan saw them all), no check launch
int launch_zstd_decode(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                       uint8_t *d_out, int32_t *d_status, ZstdScratch *s, hipStream_t stream,
                       uint32_t *d_fail_at = nullptr, uint32_t stop_last = 0xFFFFFFFFu, bool cks = true);
// host_io.hip: a host -> device upload of <= kUploadSmallMax bytes from
// pinned memory (hipHostMalloc'd, both buffers with >= 15 bytes of slack past
// `bytes`; h_src_dev its device mapping, hipHostGetDevicePointer) as a kernel
// on `stream` (no DMA-engine hand-off before the next kernel); larger ones
// (or no mapping) through hipMemcpyAsync.  0 or -1.
constexpr size_t kUploadSmallMax = 512u << 10;
int upload_small(void *d_dst, const void *h_src, const void *h_src_dev, size_t bytes, hipStream_t stream);
// ... and the download: nst status words d_status -> h_status, then len bytes
// d_src (any alignment, 19 readable bytes past the end) -> h_out (pinned,
// 16-aligned, 15 writable bytes of slack) as one kernel when len <=
// kDownloadSmallMax, else two hipMemcpyAsync.  0 or -1.
constexpr size_t kDownloadSmallMax = 256u << 10;
int download_small(uint32_t *h_status, void *h_status_dev, const uint32_t *d_status, uint32_t nst, uint8_t *h_out,
                   void *h_out_dev, const uint8_t *d_src, size_t len, hipStream_t stream);
// ... or, for a request's small batch, as one workgroup that then writes
// `seq` to a pinned word (hflag_dev: its device mapping) once every byte is
// in host memory: the host may spin on it instead of synchronizing with the
// stream.  0 (flag posted at the end), 1 (too big: nothing launched, use
// download_small), -1.
constexpr size_t kFlagMax = 64u << 10;
constexpr uint32_t kFlagMaxStatus = 4096;
int download_flagged(uint32_t *h_status, void *h_status_dev, const uint32_t *d_status, uint32_t nst, uint8_t *h_out,
                     void *h_out_dev, const uint8_t *d_src, size_t len, void *hflag_dev, uint32_t seq,
                     hipStream_t stream);
// plan + synchronize + reserve + decode (stop_last as launch_zstd_decode)
int zstd_decode_frames(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                       uint8_t *d_out, int32_t *d_status, ZstdScratch *s, hipStream_t stream,
                       uint32_t *d_fail_at = nullptr, uint32_t stop_last = 0xFFFFFFFFu);
// The same for a request's few frames whose compressed bytes are also in host
// memory (h_desc / h_comp: the reader's pinned upload, the same layout as
// d_desc / d_comp): the plan -- zstd_plan_kernel's per-frame bounds, the scans,
// the totals -- computed on the host, so the decode needs no plan launch and
// no synchronization.  nframes <= kOneMaxFrames.
int zstd_decode_frames_host(const FrameDesc *h_desc, const uint8_t *h_comp, const FrameDesc *d_desc,
                            uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                            ZstdScratch *s, hipStream_t stream, uint32_t *d_fail_at,
                            uint32_t stop_last = 0xFFFFFFFFu);
// ... in two steps, for a caller that uploads the plan with its own bytes:
// the plan (2 (nframes + 1) u64: item slot offsets, then block slot offsets)
// into h_plan before the upload, then the decode with the plan's device copy
struct ZstdHostPlan {
    uint64_t items, blocks, extent, dmax;
    bool cks;   // some frame carries a content checksum
};
void zstd_host_plan(const FrameDesc *h_desc, const uint8_t *h_comp, uint32_t nframes, uint64_t *h_plan,
                    ZstdHostPlan *P);
int zstd_decode_frames_planned(const ZstdHostPlan &P, const uint64_t *d_plan, const FrameDesc *d_desc,
                               uint32_t nframes, const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                               ZstdScratch *s, hipStream_t stream, uint32_t *d_fail_at,
                               uint32_t stop_last = 0xFFFFFFFFu);

// Parse phase, streaming lane-per-frame (lz4_scan.hip), for the frames
// under max_csize compressed bytes (the short frames of config 3).
int launch_lz4_scan(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    const uint64_t *rec_base, uint64_t capacity, uint64_t *items,
                    uint32_t *nitems, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream,
                    uint32_t max_csize = 0xFFFFFFFFu);

// Parse phase, streaming lane-per-frame with a one-sequence fast step
// (lz4_lean.hip), frames of [min_csize, max_csize) compressed bytes: the
// outputs of launch_lz4_chunk (items without padding).  diag: tuning builds.
int launch_lz4_lean(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    const uint64_t *rec_base, uint64_t capacity, uint64_t *items, uint32_t *nitems,
                    int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t max_csize,
                    int diag = 0, uint32_t min_csize = 0);
// Frames under this many compressed bytes take the older lz4_scan_kernel
// (its direct item stores beat the lean kernel's line flush on short frames:
// 4 KiB frames 5.68 vs 6.71 ms per launch, config 3)
constexpr uint32_t kLeanMinCsize = 12288;
// Block route parse: lane per job of s->jobs (the first *s->njobs), all
// lanes idle when fewer than min_jobs jobs were planned.
int launch_lz4_lean_blocks(const FrameDesc *d_desc, const uint8_t *d_comp, const uint64_t *rec_base,
                           uint64_t capacity, uint64_t *items, const SplitScratch *s, uint32_t lanes,
                           uint32_t min_jobs, hipStream_t stream);

// The one-frame route's big frames (lz4_chunk.hip): each of the first
// *s->njobs block-plan jobs (a grid of `jobs` workgroups) parsed by a
// workgroup, the one-frame route's chunk parse over the block staged in LDS,
// results into s->jres as the block route's lean parse gives them.
int launch_lz4_job_parse(const FrameDesc *d_desc, const uint8_t *d_comp, const uint64_t *rec_base, uint64_t capacity,
                         uint64_t *items, const SplitScratch *s, uint32_t jobs, hipStream_t stream);

// Parse phase, one wave per frame, chunk-parallel (lz4_chunk.hip): the same
// outputs as launch_lz4_scan for the frames of min_csize compressed bytes and
// more (other frames are left to lz4_scan_kernel), items without padding.
// With `blk`: a frame with a job list is accepted from its jobs' results
// (when at least min_jobs were planned and every job parsed cleanly at its
// speculative offset) or parsed here, its job list dropped.
// `one` (the one-frame route): one frame per workgroup, the frame staged
// whole in LDS when it fits (lz4_chunk.hip, ONE); its `blk` holds the big
// frames' jobs (launch_lz4_job_parse).
int launch_lz4_chunk(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                     const uint64_t *rec_base, uint64_t capacity, uint64_t *items, uint32_t *nitems,
                     int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t min_csize,
                     SplitScratch *blk = nullptr, uint32_t min_jobs = 0, bool one = false,
                     uint64_t *solo_total = nullptr);
// (one && solo_total: the batch has no plan launch -- one frame, or frames
// the caller laid out in order; each workgroup lays its frame's slots out by
// the plan's in-order formula and the last reports their total there)
// Frames of at least chunk_parse_min(nframes) compressed bytes go to the
// chunk parse: with >= 32768 frames the lane-per-frame scan has a lane for
// every frame it needs and wins on 64 KiB frames (2.07 vs 4.18 ms parse at
// config 2); smaller batches and bigger frames leave its lanes idle
// (1 MiB frames: 4,096 chains; 256 MiB batches: 4,096 frames).
// Env ZSEEK_PARSE=scan|chunk forces one parse for every frame.
uint32_t chunk_parse_min(uint32_t nframes);

// Wave-per-frame kernel over only the frames whose status is ST_NOT_RUN
// (the split decoder's hand-offs).
int launch_lz4_wave_deferred(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                             uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at,
                             hipStream_t stream);

// Wave-per-frame kernel (lz4_wave.hip): 4 KiB LDS ring, 4 waves per workgroup.
int launch_lz4_wave(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream);

#ifdef ZSK_TUNING
// Tuning builds (libzseek_tune.so, scripts/kbench.py): experimental launch
// variants and diagnostics, never in the product library.
int launch_lz4_frames_variant(int variant, const FrameDesc *d_desc, uint32_t nframes,
                              const uint8_t *d_comp, uint8_t *d_out, int32_t *d_status,
                              hipStream_t stream);
#endif

const char *status_name(int32_t st);

// Seek-table checksums (frame_check.hip): frames whose status is ST_OK and
// whose decoded bytes' XXH64 low 32 bits differ from d_want[f] get
// ST_SEEK_CHECKSUM.
int launch_frame_checksums(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_out,
                           const uint32_t *d_want, int32_t *d_status, hipStream_t stream);

}   // namespace zsk

#endif
