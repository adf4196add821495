// tools.cpp — bench/test input tooling (libzseek_tools.so), not the hot path.
//
//   zsk_tool_synth          the SURVEY.md §8d synthetic buffer(N): 64 MiB
//                           chunks gen(64 MiB, seed = 1 + chunk), generated in
//                           parallel (chunks are independent).
//   zsk_tool_lz4_seekable   a seekable LZ4 file image of a buffer, frames
//                           compressed in parallel with liblz4 exactly as the
//                           reference writer's direct path does when every
//                           zseek_write is frame_size bytes
//                           (/root/reference/src/compress.c:737-786: prefs
//                           {level, autoFlush=1, max64KB}, no content size;
//                           a final short frame goes through the buffered path
//                           and carries its content size, :463-518).
//   zsk_tool_zstd_seekable  same for zstd (ZSTD_compress2, level/strategy as
//                           compress.c:58-91, single worker), with the
//                           libzstd the reference writer is built against
//                           (1.4.9 under /opt/conda, opened by path into a
//                           local scope) when present, else the linked one;
//                           zsk_tool_zstd_version names the one used.
//   zsk_tool_open_mem       a reader over an in-memory image with a C pread
//   zsk_tool_close_mem      callback (memcpy), opened through the
//                           zseek_reader_open_full / close of EITHER library
//                           (ours, or the reference build in oracle/_ref):
//                           both share the zseek.h ABI, so the same callback
//                           and the same timing loop serve both sides.
//   zsk_tool_latency        per-request wall time of `count`-byte reads at
//                           given offsets (a request loops on short reads, as
//                           test/example.c:63-80 does).
//   zsk_tool_read_all       wall time of reading [0, size) with one call
//                           (looping on short reads).
#include <dlfcn.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/types.h>
#include <time.h>
#include <unistd.h>

#include <atomic>
#include <map>
#include <mutex>
#include <thread>
#include <type_traits>
#include <vector>

#include <lz4frame.h>
#include <zstd.h>

#define ZSK_TOOL extern "C" __attribute__((visibility("default")))

namespace {

constexpr size_t kSynthChunk = 64u << 20;

void gen(uint8_t *out, size_t n, uint64_t seed)
{
    uint64_t s = seed;
    auto next = [&s]() {
        s += 0x9E3779B97F4A7C15ULL;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    };
    size_t i = 0;
    while (i < n) {
        uint64_t r = next();
        if (i >= 65536 && r % 100 < 52) {
            size_t len = 4 + (size_t)((r >> 8) % 69);
            size_t off = 1 + (size_t)((r >> 24) % 8192);
            if (off > i)
                off = i;
            for (size_t k = 0; k < len && i < n; k++, i++)
                out[i] = out[i - off];
        } else {
            size_t len = 1 + (size_t)((r >> 8) % 48);
            for (size_t k = 0; k < len && i < n; k++, i++)
                out[i] = (uint8_t)(0x20 + next() % 64);
        }
    }
}

template <typename F>
void parallel_for(size_t n, int threads, F fn)
{
    if (threads < 1)
        threads = 1;
    std::atomic<size_t> next{0};
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; t++)
        pool.emplace_back([&]() {
            for (size_t i; (i = next.fetch_add(1)) < n;)
                fn(i);
        });
    for (auto &th : pool)
        th.join();
}

void put32(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v;
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)(v >> 16);
    p[3] = (uint8_t)(v >> 24);
}

// frames compressed into per-frame slots, then packed + seek table appended
template <typename Compress>
int seekable(const uint8_t *in, size_t n, size_t frame_size, int threads, size_t slot,
             uint8_t *out, size_t out_cap, size_t *out_len, Compress compress)
{
    if (frame_size == 0)
        return -1;
    size_t nf = (n + frame_size - 1) / frame_size;
    std::vector<uint8_t> tmp(nf * slot);
    std::vector<size_t> csize(nf, 0);
    std::atomic<int> bad{0};
    parallel_for(nf, threads, [&](size_t i) {
        size_t a = i * frame_size, len = n - a < frame_size ? n - a : frame_size;
        size_t c = compress(tmp.data() + i * slot, slot, in + a, len, len < frame_size);
        if (c == 0)
            bad = 1;
        csize[i] = c;
    });
    if (bad)
        return -1;
    size_t total = 0;
    for (size_t c : csize)
        total += c;
    size_t table = 8 + 8 * nf + 9;
    if (total + table > out_cap)
        return -1;
    size_t at = 0;
    for (size_t i = 0; i < nf; i++) {
        memcpy(out + at, tmp.data() + i * slot, csize[i]);
        at += csize[i];
    }
    uint8_t *t = out + at;
    put32(t, 0x184D2A5Eu);
    put32(t + 4, (uint32_t)(table - 8));
    for (size_t i = 0; i < nf; i++) {
        size_t a = i * frame_size, len = n - a < frame_size ? n - a : frame_size;
        put32(t + 8 + 8 * i, (uint32_t)csize[i]);
        put32(t + 12 + 8 * i, (uint32_t)len);
    }
    put32(t + 8 + 8 * nf, (uint32_t)nf);
    t[12 + 8 * nf] = 0;
    put32(t + 13 + 8 * nf, 0x8F92EAB1u);
    *out_len = at + table;
    return 0;
}

LZ4F_preferences_t lz4_prefs(int level, size_t content)
{
    LZ4F_preferences_t p;
    memset(&p, 0, sizeof(p));
    p.compressionLevel = level;
    p.autoFlush = 1;
    p.frameInfo.blockSizeID = LZ4F_max64KB;
    p.frameInfo.contentSize = content;
    return p;
}

}   // namespace

ZSK_TOOL void zsk_tool_synth(uint8_t *out, size_t n, int threads)
{
    size_t chunks = (n + kSynthChunk - 1) / kSynthChunk;
    parallel_for(chunks, threads, [&](size_t c) {
        size_t a = c * kSynthChunk;
        gen(out + a, n - a < kSynthChunk ? n - a : kSynthChunk, 1 + c);
    });
}

ZSK_TOOL void zsk_tool_gen(uint8_t *out, size_t n, uint64_t seed)
{
    gen(out, n, seed);
}

ZSK_TOOL size_t zsk_tool_lz4_seekable_bound(size_t n, size_t frame_size)
{
    LZ4F_preferences_t p = lz4_prefs(0, frame_size);
    size_t nf = frame_size ? (n + frame_size - 1) / frame_size : 0;
    return nf * LZ4F_compressFrameBound(frame_size, &p) + 8 + 8 * nf + 9;
}

ZSK_TOOL int zsk_tool_lz4_seekable(const uint8_t *in, size_t n, size_t frame_size, int level,
                                   int threads, uint8_t *out, size_t out_cap, size_t *out_len)
{
    LZ4F_preferences_t pb = lz4_prefs(level, frame_size);
    size_t slot = LZ4F_compressFrameBound(frame_size, &pb);
    return seekable(in, n, frame_size, threads, slot, out, out_cap, out_len,
                    [level](uint8_t *dst, size_t cap, const uint8_t *src, size_t len,
                            bool last_short) -> size_t {
                        LZ4F_preferences_t p = lz4_prefs(level, last_short ? len : 0);
                        size_t c = LZ4F_compressFrame(dst, cap, src, len, &p);
                        return LZ4F_isError(c) ? 0 : c;
                    });
}

// A seekable LZ4 image whose frames use LZ4F options the reference writer
// never sets (compress.c:203-207 fixes max64KB, autoFlush, nothing else) but
// its reader accepts through LZ4F_decompress (decompress.c:752-773): block
// size id 4..7, linked / independent blocks, content checksum, block
// checksums, content size, dictID.  One LZ4F_compressFrame per frame (which
// makes a frame that fits one block independent, as liblz4 does).
ZSK_TOOL int zsk_tool_lz4_seekable_ex(const uint8_t *in, size_t n, size_t frame_size, int level,
                                      int bsid, int independent, int content_checksum,
                                      int block_checksum, int content_size, unsigned dict_id,
                                      int threads, uint8_t *out, size_t out_cap, size_t *out_len)
{
    auto prefs = [=](size_t len) {
        LZ4F_preferences_t p = lz4_prefs(level, content_size ? len : 0);
        p.frameInfo.blockSizeID = (LZ4F_blockSizeID_t)bsid;
        p.frameInfo.blockMode = independent ? LZ4F_blockIndependent : LZ4F_blockLinked;
        p.frameInfo.contentChecksumFlag = content_checksum ? LZ4F_contentChecksumEnabled
                                                           : LZ4F_noContentChecksum;
        p.frameInfo.blockChecksumFlag = block_checksum ? LZ4F_blockChecksumEnabled : LZ4F_noBlockChecksum;
        p.frameInfo.dictID = dict_id;
        return p;
    };
    LZ4F_preferences_t pb = prefs(frame_size);
    size_t slot = LZ4F_compressFrameBound(frame_size, &pb);
    if (slot * ((n + frame_size - 1) / frame_size) + 8 + 8 * ((n + frame_size - 1) / frame_size) + 9 > out_cap)
        return -1;
    return seekable(in, n, frame_size, threads, slot, out, out_cap, out_len,
                    [prefs](uint8_t *dst, size_t cap, const uint8_t *src, size_t len, bool) -> size_t {
                        LZ4F_preferences_t p = prefs(len);
                        size_t c = LZ4F_compressFrame(dst, cap, src, len, &p);
                        return LZ4F_isError(c) ? 0 : c;
                    });
}

namespace {
// The compressor's libzstd: the reference's pinned 1.4.9 (SURVEY.md §8c,
// /root/reference/meson.build:10-11) by full path in a link namespace of its
// own (dlmopen), else the linked one.  A plain dlopen mapped the 1.4.9 copy
// beside the system libzstd.so.1 this library links, but left the copy's
// calls to its own exported functions to the global scope, where 1.4.8's
// definitions come first: a 1.4.9 CCtx reset by 1.4.8 code (a SIGSEGV in
// free under ZSTD_CCtx_reset, round 4, config-5 input under rocprofv3).
struct ZstdApi {
    unsigned (*version)(void) = ZSTD_versionNumber;
    size_t (*bound)(size_t) = ZSTD_compressBound;
    ZSTD_CCtx *(*create)(void) = ZSTD_createCCtx;
    size_t (*reset)(ZSTD_CCtx *, ZSTD_ResetDirective) = ZSTD_CCtx_reset;
    size_t (*set)(ZSTD_CCtx *, ZSTD_cParameter, int) = ZSTD_CCtx_setParameter;
    size_t (*compress2)(ZSTD_CCtx *, void *, size_t, const void *, size_t) = ZSTD_compress2;
    unsigned (*is_error)(size_t) = ZSTD_isError;
};

const ZstdApi &zstd_api()
{
    static const ZstdApi api = [] {
        ZstdApi a;
        const char *path = getenv("ZSEEK_TOOLS_LIBZSTD");
        void *h = dlmopen(LM_ID_NEWLM, path ? path : "/opt/conda/lib/libzstd.so.1.4.9", RTLD_NOW | RTLD_LOCAL);
        if (!h)
            return a;
        ZstdApi b;
        bool ok = true;
        auto get = [&](auto &fn, const char *name) {
            void *p = dlsym(h, name);
            ok = ok && p;
            if (p)
                fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(p);
        };
        get(b.version, "ZSTD_versionNumber");
        get(b.bound, "ZSTD_compressBound");
        get(b.create, "ZSTD_createCCtx");
        get(b.reset, "ZSTD_CCtx_reset");
        get(b.set, "ZSTD_CCtx_setParameter");
        get(b.compress2, "ZSTD_compress2");
        get(b.is_error, "ZSTD_isError");
        return ok ? b : a;
    }();
    return api;
}
}   // namespace

ZSK_TOOL unsigned zsk_tool_zstd_version(void)
{
    return zstd_api().version();
}

ZSK_TOOL size_t zsk_tool_zstd_seekable_bound(size_t n, size_t frame_size)
{
    size_t nf = frame_size ? (n + frame_size - 1) / frame_size : 0;
    return nf * zstd_api().bound(frame_size) + 8 + 8 * nf + 9;
}

ZSK_TOOL int zsk_tool_zstd_seekable(const uint8_t *in, size_t n, size_t frame_size, int level,
                                    int strategy, int threads, uint8_t *out, size_t out_cap,
                                    size_t *out_len)
{
    const ZstdApi &Z = zstd_api();
    size_t slot = Z.bound(frame_size);
    return seekable(in, n, frame_size, threads, slot, out, out_cap, out_len,
                    [level, strategy, &Z](uint8_t *dst, size_t cap, const uint8_t *src, size_t len,
                                          bool) -> size_t {
                        thread_local ZSTD_CCtx *cctx = nullptr;
                        if (!cctx)
                            cctx = Z.create();
                        Z.reset(cctx, ZSTD_reset_session_and_parameters);
                        Z.set(cctx, ZSTD_c_compressionLevel, level);
                        Z.set(cctx, ZSTD_c_strategy, strategy);
                        size_t c = Z.compress2(cctx, dst, cap, src, len);
                        return Z.is_error(c) ? 0 : c;
                    });
}

// ---- in-memory readers and timing loops (bench.py latency / end-to-end) ----
namespace {
struct MemFile {
    const uint8_t *p;
    size_t n;
};
struct ReadFile {   // zseek_read_file_t (zseek.h:109-116)
    void *user_data;
    ssize_t (*pread)(void *, size_t, size_t, void *, void *);
    ssize_t (*fsize)(void *, void *);
};
typedef void *(*open_full_t)(ReadFile, size_t, void *, char *);
typedef bool (*close_t)(void *, void *, char *);
typedef ssize_t (*pread_t)(void *, void *, size_t, size_t, void *, char *);

ssize_t mem_pread(void *data, size_t size, size_t offset, void *user_data, void *)
{
    const MemFile *f = (const MemFile *)user_data;
    if (offset >= f->n)
        return 0;
    size_t k = f->n - offset < size ? f->n - offset : size;
    memcpy(data, f->p + offset, k);
    return (ssize_t)k;
}

ssize_t mem_fsize(void *user_data, void *)
{
    return (ssize_t)((const MemFile *)user_data)->n;
}

std::mutex g_mem_mu;
std::map<void *, MemFile *> g_mem;

double now_s()
{
    timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}
}   // namespace

ZSK_TOOL void *zsk_tool_open_mem(void *open_full, const uint8_t *img, size_t n, size_t cache_size,
                                 char *errbuf)
{
    MemFile *f = new MemFile{img, n};
    void *r = ((open_full_t)open_full)(ReadFile{f, mem_pread, mem_fsize}, cache_size, nullptr, errbuf);
    if (!r) {
        delete f;
        return nullptr;
    }
    std::lock_guard<std::mutex> g(g_mem_mu);
    g_mem[r] = f;
    return r;
}

ZSK_TOOL bool zsk_tool_close_mem(void *close_fn, void *reader)
{
    bool ok = ((close_t)close_fn)(reader, nullptr, nullptr);
    std::lock_guard<std::mutex> g(g_mem_mu);
    auto it = g_mem.find(reader);
    if (it != g_mem.end()) {
        delete it->second;
        g_mem.erase(it);
    }
    return ok;
}

// ns_out[i] = wall time of request i; returns 0, or -1 at the first failing
// request (its index in *failed)
ZSK_TOOL int zsk_tool_latency(void *pread_fn, void *reader, const uint64_t *offs, size_t n,
                              size_t count, uint8_t *buf, uint64_t *ns_out, size_t *failed)
{
    pread_t pr = (pread_t)pread_fn;
    for (size_t i = 0; i < n; i++) {
        const double t0 = now_s();
        size_t done = 0;
        while (done < count) {
            ssize_t r = pr(reader, buf + done, count - done, offs[i] + done, nullptr, nullptr);
            if (r < 0) {
                *failed = i;
                return -1;
            }
            if (r == 0)
                break;
            done += (size_t)r;
        }
        ns_out[i] = (uint64_t)((now_s() - t0) * 1e9);
    }
    return 0;
}

ZSK_TOOL double zsk_tool_read_all(void *pread_fn, void *reader, uint8_t *buf, size_t size,
                                  size_t *got)
{
    pread_t pr = (pread_t)pread_fn;
    const double t0 = now_s();
    size_t done = 0;
    while (done < size) {
        ssize_t r = pr(reader, buf + done, size - done, done, nullptr, nullptr);
        if (r <= 0)
            break;
        done += (size_t)r;
    }
    *got = done;
    return now_s() - t0;
}

// ---- crash diagnostics (test sessions) -------------------------------------
// A native backtrace on SIGSEGV / SIGBUS / SIGABRT to stderr, then the handler
// that was installed before (Python's faulthandler prints the Python stack).
// Offsets into libzseek.so resolve with addr2line against the built library.
namespace {
struct sigaction g_prev[32];

void crash_bt(int sig)
{
    void *f[64];
    const int n = backtrace(f, 64);
    static const char m[] = "\n*** native backtrace ***\n";
    (void)!write(2, m, sizeof m - 1);
    backtrace_symbols_fd(f, n, 2);
    sigaction(sig, &g_prev[sig], nullptr);
    raise(sig);
}
}   // namespace

ZSK_TOOL int zsk_tool_install_backtrace(void)
{
    void *f[2];
    (void)backtrace(f, 2);   // loads the unwinder now, not inside a signal
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = crash_bt;
    sa.sa_flags = SA_NODEFER;
    for (int sig : {SIGSEGV, SIGBUS, SIGABRT})
        if (sigaction(sig, &sa, &g_prev[sig]) != 0)
            return -1;
    return 0;
}
