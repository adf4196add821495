// lz4_compress.hip — the reference writer's LZ4 frame compression on the GPU
// (gfx950), SURVEY §8f row 4.
//
// What it must reproduce, byte for byte: the writer compresses each seekable
// frame with one LZ4F_compressFrame call (compress.c:737-786 direct frames,
// :463-518 buffered ones) with prefs { level, autoFlush = 1, blockSizeID =
// LZ4F_max64KB } (compress.c:203-207) and contentSize = the writer's frame_uc
// counter (compress.c:741, :472).  For a frame of n <= 64 KiB liblz4 1.9.3
// writes: header (magic, FLG = 0x60 | 0x08 with a content size, BD = 0x40,
// [8-byte size], HC = XXH32 >> 8), one block made by LZ4F_makeBlock
// (fast encoder, capacity n - 1, stored raw with bit 31 when it does not
// fit), end mark.  The encoder is LZ4_compress_generic on a fresh state:
// 16-bit positions in a 2^13-entry table, hash = read32 * 2654435761 >> 19,
// search step growing by one every (64 * acceleration) misses, backward
// extension, an immediate re-match test after every match, and the
// limited-output checks that decide "stored".  oracle/lz4c_oracle.c is the
// CPU restatement (pinned against liblz4); this kernel follows it decision
// for decision.
//
// Mapping: one lane per frame (the parse is inherently serial: every table
// entry depends on all earlier probes).  The lane's 64 KiB table (8-byte
// position + input-word entries, zsk_lz4_compress_scratch_size) lives in HBM scratch (zeroed per launch: liblz4's fresh state); input is
// read in place; output goes through a little-endian dword packer so each
// lane issues dword stores.  A sequence is emitted whole once its match
// length is known, with both limited-output checks evaluated on the byte
// counts they would see.  Frames that do not fit are flagged and their raw
// block written by a second, wave-per-frame kernel (coalesced copy).
//
// Frames above 64 KiB (the reference example's 1 MiB frames, test/example.c)
// are linked: LZ4F_compressFrame then runs LZ4_compress_fast_continue over
// 64 KiB blocks on one stream.  The stream differs from the one-block state:
// a 2^12-entry table of 32-bit positions counted from the frame start, the
// 5-byte hash of an 8-byte read ((read64 << 24) * 889523592379 >> 52, the
// 64-bit build's byU32 hash), candidates more than 65535 back skipped without
// a compare, backward extension down to the frame start, match lengths
// stopping 5 bytes before the block end, and a stored block (capacity n - 1
// exceeded) still advancing the stream.  One lane walks the frame's blocks in
// order; a stored block rewinds the lane's packer and is copied inline.
//
// Lanes per wave: the parse is a serial chain of dependent table and input
// loads, so the launch spreads frames over about 2048 waves (2 per SIMD:
// fewer frames per wave, more independent chains) instead of filling every
// wave's 64 lanes; a batch of 1 MiB frames is 16 times fewer chains than
// the same bytes in 64 KiB frames.
//
// Algorithmic bytes per frame: n read + the frame's compressed size written.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <type_traits>

#include "../../include/zseek_hip.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

typedef uint32_t u32_ua __attribute__((aligned(1)));
typedef uint64_t u64_ua __attribute__((aligned(1)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_ua __attribute__((aligned(1)));

constexpr uint32_t kHashLog = 13;
constexpr uint32_t kTable = 1u << kHashLog;   // u16 entries per frame
constexpr uint32_t kMaxFrame = 65536;          // one block, independent
constexpr uint32_t kMaxLinkedFrame = 1u << 22;  // linked frames: ZSK_LZ4_COMPRESS_MAX_FRAME
constexpr uint32_t kLinkedHashLog = 12;
constexpr uint32_t kStoredFlag = 0x80000000u;
constexpr bool kDefaultVal = true;   // position + word entries: 103.7 ms against 125.8 (u16, 4 GiB)
constexpr uint32_t kDefaultWaves = 2048;   // 2 per SIMD (see "Lanes per wave")
constexpr int kDefaultProbe = 8;   // 8 / 16 / 32 measured 125.7 / 134.0 / 169.8 ms (4 GiB)

__device__ __forceinline__ uint32_t rd32(const uint8_t *p)
{
    return *reinterpret_cast<const u32_ua *>(p);
}

__device__ __forceinline__ uint64_t rd64(const uint8_t *p)
{
    return *reinterpret_cast<const u64_ua *>(p);
}

__device__ __forceinline__ uint32_t hash4(uint32_t v)
{
    return (v * 2654435761u) >> (32 - kHashLog);
}

// liblz4's byU32 hash on a 64-bit build: the low 5 bytes of an 8-byte read
__device__ __forceinline__ uint32_t hash5(uint64_t v)
{
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - kLinkedHashLog));
}

// Input word at p and the table index of the sequence starting there.
template <bool kLinked>
__device__ __forceinline__ uint32_t word_hash(const uint8_t *p, uint32_t &h)
{
    if constexpr (kLinked) {
        const uint64_t v = rd64(p);
        h = hash5(v);
        return (uint32_t)v;
    } else {
        const uint32_t v = rd32(p);
        h = hash4(v);
        return v;
    }
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r)
{
    return (x << r) | (x >> (32 - r));
}

// XXH32(seed 0) of a short header descriptor (2 or 10 bytes)
__device__ uint32_t xxh32_short(const uint8_t *p, uint32_t len)
{
    uint32_t h = 0x165667B1u + len;
    uint32_t i = 0;
    for (; i + 4 <= len; i += 4) {
        const uint32_t v = p[i] | p[i + 1] << 8 | p[i + 2] << 16 | (uint32_t)p[i + 3] << 24;
        h = rotl32(h + v * 0xC2B2AE3Du, 17) * 0x27D4EB2Fu;
    }
    for (; i < len; i++)
        h = rotl32(h + p[i] * 0x165667B1u, 11) * 0x9E3779B1u;
    h ^= h >> 15;
    h *= 0x85EBCA77u;
    h ^= h >> 13;
    h *= 0xC2B2AE3Du;
    h ^= h >> 16;
    return h;
}

// Little-endian byte packer over a 4-byte-aligned destination.
struct Packer {
    uint32_t *w;
    uint32_t acc;
    uint32_t k;   // bytes held in acc

    __device__ __forceinline__ void put(uint32_t b)
    {
        acc |= (b & 0xFF) << (8 * k);
        if (++k == 4) {
            *w++ = acc;
            acc = 0;
            k = 0;
        }
    }
    __device__ __forceinline__ void run(uint32_t len)   // 255 ... 255 rem
    {
        for (; len >= 255; len -= 255)
            put(255);
        put(len);
    }
    __device__ __forceinline__ void put4(uint32_t x)   // four bytes, little-endian
    {
        const uint64_t t = (uint64_t)x << (8 * k) | acc;
        *w++ = (uint32_t)t;
        acc = (uint32_t)(t >> 32);
    }
    // s[0..len), all inside the frame: 16-byte loads while they stay inside,
    // so a literal run costs one load latency per 16 bytes, not per byte
    __device__ __forceinline__ void copy(const uint8_t *s, uint32_t len)
    {
        uint32_t i = 0;
        for (; i + 32 <= len; i += 32) {   // two loads in flight
            const u32x4 v = *reinterpret_cast<const u32x4_ua *>(s + i);
            const u32x4 u = *reinterpret_cast<const u32x4_ua *>(s + i + 16);
            put4(v.x);
            put4(v.y);
            put4(v.z);
            put4(v.w);
            put4(u.x);
            put4(u.y);
            put4(u.z);
            put4(u.w);
        }
        if (i + 16 <= len) {
            const u32x4 v = *reinterpret_cast<const u32x4_ua *>(s + i);
            put4(v.x);
            put4(v.y);
            put4(v.z);
            put4(v.w);
            i += 16;
        }
        for (; i + 4 <= len; i += 4)
            put4(rd32(s + i));
        for (; i < len; i++)
            put(s[i]);
    }
    __device__ __forceinline__ void flush()
    {
        if (k)
            *w = acc;
    }
};

// Extra length bytes of a literal run / match code of value v (>= 15 -> 1 + (v-15)/255).
__device__ __forceinline__ uint32_t ext_bytes(uint32_t v)
{
    return v >= 15 ? (v - 15) / 255 + 1 : 0;
}

// Emit one sequence: token, literal-length bytes, literals, offset, match-length bytes.
__device__ __forceinline__ void emit_seq(Packer &o, const uint8_t *lits, uint32_t lit, uint32_t off,
                                         uint32_t mc)
{
    o.put((lit >= 15 ? 15u : lit) << 4 | (mc >= 15 ? 15u : mc));
    if (lit >= 15)
        o.run(lit - 15);
    o.copy(lits, lit);
    o.put(off);
    o.put(off >> 8);
    if (mc >= 15)
        o.run(mc - 15);
}

// Equal bytes of s[a..] and s[b..] before a reaches lim (b < a).
__device__ __forceinline__ uint32_t count_eq(const uint8_t *s, uint32_t a, uint32_t b, uint32_t lim)
{
    const uint32_t a0 = a;
    while (a + 32 <= lim) {   // 32 bytes per round trip
        const u32x4 x = *reinterpret_cast<const u32x4_ua *>(s + a) ^ *reinterpret_cast<const u32x4_ua *>(s + b);
        const u32x4 y =
            *reinterpret_cast<const u32x4_ua *>(s + a + 16) ^ *reinterpret_cast<const u32x4_ua *>(s + b + 16);
        if (x.x | x.y | x.z | x.w) {
            const uint32_t q = x.x ? 0 : x.y ? 4 : x.z ? 8 : 12;
            const uint32_t d = x.x ? x.x : x.y ? x.y : x.z ? x.z : x.w;
            return a - a0 + q + (__builtin_ctz(d) >> 3);
        }
        if (y.x | y.y | y.z | y.w) {
            const uint32_t q = y.x ? 16 : y.y ? 20 : y.z ? 24 : 28;
            const uint32_t d = y.x ? y.x : y.y ? y.y : y.z ? y.z : y.w;
            return a - a0 + q + (__builtin_ctz(d) >> 3);
        }
        a += 32;
        b += 32;
    }
    while (a + 16 <= lim) {
        const u32x4 x = *reinterpret_cast<const u32x4_ua *>(s + a) ^ *reinterpret_cast<const u32x4_ua *>(s + b);
        if (x.x | x.y | x.z | x.w) {
            const uint32_t q = x.x ? 0 : x.y ? 4 : x.z ? 8 : 12;
            const uint32_t d = x.x ? x.x : x.y ? x.y : x.z ? x.z : x.w;
            return a - a0 + q + (__builtin_ctz(d) >> 3);
        }
        a += 16;
        b += 16;
    }
    while (a + 4 <= lim) {
        const uint32_t x = rd32(s + a) ^ rd32(s + b);
        if (x)
            return a - a0 + (__builtin_ctz(x) >> 3);
        a += 4;
        b += 4;
    }
    while (a < lim && s[a] == s[b]) {
        a++;
        b++;
    }
    return a - a0;
}

// liblz4's LZ4_compress_generic (byU16, noDict, limitedOutput, capacity n-1)
// on s[0..n); writes the block payload through o and returns its size, or
// 0 when it does not fit (the frame's block is then stored raw).
// kLinked: one block s[b0, b0 + n) of a linked frame starting at s, on the
// frame's stream table (byU32, positions from s, 65535 distance limit).
// Table layouts: kVal = false is liblz4's (u16 positions; a candidate's word
// is loaded from the input); kVal = true keeps each entry's input word beside
// its position (u64: word << 32 | position + 1; 0 = liblz4's zeroed entry,
// position 0), so a probe compares without loading the candidate's word.
// VPtr: the position + word table's pointer type (HBM scratch, or LDS for
// the linked kernel: vtab).
template <uint32_t kProbe, bool kVal, bool kLinked = false, typename VPtr = uint64_t *>
__device__ uint32_t compress_block(const uint8_t *__restrict__ s, uint32_t b0, uint32_t n,
                                   void *__restrict__ table, Packer &o, uint32_t accel, VPtr vtab = VPtr())
{
    static_assert(kVal || !kLinked, "linked frames use the position + word table");
    uint16_t *__restrict__ T = static_cast<uint16_t *>(table);
    VPtr V;
    if constexpr (std::is_same<VPtr, uint64_t *>::value)
        V = static_cast<uint64_t *>(table);
    else
        V = vtab;
    const uint32_t cap = n - 1;
    uint32_t op = 0, anchor = b0;
    if (n >= 13) {
        const uint32_t mflimit1 = b0 + n - 11, matchlimit = b0 + n - 5;
        const uint32_t first4 = rd32(s);   // word at position 0: what a zeroed entry points to
        {
            uint32_t h0;
            const uint32_t w = word_hash<kLinked>(s + b0, h0);
            if constexpr (kVal)
                V[h0] = (uint64_t)w << 32 | (b0 + 1);
            else
                T[h0] = 0;
        }
        uint32_t ip = b0 + 1;
        for (;;) {
            uint32_t m;
            {
                // kProbe probes at a time: their positions follow the step
                // schedule alone, so the input words, the table entries and
                // the candidates' words are each loaded as one batch; a probe
                // whose hash an earlier probe of the batch wrote takes that
                // probe's position (what the serial loop would read back)
                uint32_t fwd = ip, step = 1, nb = accel << 6;
                for (;;) {
                    uint32_t pk[kProbe], in[kProbe], hk[kProbe], ck[kProbe], cw[kProbe];
                    uint32_t f = fwd, st = step, nbb = nb, nvalid = kProbe;
#pragma unroll
                    for (uint32_t k = 0; k < kProbe; k++) {
                        pk[k] = f;
                        f += st;
                        st = nbb++ >> 6;
                        if (f > mflimit1 && nvalid == kProbe)
                            nvalid = k;   // probe k ends the search (liblz4: goto _last_literals)
                    }
#pragma unroll
                    for (uint32_t k = 0; k < kProbe; k++)
                        in[k] = word_hash<kLinked>(s + min(pk[k], mflimit1), hk[k]);
                    if constexpr (kVal) {
#pragma unroll
                        for (uint32_t k = 0; k < kProbe; k++) {
                            const uint64_t e = V[hk[k]];
                            ck[k] = e ? (uint32_t)e - 1 : 0;
                            cw[k] = e ? (uint32_t)(e >> 32) : first4;
                        }
                    } else {
#pragma unroll
                        for (uint32_t k = 0; k < kProbe; k++)
                            ck[k] = T[hk[k]];
                    }
#pragma unroll
                    for (uint32_t k = 1; k < kProbe; k++)
#pragma unroll
                        for (uint32_t j = 0; j < k; j++) {
                            ck[k] = hk[j] == hk[k] ? pk[j] : ck[k];
                            if constexpr (kVal)
                                cw[k] = hk[j] == hk[k] ? in[j] : cw[k];
                        }
                    if constexpr (!kVal) {
#pragma unroll
                        for (uint32_t k = 0; k < kProbe; k++)
                            cw[k] = rd32(s + min(ck[k], mflimit1));   // clamped: probes past nvalid
                    }
                    uint32_t hit = kProbe;
#pragma unroll
                    for (uint32_t k = kProbe; k-- > 0;)   // linked: a candidate > 65535 back is not compared
                        hit = (k < nvalid && cw[k] == in[k] && (!kLinked || ck[k] + 65535 >= pk[k])) ? k : hit;
#pragma unroll
                    for (uint32_t k = 0; k < kProbe; k++)   // the probes that ran, in order
                        if (k < nvalid && k <= hit) {
                            if constexpr (kVal)
                                V[hk[k]] = (uint64_t)in[k] << 32 | (pk[k] + 1);
                            else
                                T[hk[k]] = (uint16_t)pk[k];
                        }
                    if (hit < kProbe) {
                        ip = pk[hit];
                        m = ck[hit];
                        break;
                    }
                    if (nvalid < kProbe)
                        goto last_literals;
                    fwd = f;
                    step = st;
                    nb = nbb;
                }
            }
            // backward extension, four bytes per compare (equal top bytes of
            // the words ending at ip and m are the bytes just before them)
            while (m >= 4 && ip > anchor) {
                const uint32_t x = rd32(s + ip - 4) ^ rd32(s + m - 4);
                const uint32_t k = min(x ? (uint32_t)__builtin_clz(x) >> 3 : 4u, ip - anchor);
                ip -= k;
                m -= k;
                if (k < 4)
                    break;
            }
            if (m < 4)
                while (ip > anchor && m > 0 && s[ip - 1] == s[m - 1]) {
                    ip--;
                    m--;
                }
            uint32_t lit = ip - anchor;
            // liblz4: after the token, op + lit + 8 + lit/255 must fit
            if (op + 1 + lit + 8 + lit / 255 > cap)
                return 0;
            for (;;) {
                const uint32_t mc = count_eq(s, ip + 4, m + 4, matchlimit);
                const uint32_t op2 = op + 1 + ext_bytes(lit) + lit + 2;
                if (op2 + 6 + (mc + 240) / 255 > cap)
                    return 0;
                emit_seq(o, s + anchor, lit, ip - m, mc);
                op = op2 + ext_bytes(mc);
                ip += mc + 4;
                anchor = ip;
                if (ip >= mflimit1)
                    goto last_literals;
                uint32_t h2, h;
                const uint32_t w2 = word_hash<kLinked>(s + ip - 2, h2), w0 = word_hash<kLinked>(s + ip, h);
                uint32_t cand, cval;
                if constexpr (kVal) {
                    V[h2] = (uint64_t)w2 << 32 | (ip - 1);
                    const uint64_t e = V[h];
                    cand = e ? (uint32_t)e - 1 : 0;
                    cval = e ? (uint32_t)(e >> 32) : first4;
                    V[h] = (uint64_t)w0 << 32 | (ip + 1);
                } else {
                    T[h2] = (uint16_t)(ip - 2);
                    cand = T[h];
                    T[h] = (uint16_t)ip;
                    cval = rd32(s + cand);
                }
                if (cval != w0 || (kLinked && cand + 65535 < ip))
                    break;
                m = cand;   // immediate match: no literals, no literal check
                lit = 0;
            }
            ip++;
        }
    }
last_literals:
    {
        const uint32_t run = b0 + n - anchor;
        if (op + run + 1 + (run + 240) / 255 > cap)
            return 0;
        o.put((run >= 15 ? 15u : run) << 4);
        if (run >= 15)
            o.run(run - 15);
        o.copy(s + anchor, run);
        op += 1 + ext_bytes(run) + run;
    }
    return op;
}

// The linked blocks of one frame of n > 64 KiB after its header; returns the
// bytes written after the header (block words + blocks).
// The frame header through o (magic, FLG, BD, [content size], HC); returns
// its length.  One independent block up to 64 KiB, linked blocks above.
__device__ uint32_t frame_header(Packer &o, uint32_t n, bool with_size)
{
    uint8_t hdr[15];
    hdr[0] = 0x04;
    hdr[1] = 0x22;
    hdr[2] = 0x4D;
    hdr[3] = 0x18;
    hdr[4] = (n > kMaxFrame ? 0x40 : 0x60) | (with_size ? 0x08 : 0);
    hdr[5] = 0x40;
    uint32_t hlen = 6;
    if (with_size) {
        for (int i = 0; i < 8; i++)
            hdr[6 + i] = i < 4 ? (uint8_t)(n >> (8 * i)) : 0;
        hlen = 14;
    }
    hdr[hlen] = (uint8_t)(xxh32_short(hdr + 4, hlen - 4) >> 8);
    hlen++;
    for (uint32_t i = 0; i < hlen; i++)
        o.put(hdr[i]);
    return hlen;
}

template <typename VPtr>
__device__ uint32_t compress_linked(const uint8_t *__restrict__ s, uint32_t n, VPtr table,
                                    uint8_t *__restrict__ out, uint32_t hlen, Packer &o, uint32_t accel)
{
    uint32_t at = hlen;
    for (uint32_t b0 = 0; b0 < n; b0 += kMaxFrame) {
        const uint32_t m = min(n - b0, kMaxFrame);
        const Packer save = o;
        o.put4(0);   // block word, patched below
        uint32_t c = compress_block<8, true, true, VPtr>(s, b0, m, nullptr, o, accel, table);
        if (c == 0) {   // did not fit: raw, the stream already advanced
            o = save;
            o.put4(m | kStoredFlag);
            o.copy(s + b0, m);
            c = m;
        } else {
            // the word's bytes: in memory if the packer flushed them, else in acc
            const uint32_t flushed = 4u * (uint32_t)(o.w - reinterpret_cast<uint32_t *>(out));
            for (uint32_t i = 0; i < 4; i++) {
                const uint32_t p = at + i, v = (c >> (8 * i)) & 0xFF;
                if (p < flushed)
                    out[p] = (uint8_t)v;
                else
                    o.acc |= v << (8 * (p - flushed));
            }
        }
        at += 4 + c;
    }
    return at - hlen;
}

template <uint32_t kProbe, bool kVal>
__global__ __launch_bounds__(64) void lz4_compress_kernel(const zsk_compress_desc_t *__restrict__ desc,
                                                          uint32_t nframes, const uint8_t *__restrict__ src,
                                                          uint8_t *__restrict__ dst,
                                                          uint32_t *__restrict__ csize,
                                                          uint8_t *__restrict__ tables,
                                                          uint32_t *__restrict__ stored, uint32_t accel,
                                                          uint32_t per_wave)
{
    const uint32_t f = blockIdx.x * per_wave + threadIdx.x;
    if (threadIdx.x >= per_wave || f >= nframes)
        return;
    const zsk_compress_desc_t d = desc[f];
    stored[f] = 0;
    if (d.src_size > kMaxLinkedFrame || (d.dst_off & 15)) {
        csize[f] = 0;
        return;
    }
    const uint32_t n = d.src_size;
    if (n > kMaxFrame)
        return;   // linked: lz4_compress_linked_kernel's frame
    uint8_t *out = dst + d.dst_off;
    Packer o{reinterpret_cast<uint32_t *>(out), 0, 0};
    const uint32_t hlen = frame_header(o, n, (d.flags & ZSK_COMPRESS_CONTENT_SIZE) && n > 0);
    if (n == 0) {
        for (int i = 0; i < 4; i++)
            o.put(0);
        o.flush();
        csize[f] = hlen + 4;
        return;
    }
    uint8_t *const table = tables + (size_t)f * kTable * (kVal ? 8 : 2);
    for (int i = 0; i < 4; i++)   // block word, patched below
        o.put(0);
    const uint32_t c = compress_block<kProbe, kVal>(src + d.src_off, 0, n, table, o, accel);
    if (c == 0) {
        // the header stays; block word, raw block and end mark come from
        // lz4_store_kernel
        o.flush();
        stored[f] = hlen;
        csize[f] = hlen + 4 + n + 4;
        return;
    }
    for (int i = 0; i < 4; i++)
        o.put(0);
    o.flush();
    for (int i = 0; i < 4; i++)
        out[hlen + i] = (uint8_t)(c >> (8 * i));
    csize[f] = hlen + 4 + c + 4;
}

// Linked frames (> 64 KiB): one frame per single-wave workgroup, the stream's
// 4,096-entry position + word table in LDS (32 KiB: five frames per CU), so a
// probe batch waits on LDS instead of an HBM round trip (the HBM-table lane
// ran at ~5 MB/s: 1 GiB of 1 MiB frames in 208 ms).  Lane 0 compresses; the
// wave zeroes the table first (the stream's fresh state).
typedef __attribute__((address_space(3))) uint64_t lds_u64;

__global__ __launch_bounds__(64) void lz4_compress_linked_kernel(const zsk_compress_desc_t *__restrict__ desc,
                                                                 uint32_t nframes, const uint8_t *__restrict__ src,
                                                                 uint8_t *__restrict__ dst,
                                                                 uint32_t *__restrict__ csize, uint32_t accel)
{
    __shared__ __attribute__((aligned(16))) uint64_t tab[1u << kLinkedHashLog];
    const uint32_t f = blockIdx.x;
    if (f >= nframes)
        return;
    const zsk_compress_desc_t d = desc[f];
    const uint32_t n = d.src_size;
    if (n <= kMaxFrame || n > kMaxLinkedFrame || (d.dst_off & 15))
        return;   // lz4_compress_kernel's frame (or refused there)
    for (uint32_t i = threadIdx.x; i < (1u << kLinkedHashLog); i += 64)
        tab[i] = 0;
    __syncthreads();
    if (threadIdx.x != 0)
        return;
    lds_u64 *const V = (lds_u64 *)(uintptr_t)(uint32_t)(uintptr_t)tab;
    uint8_t *out = dst + d.dst_off;
    Packer o{reinterpret_cast<uint32_t *>(out), 0, 0};
    const uint32_t hlen = frame_header(o, n, (d.flags & ZSK_COMPRESS_CONTENT_SIZE) != 0);
    const uint32_t body = compress_linked(src + d.src_off, n, V, out, hlen, o, accel);
    o.put4(0);   // end mark
    o.flush();
    csize[f] = hlen + body + 4;
}

// Raw blocks of the frames lz4_compress_kernel flagged: one wave per frame.
__global__ __launch_bounds__(256) void lz4_store_kernel(const zsk_compress_desc_t *__restrict__ desc,
                                                        uint32_t nframes, const uint8_t *__restrict__ src,
                                                        uint8_t *__restrict__ dst,
                                                        const uint32_t *__restrict__ stored)
{
    const uint32_t f = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (f >= nframes)
        return;
    const uint32_t hlen = stored[f];
    if (hlen == 0)
        return;
    const zsk_compress_desc_t d = desc[f];
    const uint32_t n = d.src_size;
    uint8_t *out = dst + d.dst_off + hlen;
    const uint8_t *in = src + d.src_off;
    const uint32_t word = n | kStoredFlag;
    if (lane < 4) {
        out[lane] = (uint8_t)(word >> (8 * lane));
        out[4 + n + lane] = 0;
    }
    for (uint32_t i = lane; i < n; i += 64)
        out[4 + i] = in[i];
}

}   // namespace

int launch_lz4_compress(const zsk_compress_desc_t *d_desc, uint32_t nframes, const uint8_t *d_src,
                        uint8_t *d_dst, uint32_t *d_csize, int level, void *d_scratch, hipStream_t stream)
{
    if (nframes == 0)
        return 0;
    if (!d_desc || !d_src || !d_dst || !d_csize || !d_scratch || level >= 3)
        return -1;
    const uint32_t accel = level < 0 ? (level < -65536 ? 65537u : (uint32_t)(1 - level)) : 1u;
    // probes per search batch and table layout: env ZSEEK_LZ4C_PROBE,
    // ZSEEK_LZ4C_VAL (tuning only)
    static const int probe = [] {
        const char *e = getenv("ZSEEK_LZ4C_PROBE");
        return e ? atoi(e) : kDefaultProbe;
    }();
    static const bool val = [] {
        const char *e = getenv("ZSEEK_LZ4C_VAL");
        return e ? atoi(e) != 0 : kDefaultVal;
    }();
    uint8_t *tables = static_cast<uint8_t *>(d_scratch);
    uint32_t *stored = reinterpret_cast<uint32_t *>(tables + (size_t)nframes * kTable * 8);
    if (hipMemsetAsync(tables, 0, (size_t)nframes * kTable * (val ? 8 : 2), stream) != hipSuccess)
        return -1;
    auto kern = val ? (probe == 16   ? lz4_compress_kernel<16, true>
                       : probe == 4  ? lz4_compress_kernel<4, true>
                       : probe == 12 ? lz4_compress_kernel<12, true>
                                     : lz4_compress_kernel<8, true>)
                    : probe == 16 ? lz4_compress_kernel<16, false>
                    : probe == 32 ? lz4_compress_kernel<32, false>
                                  : lz4_compress_kernel<8, false>;
    // frames per wave: about kWaves waves (env ZSEEK_LZ4C_WAVES, tuning only)
    static const uint32_t waves = [] {
        const char *e = getenv("ZSEEK_LZ4C_WAVES");
        const int v = e ? atoi(e) : 0;
        return v > 0 ? (uint32_t)v : kDefaultWaves;
    }();
    const uint32_t per_wave = min(64u, max(1u, (nframes + waves - 1) / waves));
    hipLaunchKernelGGL(kern, dim3((nframes + per_wave - 1) / per_wave), dim3(64), 0, stream, d_desc, nframes,
                       d_src, d_dst, d_csize, tables, stored, accel, per_wave);
    hipLaunchKernelGGL(lz4_compress_linked_kernel, dim3(nframes), dim3(64), 0, stream, d_desc, nframes, d_src, d_dst,
                       d_csize, accel);
    hipLaunchKernelGGL(lz4_store_kernel, dim3((nframes + 3) / 4), dim3(256), 0, stream, d_desc, nframes, d_src,
                       d_dst, stored);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk

extern "C" ZSEEK_EXPORT size_t zsk_lz4_compress_scratch_size(uint32_t nframes)
{
    return (size_t)nframes * (zsk::kTable * sizeof(uint64_t) + sizeof(uint32_t));
}

extern "C" ZSEEK_EXPORT int zsk_lz4_compress_frames(const zsk_compress_desc_t *d_desc, uint32_t nframes,
                                                    const void *d_src, void *d_dst, uint32_t *d_csize,
                                                    int level, void *d_scratch, void *stream)
{
    return zsk::launch_lz4_compress(d_desc, nframes, static_cast<const uint8_t *>(d_src),
                                    static_cast<uint8_t *>(d_dst), d_csize, level, d_scratch,
                                    static_cast<hipStream_t>(stream));
}
