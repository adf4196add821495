// lz4_lane.hip — lane-per-frame LZ4-frame decoder for CDNA4 (gfx950).
//
// Replaces the per-frame liblz4 call of the reference hot path
// (/root/reference/src/decompress.c:752-773, LZ4F_decompress in a loop).
//
// One LANE decodes one seek-table frame, start to end, exactly as liblz4
// does on a CPU core (validation: liblz4 1.9.3 rules, mirrored from
// lz4_split.hip / oracle/lz4_oracle.c) — 64 frames advance per wave
// instruction, so the serial token chain of LZ4 costs 1/64 of an instruction
// per sequence.  Every wave iteration each lane takes one step of its own
// state machine (typically: token, literal run, offset, match = one whole
// sequence) and the memory traffic is software-pipelined over kG slots:
//
//   * compressed bytes stream into a per-lane 512-byte LDS ring, 64 bytes per
//     iteration, loaded kG iterations before they are needed (a pipeline
//     slot carries them, retired into the ring by a ds_write);
//   * literal runs are copied ring -> output at once (16-byte stores that may
//     run past the run: those bytes belong to later output of the same lane,
//     which is written later in program order — except at the frame end,
//     where the stores are exact);
//   * a match's source pieces are loaded into the iteration's slot and
//     stored kG iterations later.  Stores of a match are exact (overlapping
//     full 16-byte pieces, or 8/4-byte pairs for short matches).  A lane whose
//     match source overlaps one of its own still-pending match destinations
//     waits (the slot retires within kG iterations).  Overlapping copies
//     (offset < length) read the off-byte pattern before the match modulo
//     the offset, so their pieces are independent too.
//
// Every global access is a buffer instruction on a per-wave resource; a lane
// with nothing to load or store uses an out-of-range offset, so each
// iteration issues a fixed count of vector-memory instructions and the
// compiler's vmcnt waits retire exactly the slot being consumed.
//
// Frames with block/content checksums (never written by the reference's
// writer) or that do not fit this scheme are left with status ST_NOT_RUN and
// finished by the wave-per-frame kernel (lz4_wave.hip).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kLaneWaves = 4;       // waves per workgroup
constexpr uint32_t kRing = 512;          // per-lane compressed-byte ring (LDS)
constexpr uint32_t kRingStride = 528;    // bytes between lanes' rings (bank spread)
constexpr uint32_t kFill = 32;           // ring bytes loaded per iteration
constexpr uint32_t kSlots = 6;           // pipeline depth (slots in flight per lane)
constexpr uint32_t kOff = 0x80000000u;   // out-of-range buffer offset: op disabled

enum : uint32_t {
    P_HDR = 0,
    P_BHDR,
    P_TOKEN,
    P_LITLEN,
    P_LIT,
    P_OFF,
    P_MLLEN,
    P_MATCH,
    P_END,
    P_DONE,
};

// One pipeline slot of a lane: what one iteration loads and, kG iterations
// later, writes.  Output pieces are stored in output order (literal pieces,
// then match pieces; slots retire in issue order), so a 16-byte piece may run
// past the bytes it owns: every byte after it is written again, later.
struct Slot {
    u32x4 w0, w1;           // ring bytes [wx, wx + 32)
    uint32_t wx;            // ring coordinate of w0, or kOff
    uint32_t lx;            // literal: output offset (cout coords), or kOff
    uint32_t lp;            // literal: frame offset of its bytes (still in the ring at retire)
    u32x4 m0, m1, m2, m3;   // match pieces (source bytes) at output mx + 16 i;
                            // overlapping copies: m3 = the off bytes before the match
    uint32_t mx;            // match chunk: output offset (cout coords)
    uint32_t lmn;           // literal bytes (0..32) | match bytes (0..64) << 8
    uint32_t ovr;           // overlapping copies: offset | pattern phase at mx << 16 (0 = plain)
};

__device__ __forceinline__ uint32_t slot_ln(const Slot &S) { return S.lmn & 0xFF; }
__device__ __forceinline__ uint32_t slot_mn(const Slot &S) { return S.lmn >> 8; }

struct Lane;
__device__ __forceinline__ uint32_t slot_wlo(const Lane &L, const Slot &S);

struct Lane {
    // resources (wave-uniform) and the lane's frame inside them
    __amdgpu_buffer_rsrc_t cin, cout;
    uint32_t cx0;       // coordinate of frame byte 0 in cin
    uint32_t ox0;       // offset of frame output byte 0 in cout
    uint32_t oend_x;    // cout offset of the frame's output end
    uint32_t clen, dlen;
    uint32_t ring;      // LDS byte address of this lane's ring
    // ring state (coordinates)
    uint32_t fill;      // next coordinate to load
    uint32_t avail;     // coordinates < avail are in the ring
    // decoder state
    uint32_t ph;        // phase
    int32_t st;         // status when P_DONE
    uint32_t ip;        // frame offset of the next byte to parse
    uint32_t op;        // output offset of the next byte
    uint32_t fail_op;
    uint32_t flg_csize;
    uint64_t csize;
    uint32_t indep, bsid, max_block;
    uint32_t iend, oend, floor_, bop;   // current block
    uint32_t stored;    // current literal run is a stored block
    uint32_t tok, lit, ml, off;
    uint32_t lrem;      // literal bytes left to copy
    uint32_t mrem;      // match bytes left to issue
    uint32_t mdone;     // match bytes issued so far
    uint32_t ipm;       // frame offset after the match header (fast path)
    uint32_t mparsed;   // the match of the current sequence is already parsed
};

__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// ---- ring access ------------------------------------------------------------
__device__ __forceinline__ uint32_t ring_addr(const Lane &L, uint32_t x)
{
    return L.ring + (x & (kRing - 1));
}

__device__ __forceinline__ uint32_t lds_u8(uint32_t a)
{
    return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t *>(
        (__attribute__((address_space(3))) void *)(uintptr_t)a);
}

__device__ __forceinline__ uint32_t lds_u32(uint32_t a)
{
    return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(
        (__attribute__((address_space(3))) void *)(uintptr_t)a);
}

__device__ __forceinline__ void lds_w128(uint32_t a, u32x4 v)
{
    *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(
        (__attribute__((address_space(3))) void *)(uintptr_t)a) = v;
}

// frame byte p (must be in the ring)
__device__ __forceinline__ uint32_t rb(const Lane &L, uint32_t p)
{
    return lds_u8(ring_addr(L, L.cx0 + p));
}

// 16 frame bytes from p (in the ring): 5 aligned dword reads + byte align
__device__ __forceinline__ u32x4 r16(const Lane &L, uint32_t p)
{
    const uint32_t x = L.cx0 + p;
    const uint32_t a = x & ~3u, sh = x & 3;
    const uint32_t d0 = lds_u32(ring_addr(L, a)), d1 = lds_u32(ring_addr(L, a + 4));
    const uint32_t d2 = lds_u32(ring_addr(L, a + 8)), d3 = lds_u32(ring_addr(L, a + 12));
    const uint32_t d4 = lds_u32(ring_addr(L, a + 16));
    u32x4 v;
    v.x = __builtin_amdgcn_alignbyte(d1, d0, sh);
    v.y = __builtin_amdgcn_alignbyte(d2, d1, sh);
    v.z = __builtin_amdgcn_alignbyte(d3, d2, sh);
    v.w = __builtin_amdgcn_alignbyte(d4, d3, sh);
    return v;
}

// frame bytes [p, p+n) are in the ring
__device__ __forceinline__ bool have(const Lane &L, uint32_t p, uint32_t n)
{
    return L.cx0 + p + n <= L.avail;
}

// ---- buffer memory ops (offset kOff = disabled) ------------------------------
__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t x)
{
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, x, 0, 0));
}

__device__ __forceinline__ void bstore16(__amdgpu_buffer_rsrc_t r, uint32_t x, u32x4 v)
{
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                           r, x, 0, 0);
}

__device__ __forceinline__ void bstore1(__amdgpu_buffer_rsrc_t r, uint32_t x, uint32_t v)
{
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, r, x, 0, 0);
}

// first n (0..16) bytes of v at output offset x, exactly (rare paths)
__device__ __forceinline__ void bstore_exact(__amdgpu_buffer_rsrc_t r, uint32_t x, u32x4 v, uint32_t n)
{
    for (uint32_t i = 0; i < n; i++)
        bstore1(r, x + i, vbyte(v, i));
}

// 16 bytes: a[0..k) then b[0..16-k)   (0 <= k <= 16)
__device__ __forceinline__ u32x4 splice(u32x4 a, u32x4 b, uint32_t k)
{
    if (k >= 16)
        return a;
    // b shifted up by k bytes
    uint32_t bw[4] = {b.x, b.y, b.z, b.w};
    uint32_t s[4];
    const uint32_t q = k >> 2, r = k & 3;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int j = i - (int)q;
        const uint32_t hi = j >= 0 ? bw[j & 3] : 0;
        const uint32_t lo = j >= 1 ? bw[(j - 1) & 3] : 0;
        s[i] = r ? ((hi << (8 * r)) | (lo >> (32 - 8 * r))) : hi;
    }
    uint32_t aw[4] = {a.x, a.y, a.z, a.w};
    u32x4 o;
    uint32_t ow[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t lo_bytes = k >= 4u * (i + 1) ? 4 : (k > 4u * i ? k - 4u * i : 0);
        const uint32_t m = lo_bytes >= 4 ? 0xFFFFFFFFu : ((1u << (8 * lo_bytes)) - 1);
        ow[i] = (aw[i] & m) | (s[i] & ~m);
    }
    o.x = ow[0];
    o.y = ow[1];
    o.z = ow[2];
    o.w = ow[3];
    return o;
}

// 16 bytes of the period-off pattern pat[0..off) starting at phase s
__device__ __forceinline__ u32x4 repeat16(u32x4 pat, uint32_t off, uint32_t s)
{
    uint32_t w[4] = {0, 0, 0, 0};
    uint32_t m = s;
#pragma unroll
    for (int i = 0; i < 16; i++) {
        w[i >> 2] |= vbyte(pat, m) << (8 * (i & 3));
        m = m + 1 == off ? 0 : m + 1;
    }
    u32x4 v;
    v.x = w[0];
    v.y = w[1];
    v.z = w[2];
    v.w = w[3];
    return v;
}

// ---- pipeline slot ------------------------------------------------------------

// first output byte (frame offset) a busy slot writes
__device__ __forceinline__ uint32_t slot_wlo(const Lane &L, const Slot &S)
{
    return (S.lx != kOff ? S.lx : S.mx) - L.ox0;
}

// 16 bytes at output offset x (cout coords); a piece reaching past the
// frame's output end is skipped here and written exactly by put_tails
template <int DIAG>
__device__ __forceinline__ void put16(const Lane &L, uint32_t x, u32x4 v, bool &tail)
{
    const bool t = x != kOff && x + 16 > L.oend_x;
    tail |= t;
    bstore16(L.cout, (t || (DIAG & 1)) ? kOff : ((DIAG & 4) ? x & ~15u : x), v);
}


template <int DIAG>
__device__ __forceinline__ void retire(Lane &L, Slot &S)
{
    if (S.wx != kOff) {
        const uint32_t a = ring_addr(L, S.wx);
        lds_w128(a, S.w0);
        lds_w128(a + 16, S.w1);
        L.avail = S.wx + kFill;
    }
    bool tail = false;
    const uint32_t ln = slot_ln(S), mn = slot_mn(S);
    const uint32_t lx1 = ln > 16 ? S.lx + 16 : kOff;
    const u32x4 l0 = r16(L, S.lp), l1 = r16(L, S.lp + 16);
    put16<DIAG>(L, S.lx, l0, tail);
    put16<DIAG>(L, lx1, l1, tail);
    // match pieces
    u32x4 v0 = S.m0, v1 = S.m1, v2 = S.m2, v3 = S.m3;
    if (S.ovr) {
        // overlapping copy (<= 48 bytes a chunk): piece i = pattern bytes from
        // phase (mph + 16 i) mod off; the pattern itself is in m3
        const uint32_t off = S.ovr & 0xFFFF, mph = S.ovr >> 16;
        const u32x4 pat = S.m3;
#pragma unroll 1
        for (uint32_t i = 0; i < 3; i++) {
            const u32x4 a = i == 0 ? v0 : i == 1 ? v1 : v2;
            const uint32_t ph = (mph + 16 * i) % off;
            const u32x4 r = off < 16 ? repeat16(pat, off, ph) : splice(a, pat, off - ph);
            v0 = i == 0 ? r : v0;
            v1 = i == 1 ? r : v1;
            v2 = i == 2 ? r : v2;
        }
    }
    const uint32_t mx = mn ? S.mx : kOff;
    const uint32_t mx1 = mn > 16 ? mx + 16 : kOff, mx2 = mn > 32 ? mx + 32 : kOff;
    const uint32_t mx3 = mn > 48 ? mx + 48 : kOff;
    put16<DIAG>(L, mx, v0, tail);
    put16<DIAG>(L, mx1, v1, tail);
    put16<DIAG>(L, mx2, v2, tail);
    put16<DIAG>(L, mx3, v3, tail);
    if (tail) {
        // exact stores of the pieces put16 skipped (the last bytes of a frame)
#pragma unroll 1
        for (uint32_t i = 0; i < 6; i++) {
            const uint32_t x = i == 0 ? S.lx : i == 1 ? lx1 : i == 2 ? mx : i == 3 ? mx1 : i == 4 ? mx2 : mx3;
            const u32x4 v = i == 0 ? l0 : i == 1 ? l1 : i == 2 ? v0 : i == 3 ? v1 : i == 4 ? v2 : v3;
            if (x != kOff && x + 16 > L.oend_x)
                bstore_exact(L.cout, x, v, L.oend_x - x);
        }
    }
    S.wx = kOff;
    S.lx = kOff;
    S.lmn = 0;
    S.ovr = 0;
}

// ---- state machine handlers ---------------------------------------------------
__device__ __forceinline__ void fail_block(Lane &L)
{
    const bool direct = (L.dlen - L.bop) >= L.max_block;
    const int32_t bits = (int32_t)((L.bsid - 4) << ST_BSID_SHIFT);
    L.st = (direct ? (ST_GENERIC | ST_DIRECT_FLAG) : ST_DECOMPRESS_FAILED) | ST_BLOCK_FAIL_FLAG | bits;
    L.ph = P_DONE;
}

__device__ __forceinline__ void finish(Lane &L, int32_t st)
{
    L.st = st;
    L.ph = P_DONE;
}

__device__ __forceinline__ uint32_t rd32(const Lane &L, uint32_t p)
{
    return rb(L, p) | (rb(L, p + 1) << 8) | (rb(L, p + 2) << 16) | (rb(L, p + 3) << 24);
}

// Frame header (LZ4F_decodeHeader order, as lz4_split.hip / the oracle).
// Returns a final status, or -1 when the frame continues with its blocks.
__device__ __forceinline__ int32_t hdr_status(Lane &L)
{
    const uint32_t clen = L.clen;
    if (clen < 7)
        return ST_HDR_INCOMPLETE;
    const uint32_t magic = rd32(L, 0);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u)
        return ST_SHORT_FRAME;
    if (magic != kLz4Magic)
        return ST_FRAME_TYPE;
    const uint32_t flg = rb(L, 4), bd = rb(L, 5);
    if (flg & 0x14)   // block / content checksums: the wave kernel verifies them
        return ST_NOT_RUN;
    const uint32_t dictid = flg & 1;
    if ((flg >> 1) & 1)
        return ST_RESERVED;
    if (((flg >> 6) & 3) != 1)
        return ST_VERSION;
    const uint32_t csz = (flg >> 3) & 1;
    const uint32_t hdr = 7 + (csz ? 8 : 0) + (dictid ? 4 : 0);
    if (clen < hdr)
        return ST_HDR_INCOMPLETE;
    const uint32_t bsid = (bd >> 4) & 7;
    if ((bd >> 7) & 1)
        return ST_RESERVED;
    if (bsid < 4)
        return ST_MAXBLOCK;
    if (bd & 15)
        return ST_RESERVED;
    // header checksum: (XXH32(descriptor, 0) >> 8) & 0xFF over bytes [4, hdr-1)
    const uint32_t n = hdr - 5;
    uint32_t acc = 0x165667B1u + n;
    uint32_t i = 0;
    for (; i + 4 <= n; i += 4) {
        acc += rd32(L, 4 + i) * 0xC2B2AE3Du;
        acc = ((acc << 17) | (acc >> 15)) * 0x27D4EB2Fu;
    }
    for (; i < n; i++) {
        acc += rb(L, 4 + i) * 0x165667B1u;
        acc = ((acc << 11) | (acc >> 21)) * 0x9E3779B1u;
    }
    acc ^= acc >> 15;
    acc *= 0x85EBCA77u;
    acc ^= acc >> 13;
    acc *= 0xC2B2AE3Du;
    acc ^= acc >> 16;
    if (((acc >> 8) & 0xFF) != rb(L, hdr - 1))
        return ST_HDR_CHECKSUM;
    L.indep = (flg >> 5) & 1;
    L.flg_csize = csz;
    L.bsid = bsid;
    if (csz)
        L.csize = (uint64_t)rd32(L, 6) | ((uint64_t)rd32(L, 10) << 32);
    L.max_block = 1u << (8 + 2 * bsid);
    L.ip = hdr;
    return -1;
}

__device__ __forceinline__ void do_bhdr(Lane &L)
{
    L.fail_op = L.op;
    if (L.clen - L.ip < 4) {
        finish(L, ST_TRUNCATED);
        return;
    }
    if (!have(L, L.ip, 4))
        return;
    const uint32_t bh = rd32(L, L.ip);
    L.ip += 4;
    if (bh == 0) {
        L.ph = P_END;
        return;
    }
    const uint32_t bsize = bh & 0x7FFFFFFFu;
    if (bsize > L.max_block) {
        finish(L, ST_MAXBLOCK);
        return;
    }
    if (L.clen - L.ip < bsize) {
        finish(L, ST_TRUNCATED);
        return;
    }
    L.bop = L.op;
    L.iend = L.ip + bsize;
    if (bh & 0x80000000u) {
        if (L.op + bsize > L.dlen) {
            finish(L, ST_DST_OVERFLOW);
            return;
        }
        L.stored = 1;
        L.lit = bsize;
        L.lrem = bsize;
        L.ph = bsize ? P_LIT : P_BHDR;
        return;
    }
    if (bsize == 0) {
        fail_block(L);
        return;
    }
    L.stored = 0;
    L.oend = L.op + L.max_block;
    L.floor_ = L.indep ? L.op : 0;
    L.ph = P_TOKEN;
}

// decide whether the literal run just measured is the block's last sequence
__device__ __forceinline__ void lit_measured(Lane &L)
{
    const uint32_t p = L.ip, lit = L.lit;
    if (L.op + lit > L.oend - kMfLimit || L.iend - p < lit + 2 + 1 + kLastLiterals) {
        if (L.iend - p != lit || L.op + lit > L.oend) {
            fail_block(L);
            return;
        }
        if (L.op + lit > L.dlen) {
            finish(L, ST_DST_OVERFLOW);
            return;
        }
        L.stored = 2;   // last sequence of the block: literal run only
    } else if (L.op + lit > L.dlen) {
        finish(L, ST_DST_OVERFLOW);
        return;
    }
    L.lrem = lit;
    L.ph = P_LIT;
}

__device__ __forceinline__ void do_token(Lane &L)
{
    if (L.ip >= L.iend) {
        fail_block(L);
        return;
    }
    if (!have(L, L.ip, 1))
        return;
    L.tok = rb(L, L.ip);
    L.lit = L.tok >> 4;
    L.ip++;
    if (L.lit == 15) {
        if (L.iend - L.ip <= 15) {
            fail_block(L);
            return;
        }
        L.ph = P_LITLEN;
        return;
    }
    lit_measured(L);
}

__device__ __forceinline__ void do_litlen(Lane &L)
{
    for (;;) {
        if (L.ip >= L.iend) {
            fail_block(L);
            return;
        }
        if (!have(L, L.ip, 1))
            return;
        const uint32_t s = rb(L, L.ip++);
        L.lit += s;
        if (s != 255)
            break;
    }
    lit_measured(L);
}

// Up to 32 literal bytes ring -> slot (stored at retire).
__device__ __forceinline__ void do_lit(Lane &L, Slot &S)
{
    const uint32_t n = L.lrem < 32 ? L.lrem : 32;
    if (n && !have(L, L.ip, n))
        return;
    if (n) {
        S.lp = L.ip;
        S.lx = L.ox0 + L.op;
        S.lmn = n;
    }
    L.ip += n;
    L.op += n;
    L.lrem -= n;
    if (L.lrem == 0) {
        if (L.stored == 1) {
            L.ph = P_BHDR;
        } else if (L.stored == 2) {
            L.ph = P_BHDR;
            L.ip = L.iend;
        } else if (L.mparsed) {
            L.mparsed = 0;
            L.ip = L.ipm;
            L.mrem = L.ml;
            L.mdone = 0;
            L.ph = P_MATCH;
        } else {
            L.ph = P_OFF;
        }
    }
}

__device__ __forceinline__ void match_measured(Lane &L)
{
    L.ml += kMinMatch;
    if (L.off > L.op - L.floor_) {
        fail_block(L);
        return;
    }
    if (L.off == 0) {   // liblz4 writes zeros: the wave kernel decodes the frame
        finish(L, ST_NOT_RUN);
        return;
    }
    if (L.op + L.ml > L.oend - kLastLiterals) {
        fail_block(L);
        return;
    }
    if (L.op + L.ml > L.dlen) {
        finish(L, ST_DST_OVERFLOW);
        return;
    }
    L.mrem = L.ml;
    L.mdone = 0;
    L.ph = P_MATCH;
}

__device__ __forceinline__ void do_off(Lane &L)
{
    if (!have(L, L.ip, 2))
        return;
    L.off = rb(L, L.ip) | (rb(L, L.ip + 1) << 8);
    L.ip += 2;
    L.ml = L.tok & 15;
    if (L.ml == 15) {
        L.ph = P_MLLEN;
        return;
    }
    match_measured(L);
}

__device__ __forceinline__ void do_mllen(Lane &L)
{
    for (;;) {
        if (L.ip >= L.iend) {
            fail_block(L);
            return;
        }
        if (!have(L, L.ip, 1))
            return;
        const uint32_t s = rb(L, L.ip++);
        L.ml += s;
        if (L.ip >= L.iend - (kLastLiterals - 1)) {
            fail_block(L);
            return;
        }
        if (s != 255)
            break;
    }
    match_measured(L);
}

// Issue the next chunk (<= 64 bytes) of the current match into slot S once
// every byte it reads is final: below `pend`, the first output byte still
// owned by a pending slot (older slots a, b, c, or S's own literal).
__device__ __forceinline__ void do_match(Lane &L, Slot &S, uint32_t pend, uint32_t &src0,
                                         uint32_t &src1, uint32_t &src2, uint32_t &src3)
{
    const uint32_t off = L.off, ml = L.ml;
    const uint32_t mb = L.op - L.mdone;   // match start (frame output offset)
    const bool over = off < ml;
    const uint32_t need = over ? mb : mb - off + ml;   // end of the bytes the copy reads
    if (need > pend)
        return;   // wait for the pending slot to land
    const uint32_t x0 = L.mdone;
    const uint32_t n = L.mrem < (over ? 48u : 64u) ? L.mrem : (over ? 48u : 64u);
    S.mx = L.ox0 + mb + x0;
    S.lmn |= n << 8;
    if (over) {
        const uint32_t mph = x0 % off;
        S.ovr = off | (mph << 16);
        const uint32_t s = L.ox0 + mb - off;
        src3 = s;   // the pattern
        if (off >= 16) {
            src0 = s + mph;
            src1 = n > 16 ? s + (mph + 16) % off : kOff;
            src2 = n > 32 ? s + (mph + 32) % off : kOff;
        }
    } else {
        S.ovr = 0;
        const uint32_t s = L.ox0 + mb - off + x0;
        src0 = s;
        src1 = n > 16 ? s + 16 : kOff;
        src2 = n > 32 ? s + 32 : kOff;
        src3 = n > 48 ? s + 48 : kOff;
    }
    L.mdone += n;
    L.mrem -= n;
    L.op += n;
    if (L.mrem == 0)
        L.ph = P_TOKEN;
}

__device__ __forceinline__ void do_end(Lane &L)
{
    L.fail_op = L.op;
    if (L.flg_csize && L.csize != L.op) {
        finish(L, ST_FRAME_SIZE);
        return;
    }
    finish(L, L.op != L.dlen ? ST_SHORT_FRAME : ST_OK);
}

// Fast path: a whole sequence whose literal run (<= 32 bytes), offset and
// length bytes (at most one extension byte each) sit in the ring — the
// common case.  Anything else (and every error) is left to the
// byte-at-a-time handlers above, which re-parse from the token.
__device__ __forceinline__ void seq_fast(Lane &L)
{
    const uint32_t ip = L.ip;
    if (ip >= L.iend || !have(L, ip, L.iend - ip < 2 ? 1 : 2))
        return;
    const uint32_t x = L.cx0 + ip, xa = x & ~3u, sh = x & 3;
    const uint32_t w = __builtin_amdgcn_alignbyte(lds_u32(ring_addr(L, xa + 4)),
                                                  lds_u32(ring_addr(L, xa)), sh);
    const uint32_t tok = w & 0xFF;
    uint32_t lit = tok >> 4, t = 1;
    if (lit == 15) {
        const uint32_t e = (w >> 8) & 0xFF;
        if (e == 255 || L.iend - (ip + 1) <= 15)
            return;
        lit += e;
        t = 2;
    }
    const uint32_t p = ip + t;
    if (L.op + lit > L.oend - kMfLimit || L.iend - p < lit + 2 + 1 + kLastLiterals) {
        // the block's last sequence: literals only, ending the block exactly
        if (L.iend - p != lit || L.op + lit > L.oend || L.op + lit > L.dlen)
            return;
        L.tok = tok;
        L.lit = lit;
        L.lrem = lit;
        L.stored = 2;
        L.ip = p;
        L.ph = P_LIT;
        return;
    }
    if (L.op + lit > L.dlen)
        return;
    const uint32_t q = p + lit;   // offset, then the first length extension byte
    if (!have(L, q, 3))
        return;
    const uint32_t y = L.cx0 + q, ya = y & ~3u;
    const uint32_t o4 = __builtin_amdgcn_alignbyte(lds_u32(ring_addr(L, ya + 4)),
                                                   lds_u32(ring_addr(L, ya)), y & 3);
    const uint32_t off = o4 & 0xFFFF;
    uint32_t ml = tok & 15, p2 = q + 2;
    if (ml == 15) {
        if (p2 >= L.iend)
            return;
        const uint32_t e2 = (o4 >> 16) & 0xFF;
        p2++;
        if (e2 == 255 || p2 >= L.iend - (kLastLiterals - 1))
            return;
        ml += e2;
    }
    ml += kMinMatch;
    const uint32_t mb = L.op + lit;
    if (off == 0 || off > mb - L.floor_ || mb + ml > L.oend - kLastLiterals || mb + ml > L.dlen)
        return;
    // commit: literal run (copied by do_lit, possibly over several
    // iterations), then the match
    L.tok = tok;
    L.lit = lit;
    L.lrem = lit;
    L.off = off;
    L.ml = ml;
    L.ipm = p2;
    L.mparsed = 1;
    L.ip = p;
    L.ph = P_LIT;
}

// One iteration of one lane, using pipeline slot S; `older` = the first
// output byte still owned by the lane's older pending slots (kOff if none).
template <int DIAG>
__device__ __forceinline__ void step(Lane &L, Slot &S, uint32_t older)
{
    retire<DIAG>(L, S);
    uint32_t s0 = kOff, s1 = kOff, s2 = kOff, s3 = kOff;
    if (L.ph == P_TOKEN)
        seq_fast(L);
    if (L.ph == P_TOKEN)
        do_token(L);
    if (L.ph == P_LITLEN)
        do_litlen(L);
    if (L.ph == P_LIT)
        do_lit(L, S);
    if (L.ph == P_OFF)
        do_off(L);
    if (L.ph == P_MLLEN)
        do_mllen(L);
    if (L.ph == P_MATCH) {
        // first output byte still owned by a pending slot
        const uint32_t pend = older != kOff ? older : S.lmn ? slot_wlo(L, S) : L.op - L.mdone;
        do_match(L, S, pend, s0, s1, s2, s3);
    }
    if (L.ph == P_BHDR)
        do_bhdr(L);
    if (L.ph == P_END)
        do_end(L);
    if (DIAG & 2)
        s0 = s1 = s2 = s3 = kOff;
    S.m0 = bload16(L.cout, s0);
    S.m1 = bload16(L.cout, s1);
    S.m2 = bload16(L.cout, s2);
    S.m3 = bload16(L.cout, s3);
    // ring fill: 64 bytes if there is room behind the oldest byte still needed
    // ring bytes below keep - 192 are consumed: the literal runs of pending
    // slots (at most 4 x 32 bytes before ip) are read back at retire
    const uint32_t keep = L.cx0 + L.ip;
    const bool fill = L.ph != P_DONE && L.fill < L.cx0 + L.clen && L.fill + kFill <= keep - 192 + kRing;
    const uint32_t fx = fill ? L.fill : kOff;
    S.wx = fx;
    S.w0 = bload16(L.cin, fx);
    S.w1 = bload16(L.cin, fill ? fx + 16 : kOff);
    if (fill)
        L.fill += kFill;
}

__device__ __forceinline__ bool slot_busy(const Slot &S)
{
    return S.wx != kOff || S.lmn != 0;
}

// DIAG (tuning builds only): 1 = no output stores, 2 = no match loads
template <int DIAG>
__global__ __launch_bounds__(64 * kLaneWaves) __attribute__((amdgpu_waves_per_eu(1, 1))) void lz4_lane_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    uint8_t *__restrict__ out, int32_t *__restrict__ status, uint32_t *__restrict__ fail_at)
{
    __shared__ __attribute__((aligned(16))) uint8_t rings[kLaneWaves * 64 * kRingStride];
    const uint32_t f = blockIdx.x * (64 * kLaneWaves) + threadIdx.x;
    const bool act = f < n;
    FrameDesc d = {0, 0, 0, 0};
    if (act)
        d = desc[f];
    // per-wave resources over the wave's frames
    // (wave-uniform: broadcast from lane 0 so they live in scalar registers)
    const uint64_t clo = uni64(wave_min64(act ? d.c_off : ~0ull));
    const uint64_t chi = uni64(wave_max64(act ? d.c_off + d.c_size : 0ull));
    const uint64_t olo = uni64(wave_min64(act ? d.d_off : ~0ull));
    const uint64_t ohi = uni64(wave_max64(act ? d.d_off + d.d_size : 0ull));
    const uint32_t cap = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(wave_max64(act ? (uint64_t)d.c_size + d.d_size / 4 : 0ull) / 2 + 256));
    if (!act)
        return;
    Lane L;
    const uintptr_t cbase = reinterpret_cast<uintptr_t>(comp + clo) & ~(uintptr_t)15;
    const uint64_t cspan = reinterpret_cast<uintptr_t>(comp + chi) - cbase;
    const uint64_t ospan = ohi - olo;
    L.cin = __builtin_amdgcn_make_buffer_rsrc((void *)cbase, 0, (int)(uint32_t)((cspan + 3) & ~3ull), 0x00020000);
    L.cout = __builtin_amdgcn_make_buffer_rsrc((void *)(out + olo), 0, (int)(uint32_t)ospan, 0x00020000);
    L.cx0 = (uint32_t)(reinterpret_cast<uintptr_t>(comp + d.c_off) - cbase);
    L.ox0 = (uint32_t)(d.d_off - olo);
    L.oend_x = L.ox0 + d.d_size;
    L.clen = d.c_size;
    L.dlen = d.d_size;
    L.ring = (uint32_t)(uintptr_t)(rings) + threadIdx.x * kRingStride;
    L.fill = L.cx0 & ~(kFill - 1);
    L.avail = L.fill;
    L.ph = P_HDR;
    L.st = ST_NOT_RUN;
    L.ip = 0;
    L.op = 0;
    L.fail_op = 0;
    L.flg_csize = 0;
    L.csize = 0;
    L.stored = 0;
    L.lrem = L.mrem = L.mdone = 0;
    L.ipm = L.mparsed = 0;
    L.tok = L.lit = L.ml = L.off = 0;
    L.indep = L.bsid = L.max_block = 0;
    L.iend = L.oend = L.floor_ = L.bop = 0;
    // spans beyond 32-bit offsets: leave the frame to the wave kernel
    if (cspan >= 0x7FFFFF00ull || ospan >= 0x7FFFFF00ull)
        L.ph = P_DONE;
    Slot sl[kSlots];
#pragma unroll
    for (int i = 0; i < (int)kSlots; i++) {
        sl[i].wx = kOff;
        sl[i].lx = kOff;
        sl[i].lmn = 0;
        sl[i].ovr = 0;
    }
    // frame header: the first 128 ring bytes are loaded synchronously
    if (L.ph == P_HDR) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint32_t fx = L.fill;
            const u32x4 a = bload16(L.cin, fx), b = bload16(L.cin, fx + 16);
            const uint32_t ra = ring_addr(L, fx);
            lds_w128(ra, a);
            lds_w128(ra + 16, b);
            L.fill += kFill;
        }
        L.avail = L.fill;
        const int32_t hs = hdr_status(L);
        if (hs >= 0)
            finish(L, hs);
        else
            L.ph = P_BHDR;
    }
    uint32_t rounds = 0;
    for (;;) {
#pragma unroll
        for (int k = 0; k < (int)kSlots; k++) {
            // oldest pending slot after k: k+1, k+2, ... (mod kSlots)
            uint32_t older = kOff;
#pragma unroll
            for (int j = (int)kSlots - 1; j >= 1; j--) {
                const Slot &o = sl[(k + j) % kSlots];
                older = o.lmn ? slot_wlo(L, o) : older;
            }
            step<DIAG>(L, sl[k], older);
        }
        bool busy = L.ph != P_DONE;
#pragma unroll
        for (int i = 0; i < (int)kSlots; i++)
            busy = busy || slot_busy(sl[i]);
        if (!__any(busy))
            break;
        if (++rounds > cap) {
            if (busy)
                L.st = ST_NOT_RUN;
            break;
        }
    }
    status[f] = L.st;
    if (fail_at)
        fail_at[f] = L.fail_op;
}

}   // namespace

int launch_lz4_lane(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    uint8_t *d_out, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream,
                    int diag)
{
    if (nframes == 0)
        return 0;
    const uint32_t per = 64 * kLaneWaves;
    const dim3 grid((nframes + per - 1) / per), block(per);
    switch (diag) {
    case 1: hipLaunchKernelGGL(lz4_lane_kernel<1>, grid, block, 0, stream, d_desc, nframes, d_comp, d_out, d_status, d_fail_at); break;
    case 4: hipLaunchKernelGGL(lz4_lane_kernel<4>, grid, block, 0, stream, d_desc, nframes, d_comp, d_out, d_status, d_fail_at); break;
    case 3: hipLaunchKernelGGL(lz4_lane_kernel<3>, grid, block, 0, stream, d_desc, nframes, d_comp, d_out, d_status, d_fail_at); break;
    default: hipLaunchKernelGGL(lz4_lane_kernel<0>, grid, block, 0, stream, d_desc, nframes, d_comp, d_out, d_status, d_fail_at); break;
    }
    if (hipGetLastError() != hipSuccess)
        return -1;
    if (diag)
        return 0;
    return launch_lz4_wave_deferred(d_desc, nframes, d_comp, d_out, d_status, d_fail_at, stream);
}

}   // namespace zsk
