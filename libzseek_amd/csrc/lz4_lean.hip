// lz4_lean.hip — parse phase of the two-phase LZ4 decoder, lane per frame,
// streaming, lean fast path (gfx950).
//
// Same outputs as lz4_scan_kernel (per-frame status, fail_at, item count and
// the 8-byte sequence items of lz4_split.hip's format, without the padding
// item older execute kernels needed) and the same liblz4 1.9.3 validation
// (parse_block / parse_frame in lz4_split.hip, decode_block in
// oracle/lz4_oracle.c), with a shorter step:
//
//   * one sub-step parses one whole sequence — token, literal length with at
//     most one extension byte, offset, match length with at most one
//     extension byte — from two 4-byte reads of a 512-byte per-lane LDS ring,
//     checks every liblz4 rule that applies to it, and stores its item(s)
//     with one 16-byte store (a short item's second half is overwritten by
//     the next item);
//   * anything else (a longer extension chain, the block's last sequence,
//     block headers, stored blocks, the end mark, every failure) goes to the
//     exact byte-at-a-time step, which runs only when some lane of the wave
//     needs it;
//   * the ring is filled through a D-deep software pipeline of 32-byte
//     loads (one slot retired into the ring and one load issued per
//     sub-step, every sub-step issuing the same vector-memory ops so the
//     compiler's vmcnt waits retire exactly the slot consumed).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kItemExt = 0x80000000u;
constexpr uint32_t kItemPos = 0x3FFFFFFFu;
constexpr uint32_t kLW = 4;              // waves per workgroup
constexpr uint32_t kRing = 256;          // per-lane ring bytes
// per lane: ring [0, 256), mirror of ring bytes [0, 16) at [256, 272) (4-byte
// reads never wrap), a 32-byte sink for disabled writes at [272, 304), the
// item buffer (32 slots = two 128-byte lines) at [304, 560)
constexpr uint32_t kMirror = 256, kSink = 272, kIBuf = 304;
constexpr uint32_t kStride = 560;        // bytes between lanes' areas
// (an odd dword count spreads same-offset accesses over every LDS bank but
// misaligns the 16-byte ring and item writes: 564 / 568 bytes 4.46 / 4.32 vs
// 4.02 ms per launch at config 2)
constexpr uint32_t kFlush = 8;           // item lines written per flush (one store)
// The fill keeps the ring within [ip, ip + kRing - 16) and moves in 32-byte
// slots; a literal run whose offset lies past what has arrived is taken in
// two halves (fast())
constexpr uint32_t kOff = 0x80000000u;   // out-of-range buffer offset: op disabled

enum : uint32_t { P_TOKEN = 0, P_LEXT, P_OFF, P_MEXT, P_BHDR, P_END, P_DONE };

struct Fill {
    u32x4 a, b, c, d;   // ring bytes [x, x + 64): the first 32, and the second 32 if h2
    uint32_t x;         // ring coordinate, or kOff
    bool h2;
};

struct Lane {
    __amdgpu_buffer_rsrc_t cin, irs;   // compressed bytes; items (byte offsets)
    uint32_t cx0;                      // coordinate of frame byte 0 in cin
    uint32_t clen, dlen;
    uint32_t ring;                     // LDS address of the lane's ring
    uint32_t fill, avail;              // next coordinate to load; coordinates < avail are in the ring
    uint32_t ph;
    int32_t st;
    uint32_t ip, op, fail_op;
    uint32_t csz_flag;
    uint64_t csize;
    uint32_t indep, bsid, max_block;
    uint32_t iend, oend, floor_, bop;
    uint32_t mlim;                     // min(oend - LASTLITERALS, dlen): a match's end bound
    uint32_t tok, lsrc, nlit;          // sequence whose offset is pending (P_OFF, slow step)
    uint32_t acc, moff;                // partial extension sum (P_LEXT / P_MEXT), offset (P_MEXT)
    uint32_t stop;                     // block route: the header that ends the job (else ~0)
    uint32_t ib, k, cap;               // item 0 at irs byte 8*ib; k emitted, cap slots
    uint32_t kf;                       // items [0, kf) written to HBM (a multiple of 16)
    // the sub-step's item store: slots k0, k0+1 (nk = 0: none)
    uint32_t ia, ibw, ia2, ib2, nk;
    uint32_t cnt[22];  // DIAG 4: sub-steps fast / exact-needed / waiting / done / slow-run, sequences,
                       // then per exact-needed sub-step the failed rules (why bits) and the phase
    uint32_t why;      // DIAG 4: the fast step's failed rules (bit per slack, see fast())
};

constexpr int kLeanStats = 22;
__device__ unsigned long long g_lean_stats[kLeanStats];

__device__ __forceinline__ uint32_t lds_u32(uint32_t a)
{
    return *reinterpret_cast<const __attribute__((address_space(3))) uint32_t *>(
        (__attribute__((address_space(3))) void *)(uintptr_t)a);
}

__device__ __forceinline__ uint32_t lds_u8(uint32_t a)
{
    return *reinterpret_cast<const __attribute__((address_space(3))) uint8_t *>(
        (__attribute__((address_space(3))) void *)(uintptr_t)a);
}

template <typename T>
__device__ __forceinline__ __attribute__((address_space(3))) T *lp(uint32_t a)
{
    return (__attribute__((address_space(3))) T *)(uintptr_t)a;
}

__device__ __forceinline__ void lds_w128(uint32_t a, u32x4 v)
{
    *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(
        (__attribute__((address_space(3))) void *)(uintptr_t)a) = v;
}

__device__ __forceinline__ uint32_t raddr(const Lane &L, uint32_t x)
{
    return L.ring + (x & (kRing - 1));
}

__device__ __forceinline__ bool have(const Lane &L, uint32_t p, uint32_t n)
{
    return L.cx0 + p + n <= L.avail;
}

__device__ __forceinline__ uint32_t rb(const Lane &L, uint32_t p)
{
    return lds_u8(raddr(L, L.cx0 + p));
}

// 4 frame bytes from p: two adjacent dwords (the mirror covers the wrap)
__device__ __forceinline__ uint32_t r4(const Lane &L, uint32_t p)
{
    const uint32_t x = L.cx0 + p;
    const uint32_t a = L.ring + (x & (kRing - 4));
    return __builtin_amdgcn_alignbyte(lds_u32(a + 4), lds_u32(a), x & 3);
}

// ring bytes [x, x + 32) (x 32-aligned) from a retired slot, or into the
// sink when off; ring bytes [0, 16) are mirrored at kMirror
__device__ __forceinline__ void ring_put(const Lane &L, uint32_t x, u32x4 a, u32x4 b, bool on)
{
    const uint32_t i = x & (kRing - 1);
    lds_w128(L.ring + (on ? i : kSink), a);
    lds_w128(L.ring + (on ? i + 16 : kSink + 16), b);
    lds_w128(L.ring + ((on && i == 0) ? kMirror : kSink), a);
}

__device__ __forceinline__ uint32_t rd32(const Lane &L, uint32_t p)
{
    return rb(L, p) | (rb(L, p + 1) << 8) | (rb(L, p + 2) << 16) | (rb(L, p + 3) << 24);
}

__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t x)
{
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, x, 0, 0));
}

__device__ __forceinline__ void finish(Lane &L, int32_t st)
{
    L.st = st;
    L.ph = P_DONE;
}

__device__ __forceinline__ void fail_block(Lane &L)
{
    const bool direct = (L.dlen - L.bop) >= L.max_block;
    const int32_t bits = (int32_t)((L.bsid - 4) << ST_BSID_SHIFT);
    finish(L, (direct ? (ST_GENERIC | ST_DIRECT_FLAG) : ST_DECOMPRESS_FAILED) | ST_BLOCK_FAIL_FLAG | bits);
}

// stage a sequence's item(s) for this sub-step's store; false: no slots left
__device__ __forceinline__ bool emit(Lane &L, uint32_t lsrc, uint32_t lit, uint32_t off, uint32_t ml)
{
    if (L.k + 2 > L.cap)
        return false;   // (the item buffer has room: slow() checked)
    if (lit > 255 || ml > 258) {
        L.ia = lsrc | kItemExt;
        L.ibw = off;
        L.ia2 = lit;
        L.ib2 = ml;
        L.nk = 2;
    } else {
        L.ia = lsrc;
        L.ibw = off | (lit << 16) | ((ml ? ml - 3 : 0) << 24);
        L.ia2 = 0;
        L.ib2 = 0;
        L.nk = 1;
    }
    return true;
}

// ---- frame header (LZ4F_decodeHeader order; as parse_frame) ------------------
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
    const uint32_t n = hdr - 5;   // XXH32(descriptor, 0): bytes [4, hdr - 1)
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
    L.csz_flag = csz;
    L.bsid = bsid;
    if (csz)
        L.csize = (uint64_t)rd32(L, 6) | ((uint64_t)rd32(L, 10) << 32);
    L.max_block = 1u << (8 + 2 * bsid);
    L.ip = hdr;
    return -1;
}

// ---- fast step: one whole ordinary sequence, or half of one -------------------
// Every liblz4 rule that an ordinary sequence meets, as one min over signed
// slacks (no short-circuit branches): the token and offset bytes are in the
// ring, at most one extension byte each (lit <= 269, ml <= 273), not the
// block's last sequence (input side: the offset and 8 more bytes lie inside
// the block — which also covers the extension-byte bounds; output side:
// op + lit <= oend - MFLIMIT), 1 <= off <= op + lit - floor, the match ends
// by min(oend - LASTLITERALS, dSize), two item slots free.
// A sequence whose token passes its rules while its offset bytes are not in
// the ring yet (a literal run longer than the ring reaches, or bytes still in
// flight) takes its literal half now: the lane moves to the offset in phase
// P_OFF (lit_done's state: lsrc, nlit, op past the literals) and the fill
// restarts the stream there; the match half is then this same step in P_OFF
// (w is the offset word, the token kept in L.tok).  Round 3 sent such
// literals (~10 per 64 KiB frame at the frames' starts) to the exact step.
// Returns true when the lane needs the exact step (a rule failed for a reason
// other than bytes still in flight, or the lane is in another phase).
// (fe: the flush-table entry read with the token; the line it names is read
// with the offset, so the flush adds no LDS round trip of its own)
__device__ __forceinline__ bool fast(Lane &L, uint32_t fe, uint32_t pc, u32x4 &fv)
{
    const uint32_t ip = L.ip, ph = L.ph;
    const bool po = ph == P_OFF;
    const uint32_t w = r4(L, ip);
    const uint32_t tok = w & 0xFF, e = (w >> 8) & 0xFF;
    const bool lext = (tok >> 4) == 15;
    const uint32_t lit = lext ? 15 + e : tok >> 4;
    const uint32_t p = ip + (lext ? 2 : 1);
    const uint32_t q = p + lit;
    fv = *lp<u32x4>(fe + 16 * pc);
    const uint32_t o4q = r4(L, q);
    const uint32_t qq = po ? ip : q;
    const uint32_t o4 = po ? w : o4q;
    const uint32_t mtok = po ? L.tok : tok;
    const uint32_t off = o4 & 0xFFFF, e2 = (o4 >> 16) & 0xFF;
    const bool mext = (mtok & 15) == 15;
    const uint32_t ml = (mext ? 15 + e2 : mtok & 15) + kMinMatch;
    const uint32_t nip = qq + (mext ? 3 : 2);
    const uint32_t lt = po ? L.nlit : lit, ls = po ? L.lsrc : p;
    const uint32_t cop = po ? L.op : L.op + lit;
    const int32_t s_av = (int32_t)(L.avail - (L.cx0 + qq + 3));
    const int32_t s_in = (int32_t)(L.iend - qq - 8);
    // one extension byte at most (lit <= 269, ml <= 273); the literal half's
    // rules hold already in P_OFF
    const int32_t s_lx = (!po & lext & (e == 255)) ? -1 : 0, s_mx = (int32_t)(273 - ml);
    const int32_t s_mf = po ? 0 : (int32_t)(L.oend - kMfLimit - cop);
    const int32_t s_dl = po ? 0 : (int32_t)(L.dlen - cop);
    const int32_t s_off = min((int32_t)(off - 1), (int32_t)(cop - L.floor_ - off));
    const int32_t s_end = (int32_t)(L.mlim - cop - ml);
    const int32_t s_cap = (int32_t)(min(L.cap, L.kf + 32) - L.k - 2);   // slots, and room in the buffer
    const int32_t s_ph = ((ph == P_TOKEN) | po) ? 0 : -1;
    const int32_t s_t = min(min(s_in, s_dl), min(s_lx, s_mf));   // the literal half's rules
    const int32_t slack = min(min(min(s_av, s_t), min(s_mx, s_off)), min(s_end, min(s_cap, s_ph)));
    const bool go = slack >= 0;
    const bool tok_av = (int32_t)(L.avail - (L.cx0 + ip + 2)) >= 0;
    // the literal half alone: a token whose rules hold, offset bytes not in
    const bool half = (ph == P_TOKEN) & tok_av & (s_t >= 0) & (s_av < 0);
    L.why = (s_av < 0) | (s_in < 0) << 1 | (s_lx < 0) << 2 | (s_mf < 0) << 3 | (s_mx < 0) << 4 |
            (s_off < 0) << 5 | (s_end < 0) << 6 | (s_cap < 0) << 7 | (!po & (ph != P_TOKEN)) << 8;
    const bool big = (lt > 255) | (ml > 258);
    L.ia = big ? ls | kItemExt : ls;
    L.ibw = big ? off : off | (lt << 16) | ((ml - 3) << 24);
    L.ia2 = lt;
    L.ib2 = ml;
    L.nk = go ? (big ? 2 : 1) : 0;
    L.ip = go ? nip : (half ? q : ip);
    L.op = go ? cop + ml : (half ? cop : L.op);
    L.lsrc = half ? p : L.lsrc;
    L.nlit = half ? lit : L.nlit;
    L.tok = half ? tok : L.tok;
    L.ph = go ? (uint32_t)P_TOKEN : (half ? (uint32_t)P_OFF : ph);
    // waiting, not failing: the token bytes are not in yet (and exist), or
    // the item buffer waits for a flush
    const bool full = L.k + 2 > L.kf + 32;
    const bool wait = (!tok_av & (ip + 2 <= L.clen)) | full;
    // the exact step's phases (P_OFF included) wait here too while their
    // next bytes are in flight (4 from ip, or the frame's end), rather than
    // run to find out
    const bool x_wait = (ph != P_END) & ((int32_t)(L.avail - (L.cx0 + ip + 4)) < 0) & (ip + 4 <= L.clen);
    return !go & !half & (ph != P_DONE) & (((ph != P_TOKEN) | po) ? !x_wait & !(po & full) : !wait);
}

// ---- exact step: byte at a time, every rule (parse_block / parse_frame) ------
// Returns with the lane waiting when bytes are not yet in the ring; a length
// extension chain is resumable (P_LEXT / P_MEXT keep the partial sum and the
// position), so the ring always advances.
__device__ __forceinline__ void lit_done(Lane &L, uint32_t p, uint32_t lit)
{
    if (L.op + lit > L.oend - kMfLimit || L.iend - p < lit + 2 + 1 + kLastLiterals) {
        // the block's last sequence: literals only, ending the block
        if (L.iend - p != lit || L.op + lit > L.oend) {
            fail_block(L);
            return;
        }
        if (L.op + lit > L.dlen) {
            finish(L, ST_DST_OVERFLOW);
            return;
        }
        if (!emit(L, p, lit, 0, 0)) {
            finish(L, ST_NOT_RUN);
            return;
        }
        L.op += lit;
        L.ip = L.iend;
        L.ph = P_BHDR;
        return;
    }
    if (L.op + lit > L.dlen) {
        finish(L, ST_DST_OVERFLOW);
        return;
    }
    L.lsrc = p;
    L.nlit = lit;
    L.op += lit;
    L.ip = p + lit;
    L.ph = P_OFF;
}

__device__ __forceinline__ void match_done(Lane &L, uint32_t p, uint32_t off, uint32_t ml)
{
    ml += kMinMatch;
    if (off > L.op - L.floor_) {
        fail_block(L);
        return;
    }
    if (off == 0) {   // liblz4 writes zeros: the wave kernel decodes it
        finish(L, ST_NOT_RUN);
        return;
    }
    if (L.op + ml > L.oend - kLastLiterals) {
        fail_block(L);
        return;
    }
    if (L.op + ml > L.dlen) {
        finish(L, ST_DST_OVERFLOW);
        return;
    }
    if (!emit(L, L.lsrc, L.nlit, off, ml)) {
        finish(L, ST_NOT_RUN);
        return;
    }
    L.op += ml;
    L.ip = p;
    L.ph = P_TOKEN;
}

__device__ __forceinline__ void slow(Lane &L)
{
    if (L.k + 2 > L.kf + 32)
        return;   // the item buffer waits for a flush
    if (L.ph == P_TOKEN) {
        uint32_t p = L.ip;
        if (p >= L.iend) {
            fail_block(L);
            return;
        }
        if (!have(L, p, 1))
            return;
        const uint32_t tok = rb(L, p++);
        L.tok = tok;
        if ((tok >> 4) != 15) {
            lit_done(L, p, tok >> 4);
            return;
        }
        if (L.iend - p <= 15) {
            fail_block(L);
            return;
        }
        L.acc = 15;
        L.ip = p;
        L.ph = P_LEXT;
    }
    if (L.ph == P_LEXT) {
        uint32_t p = L.ip, lit = L.acc, e;
        do {
            if (p >= L.iend) {
                fail_block(L);
                return;
            }
            if (!have(L, p, 1)) {
                L.ip = p;
                L.acc = lit;
                return;
            }
            e = rb(L, p++);
            lit += e;
        } while (e == 255);
        lit_done(L, p, lit);
        return;
    }
    if (L.ph == P_OFF) {
        uint32_t p = L.ip;
        if (!have(L, p, 2))
            return;
        const uint32_t off = rb(L, p) | (rb(L, p + 1) << 8);
        p += 2;
        if ((L.tok & 15) != 15) {
            match_done(L, p, off, L.tok & 15);
            return;
        }
        L.moff = off;
        L.acc = 15;
        L.ip = p;
        L.ph = P_MEXT;
    }
    if (L.ph == P_MEXT) {
        uint32_t p = L.ip, ml = L.acc, e;
        do {
            if (p >= L.iend) {
                fail_block(L);
                return;
            }
            if (!have(L, p, 1)) {
                L.ip = p;
                L.acc = ml;
                return;
            }
            e = rb(L, p++);
            ml += e;
            if (p >= L.iend - (kLastLiterals - 1)) {
                fail_block(L);
                return;
            }
        } while (e == 255);
        match_done(L, p, L.moff, ml);
        return;
    }
    if (L.ph == P_BHDR) {
        if (L.ip == L.stop) {   // block route: the job's block parsed
            finish(L, ST_OK);
            return;
        }
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
        } else {
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
            if (bh & 0x80000000u) {
                if (L.op + bsize > L.dlen) {
                    finish(L, ST_DST_OVERFLOW);
                    return;
                }
                if (!emit(L, L.ip, bsize, 0, 0)) {
                    finish(L, ST_NOT_RUN);
                    return;
                }
                L.op += bsize;
                L.ip += bsize;
                return;   // next block header
            }
            if (bsize == 0) {
                fail_block(L);
                return;
            }
            L.iend = L.ip + bsize;
            L.oend = L.op + L.max_block;
            L.floor_ = L.indep ? L.op : 0;
            L.mlim = min(L.oend - kLastLiterals, L.dlen);
            L.ph = P_TOKEN;
            return;
        }
    }
    if (L.ph == P_END) {
        L.fail_op = L.op;
        if (L.csz_flag && L.csize != L.op)
            finish(L, ST_FRAME_SIZE);
        else
            finish(L, L.op != L.dlen ? ST_SHORT_FRAME : ST_OK);
    }
}

// One sub-step with pipeline slot S: retire S into the ring (when it is the
// next 32 bytes of the stream: a jump orphans the slots in flight), parse one
// sequence (fast, else the exact step where needed), store its item(s),
// issue S's next load.  Branch-free but for the exact step.
// The flush of item lines, in two halves a sub-step apart: lanes with a
// complete 16-item line (up to kFlush of them, by rank) write its LDS address
// and HBM offset into the wave's table and count it flushed; next sub-step
// the table entry is read with the token, the line with the offset, and
// 8-lane group g stores line g — one 16-byte piece per lane, whole lines.
__device__ __forceinline__ uint32_t flush_hand(Lane &L, uint32_t tab)
{
    const bool ready = L.k - L.kf >= 16;
    const uint64_t rm = __ballot(ready);
    const uint32_t j = __builtin_amdgcn_mbcnt_hi((uint32_t)(rm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)rm, 0u));
    const bool mine = ready && j < kFlush;
    const uint32_t line = L.ring + kIBuf + 128 * ((L.kf >> 4) & 1);
    *lp<uint64_t>(mine ? tab + 8 * j : tab + 8 * kFlush) = ((uint64_t)(8 * (L.ib + L.kf)) << 32) | line;
    L.kf = mine ? L.kf + 16 : L.kf;
    return min((uint32_t)__builtin_popcountll(rm), kFlush);
}

template <int DIAG>
__device__ __forceinline__ void flush_store(const Lane &L, uint64_t fe, const u32x4 &fv, uint32_t g,
                                            uint32_t pc, uint32_t fcnt)
{
    const uint32_t at = (DIAG & 2) ? 16 * pc : (uint32_t)(fe >> 32) + 16 * pc;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, fv), L.irs,
                                           g < fcnt && !(DIAG & 1) ? at : kOff, 0, 0);
}

// One sub-step with pipeline slot S: retire S into the ring (when it is the
// next 32 bytes of the stream: a jump orphans the slots in flight), parse one
// sequence (fast, else the exact step where needed), buffer its item(s),
// store the lines handed over last sub-step and hand over new ones, issue
// S's next load.  Branch-free but for the exact step.
template <bool SLOW, bool FILL, int DIAG>
__device__ __forceinline__ void sub(Lane &L, Fill &S, uint32_t lane, uint32_t tab, uint32_t &fcnt)
{
    if (FILL) {
        const bool in = S.x == L.avail;
        ring_put(L, S.x, S.a, S.b, in);
        ring_put(L, S.x + 32, S.c, S.d, in && S.h2);
        L.avail = in ? L.avail + (S.h2 ? 64 : 32) : L.avail;
    }
    const uint32_t g = lane >> 3, pc = lane & 7;
    const uint64_t fe = *lp<uint64_t>(tab + 8 * (g < fcnt ? g : kFlush));
    u32x4 fv;
    const bool need = fast(L, (uint32_t)fe, pc, fv);
    if (DIAG & 4) {
        L.cnt[0] += L.nk != 0;
        L.cnt[1] += need;
        L.cnt[2] += L.nk == 0 && !need && L.ph != P_DONE;
        L.cnt[3] += L.ph == P_DONE;
        if (need) {
            for (int b = 0; b < 9; b++)
                L.cnt[6 + b] += (L.why >> b) & 1;
            L.cnt[15 + min(L.ph, 6u)] += 1;
        }
    }
    flush_store<DIAG>(L, fe, fv, g, pc, fcnt);
    if (SLOW && __builtin_expect(__ballot(need) != 0, 0)) {
        if (DIAG & 4)
            L.cnt[4] += 1;
        if (need)
            slow(L);
    }
    // the item(s) into the lane's buffer (slots k, k + 1 mod 32): after the
    // handed-over line was read
    auto put_items = [&]() {
        const uint32_t ibuf = L.ring + kIBuf;
        const uint32_t a0 = L.nk ? ibuf + 8 * (L.k & 31) : L.ring + kSink;
        const uint32_t a1 = L.nk == 2 ? ibuf + 8 * ((L.k + 1) & 31) : L.ring + kSink + 8;
        *lp<uint64_t>(a0) = ((uint64_t)L.ibw << 32) | L.ia;
        *lp<uint64_t>(a1) = ((uint64_t)L.ib2 << 32) | L.ia2;
        L.k += L.nk;
        L.nk = 0;
    };
    put_items();
    if (!(DIAG & 32)) {
        // a second sequence in the same sub-step when its bytes are in the
        // ring: the fill, flush and loop work then serve two (config 2, plan +
        // parse: 1.085 -> 1.032 ms; DIAG 32, tuning: one sequence, as round 3)
        u32x4 dv;
        (void)fast(L, L.ring + kSink, 0, dv);
        put_items();
    }
    wave_lds_sync();
    fcnt = flush_hand(L, tab);
    wave_lds_sync();
    if (!FILL)
        return;
    // the next byte needed was never requested (a long literal run was
    // skipped): restart the stream there
    const uint32_t need_x = L.cx0 + L.ip;
    const bool jump = need_x >= L.fill;
    L.fill = jump ? need_x & ~31u : L.fill;
    L.avail = jump ? L.fill : L.avail;
    // ring fill: 32 bytes if that leaves every byte from ip on intact, and 32
    // more if those do too
    const uint32_t lim = need_x + kRing - 16;
    const bool fl = (L.ph < P_END) & (L.fill < L.cx0 + L.clen) & (L.fill + 32 <= lim);
    const bool f2 = fl & (L.fill + 32 < L.cx0 + L.clen) & (L.fill + 64 <= lim);
    const uint32_t fx = fl ? L.fill : kOff;
    S.x = fx;
    S.h2 = f2;
    S.a = bload16(L.cin, fx);
    S.b = bload16(L.cin, fl ? fx + 16 : kOff);
    S.c = bload16(L.cin, f2 ? fx + 32 : kOff);
    S.d = bload16(L.cin, f2 ? fx + 48 : kOff);
    L.fill = fl ? L.fill + (f2 ? 64 : 32) : L.fill;
}

// DIAG (tuning builds): 1 = no line stores, 2 = every line to the wave's first line,
// 4 = sub-step outcome counters (printed), 8 / 16 = a 4- / 1-deep fill pipeline,
// 32 = one sequence per sub-step (round 3), 64 = every sub-step fills (D = 4:
// 1.260 ms against 1.085, not kept); a third sequence per sub-step measured
// 1.265 against 1.031 (removed)
// (default 2: at ~1,400 cycles per sub-step, 4 sub-steps cover the loads)
// D: fill pipeline depth (slots of up to 64 bytes, retired every other sub-step)
// BLK: the block route -- lane t parses job t of `jobs` (one LZ4 block from
// its header at the job's speculative output offset, every liblz4 rule, up
// to the next header) into the job's slots and result; n = the job slots.
template <int DIAG, int D, bool BLK>
__global__ __launch_bounds__(64 * kLW) __attribute__((amdgpu_waves_per_eu(1, 1))) void lz4_lean_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    const uint64_t *__restrict__ rec_base, uint64_t capacity, uint64_t *__restrict__ items,
    uint32_t *__restrict__ nitems, int32_t *__restrict__ status, uint32_t *__restrict__ fail_at,
    uint32_t max_csize, uint32_t min_csize, const BlockJob *__restrict__ jobs, BlockRes *__restrict__ jres,
    const uint32_t *__restrict__ njobs)
{
    __shared__ __attribute__((aligned(16))) uint8_t rings[kLW * 64 * kStride];
    __shared__ __attribute__((aligned(16))) uint64_t tabs[kLW * (kFlush + 1)];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t tab = (uint32_t)(uintptr_t)(tabs) + (threadIdx.x >> 6) * 8 * (kFlush + 1);
    const uint32_t f = blockIdx.x * (64 * kLW) + threadIdx.x;
    FrameDesc d = {0, 0, 0, 0};
    BlockJob J = {kNoJob, 0, 0, 0, 0, 0, 0, 0};
    bool act;
    if (BLK) {
        // min_csize: the job minimum (fewer planned: the chunk parse takes
        // the frames)
        const uint32_t nj = uni(*njobs);
        if (nj >= min_csize && f < nj && f < n)
            J = jobs[f];
        act = J.f != kNoJob;
        if (act)
            d = desc[J.f];
    } else {
        if (f < n)
            d = desc[f];
        // frames of max_csize bytes and more belong to lz4_chunk_kernel,
        // frames under min_csize to lz4_scan_kernel
        act = f < n && d.c_size < max_csize && d.c_size >= min_csize;
    }
    uint64_t rb0 = 0;
    uint32_t cap = 0;
    if (act) {
        rb0 = rec_base[BLK ? J.f : f] + J.slot_off * (uint32_t)BLK;
        cap = BLK ? J.slot_cap : slots_of(d.c_size);
    }
    const uint64_t clo = uni64(wave_min64(act ? d.c_off : ~0ull));
    const uint64_t chi = uni64(wave_max64(act ? d.c_off + d.c_size : 0ull));
    const uint64_t ilo = uni64(wave_min64(act ? rb0 : ~0ull));
    const uint64_t ihi = uni64(wave_max64(act ? rb0 + cap : 0ull));
    const uint64_t work = BLK ? (uint64_t)(J.stop - J.hpos) : (uint64_t)d.c_size;
    const uint32_t steps = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(wave_max64(act ? work : 0ull) * 2 + 64 * D + 1024));
    if (clo == ~0ull)
        return;   // no frame in this wave (inactive lanes stay: flushes take all 64)
    Lane L;
    const uintptr_t cbase = reinterpret_cast<uintptr_t>(comp + clo) & ~(uintptr_t)31;
    const uint64_t cspan = reinterpret_cast<uintptr_t>(comp + chi) - cbase;
    L.cin = __builtin_amdgcn_make_buffer_rsrc((void *)cbase, 0, (int)(uint32_t)((cspan + 3) & ~3ull), kRsrcDw3);
    const uint64_t ispan = (ihi - ilo) * 8;
    L.irs = __builtin_amdgcn_make_buffer_rsrc((void *)(items + ilo), 0, (int)(uint32_t)ispan, kRsrcDw3);
    L.ib = (uint32_t)(rb0 - ilo);
    L.cx0 = (uint32_t)(reinterpret_cast<uintptr_t>(comp + d.c_off) - cbase);
    L.clen = d.c_size;
    L.dlen = d.d_size;
    L.ring = (uint32_t)(uintptr_t)(rings) + threadIdx.x * kStride;
    L.fill = L.cx0 & ~31u;
    L.avail = L.fill;
    L.ph = P_BHDR;
    L.st = ST_NOT_RUN;
    L.ip = L.op = L.fail_op = 0;
    L.csz_flag = 0;
    L.csize = 0;
    L.indep = L.bsid = L.max_block = 0;
    L.iend = L.oend = L.floor_ = L.bop = L.mlim = 0;
    L.tok = L.lsrc = L.nlit = L.acc = L.moff = 0;
    L.k = L.kf = 0;
    L.stop = 0xFFFFFFFFu;
    L.cap = cap;
    L.ia = L.ibw = L.ia2 = L.ib2 = L.nk = 0;
    for (int i = 0; i < kLeanStats; i++)
        L.cnt[i] = 0;
    L.why = 0;
    if (!act || cspan >= 0x7FFFFF00ull || ispan >= 0x7FFFFF00ull || d.c_size > kItemPos ||
        rb0 + cap > capacity) {
        finish(L, ST_NOT_RUN);
    } else if (BLK) {
        // the job's block: its header's 128 bytes synchronously, the frame
        // header's fields from the plan
        L.ip = J.hpos;
        L.op = J.bop;
        L.stop = J.stop;
        L.bsid = J.info & 0xFF;
        L.indep = (J.info >> 8) & 1;
        L.max_block = 1u << (8 + 2 * L.bsid);
        L.fill = (L.cx0 + J.hpos) & ~31u;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t fx = L.fill;
            const u32x4 a = bload16(L.cin, fx), b = bload16(L.cin, fx + 16);
            ring_put(L, fx, a, b, true);
            L.fill += 32;
        }
        L.avail = L.fill;
    } else {
        // frame header: the first 128 bytes, synchronously
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t fx = L.fill;
            const u32x4 a = bload16(L.cin, fx), b = bload16(L.cin, fx + 16);
            ring_put(L, fx, a, b, true);
            L.fill += 32;
        }
        L.avail = L.fill;
        const int32_t hs = hdr_status(L);
        if (hs >= 0)
            finish(L, hs);
    }
    Fill sl[D];
#pragma unroll
    for (int i = 0; i < D; i++) {
        sl[i].x = kOff;
        sl[i].h2 = false;
    }
    uint32_t rounds = 0, fcnt = 0;
    // the table's sink entry names a valid line from the start
    *lp<uint64_t>(tab + 8 * kFlush) = L.ring + kIBuf;
    wave_lds_sync();
    for (;;) {
        // two sub-steps per slot: the first retires and refills it, the
        // second may run the exact step (DIAG 64, tuning: every sub-step
        // retires and refills its own slot, every other one may run the exact
        // step -- twice the fill rate at the same latency budget with D = 4)
        if (DIAG & 64) {
#pragma unroll
            for (int i = 0; i < D; i += 2) {
                sub<false, true, DIAG>(L, sl[i], lane, tab, fcnt);
                sub<true, true, DIAG>(L, sl[i + 1], lane, tab, fcnt);
            }
        } else {
#pragma unroll
            for (int i = 0; i < D; i++) {
                sub<false, true, DIAG>(L, sl[i], lane, tab, fcnt);
                sub<true, false, DIAG>(L, sl[i], lane, tab, fcnt);
            }
        }
        const bool busy = L.ph != P_DONE;
        if (!__any(busy))
            break;
        if (++rounds > steps) {
            if (busy)
                L.st = ST_NOT_RUN;
            break;
        }
    }
    // the lines handed over in the last sub-step
    {
        const uint32_t g = lane >> 3, pc = lane & 7;
        const uint64_t fe = *lp<uint64_t>(tab + 8 * (g < fcnt ? g : kFlush));
        const u32x4 fv = *lp<u32x4>((uint32_t)fe + 16 * pc);
        flush_store<DIAG>(L, fe, fv, g, pc, fcnt);
    }
    // the items not yet flushed: pairs of slots from the buffer (a pair past
    // k holds garbage in a slot below cap)
    for (uint32_t x = L.kf; x < L.k; x += 2) {
        const uint32_t a = L.ring + kIBuf + 8 * (x & 31);
        const u32x4 v = (u32x4){lp<uint32_t>(a)[0], lp<uint32_t>(a)[1],
                                lp<uint32_t>(L.ring + kIBuf + 8 * ((x + 1) & 31))[0],
                                lp<uint32_t>(L.ring + kIBuf + 8 * ((x + 1) & 31))[1]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), L.irs, 8 * (L.ib + x), 0, 0);
    }
    if ((DIAG & 4) && act) {
        L.cnt[5] = L.k;
        for (int i = 0; i < kLeanStats; i++)
            atomicAdd(&g_lean_stats[i], (unsigned long long)L.cnt[i]);
    }
    if (!act)
        return;
    if (BLK) {
        jres[f] = BlockRes{L.k, L.op, L.st, 0};
        return;
    }
    status[f] = L.st;
    nitems[f] = L.k;
    if (fail_at)
        fail_at[f] = L.fail_op;
}

}   // namespace

int launch_lz4_lean(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    const uint64_t *rec_base, uint64_t capacity, uint64_t *items, uint32_t *nitems,
                    int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream, uint32_t max_csize,
                    int diag, uint32_t min_csize)
{
    if (nframes == 0)
        return 0;
    const uint32_t per = 64 * kLW;
    const dim3 grid((nframes + per - 1) / per), block(per);
#define ZSK_LEAN(D, P)                                                                                         \
    hipLaunchKernelGGL((lz4_lean_kernel<D, P, false>), grid, block, 0, stream, d_desc, nframes, d_comp, rec_base, \
                       capacity, items, nitems, d_status, d_fail_at, max_csize, min_csize, nullptr, nullptr,       \
                       nullptr)
#ifdef ZSK_TUNING
    if (diag & 4) {
        unsigned long long z[kLeanStats] = {0};
        (void)hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lean_stats), z, sizeof(z), 0, hipMemcpyHostToDevice, stream);
        ZSK_LEAN(4, 2);
        (void)hipMemcpyFromSymbolAsync(z, HIP_SYMBOL(g_lean_stats), sizeof(z), 0, hipMemcpyDeviceToHost, stream);
        (void)hipStreamSynchronize(stream);
        const double fr = nframes;
        fprintf(stderr, "lean parse per frame: sub-steps fast %.1f exact-needed %.1f waiting %.1f done %.1f "
                        "exact-step runs %.1f items %.1f\n", z[0] / fr, z[1] / fr, z[2] / fr, z[3] / fr, z[4] / fr, z[5] / fr);
        fprintf(stderr, "  exact-needed rules per frame: av %.1f in %.1f lx %.1f mf %.1f mx %.1f off %.1f end %.1f cap %.1f "
                        "phase %.1f; by phase TOKEN %.1f LEXT %.1f OFF %.1f MEXT %.1f BHDR %.1f END %.1f DONE %.1f\n",
                z[6] / fr, z[7] / fr, z[8] / fr, z[9] / fr, z[10] / fr, z[11] / fr, z[12] / fr, z[13] / fr, z[14] / fr,
                z[15] / fr, z[16] / fr, z[17] / fr, z[18] / fr, z[19] / fr, z[20] / fr, z[21] / fr);
    } else if ((diag & 96) == 96)
        ZSK_LEAN(96, 4);
    else if (diag & 64)
        ZSK_LEAN(64, 4);
    else if (diag & 32)
        ZSK_LEAN(32, 2);
    else if (diag & 2)
        ZSK_LEAN(2, 2);
    else if (diag & 1)
        ZSK_LEAN(1, 2);
    else if (diag & 8)
        ZSK_LEAN(0, 4);
    else if (diag & 16)
        ZSK_LEAN(0, 1);
    else
#else
    (void)diag;
#endif
        ZSK_LEAN(0, 2);
#undef ZSK_LEAN
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_lz4_lean_blocks(const FrameDesc *d_desc, const uint8_t *d_comp, const uint64_t *rec_base,
                           uint64_t capacity, uint64_t *items, const SplitScratch *s, uint32_t lanes,
                           uint32_t min_jobs, hipStream_t stream)
{
    if (lanes == 0)
        return 0;
    if (lanes > s->jobs_cap || !s->jobs || !s->jres || !s->njobs)
        return -1;
    const uint32_t per = 64 * kLW;
    hipLaunchKernelGGL((lz4_lean_kernel<0, 2, true>), dim3((lanes + per - 1) / per), dim3(per), 0, stream,
                       d_desc, lanes, d_comp, rec_base, capacity, items, nullptr, nullptr, nullptr, 0u,
                       min_jobs, s->jobs, s->jres, s->njobs);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
