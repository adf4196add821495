// lz4_scan.hip — parse phase of the two-phase LZ4 decoder, lane per frame,
// streaming (gfx950).
//
// Produces exactly what lz4_parse_kernel (lz4_split.hip) produces — per-frame
// status, item count and the 8-byte sequence items — with the same liblz4
// 1.9.3 validation order (parse_block / parse_frame there, decode_block in
// oracle/lz4_oracle.c), but never waits on a dependent global load:
//
//   * each lane's compressed bytes stream into a 128-byte LDS ring through a
//     D-deep software pipeline (32 bytes per sub-step; a slot's registers are
//     written to the ring D sub-steps after its load was issued);
//   * a sub-step parses one whole sequence from the ring (token + one
//     length-extension byte, offset + one extension byte: four dword reads)
//     and emits its item;
//   * each sub-step issues the same vector-memory ops (2 ring loads, 1 item
//     store; unused ones get an out-of-range offset), so the compiler's
//     vmcnt waits retire exactly the slot being consumed;
//   * everything rare — longer length extensions, block headers, stored
//     blocks, the end mark, every error — runs in a byte-at-a-time slow step
//     once per D sub-steps.
//
// A literal run longer than the ring lookahead makes the lane jump its fill
// pointer (in-flight slots are dropped); the literal bytes themselves are
// never read here (the execute phase copies them from HBM).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "lz4_dev.h"
#include "zsk_internal.h"

namespace zsk {

namespace {

using namespace lz4d;

constexpr uint32_t kItemExt = 0x80000000u;
constexpr uint32_t kItemPos = 0x3FFFFFFFu;
constexpr uint32_t kSW = 4;              // waves per workgroup
// per-lane ring bytes: 128 (4 waves per SIMD by LDS) parses the 4 KiB
// frames' config in 1.93 ms, 256 (2 waves) in 2.10, 512 (1 wave) in 2.27 —
// the many short chains want waves to hide their LDS round trips more than
// lookahead (a literal run past it only parks the offset for a sub-step);
// 64 bytes is too short for the frame header's synchronous first read
constexpr uint32_t kRing = 128;
constexpr uint32_t kStride = 144;        // bytes between lanes' rings (bank spread)
constexpr uint32_t kD = 3;               // pipeline depth (slots)
constexpr uint32_t kOff = 0x80000000u;   // out-of-range buffer offset: op disabled

enum : uint32_t { P_TOKEN = 0, P_OFF, P_BHDR, P_END, P_DONE };

struct Fill {
    u32x4 a, b;     // ring bytes [x, x + 32)
    uint32_t x;     // ring coordinate, or kOff
};

struct Scan {
    __amdgpu_buffer_rsrc_t cin, irs;   // compressed bytes; items (8-byte units)
    uint32_t cx0;      // coordinate of frame byte 0 in cin
    uint32_t clen, dlen;
    uint32_t ring;     // LDS address of the lane's ring
    uint32_t fill;     // next coordinate to load (16-aligned)
    uint32_t avail;    // coordinates < avail are in the ring
    uint32_t ph;
    int32_t st;
    uint32_t ip, op, fail_op;
    uint32_t csz_flag;
    uint64_t csize;
    uint32_t indep, bsid, max_block;
    uint32_t iend, oend, floor_, bop;
    uint32_t tok, lsrc, nlit;          // sequence whose offset is pending (P_OFF)
    // items: emitted k, stored ks (ks <= k), queue of k - ks <= 3
    uint32_t ib;       // item coordinate (8-byte units) of item 0 in irs
    uint32_t k, ks, cap;
    uint32_t q0a, q0b, q1a, q1b, q2a, q2b;
};

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

__device__ __forceinline__ void lds_w128(uint32_t a, u32x4 v)
{
    *reinterpret_cast<__attribute__((address_space(3))) u32x4 *>(
        (__attribute__((address_space(3))) void *)(uintptr_t)a) = v;
}

__device__ __forceinline__ uint32_t raddr(const Scan &L, uint32_t x)
{
    return L.ring + (x & (kRing - 1));
}

__device__ __forceinline__ bool have(const Scan &L, uint32_t p, uint32_t n)
{
    return L.cx0 + p + n <= L.avail;
}

__device__ __forceinline__ uint32_t rb(const Scan &L, uint32_t p)
{
    return lds_u8(raddr(L, L.cx0 + p));
}

// 4 frame bytes from p (two aligned dword reads)
__device__ __forceinline__ uint32_t r4(const Scan &L, uint32_t p)
{
    const uint32_t x = L.cx0 + p, xa = x & ~3u;
    return __builtin_amdgcn_alignbyte(lds_u32(raddr(L, xa + 4)), lds_u32(raddr(L, xa)), x & 3);
}

__device__ __forceinline__ uint32_t rd32(const Scan &L, uint32_t p)
{
    return rb(L, p) | (rb(L, p + 1) << 8) | (rb(L, p + 2) << 16) | (rb(L, p + 3) << 24);
}

__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t x)
{
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, x, 0, 0));
}

__device__ __forceinline__ void finish(Scan &L, int32_t st)
{
    L.st = st;
    L.ph = P_DONE;
}

__device__ __forceinline__ void fail_block(Scan &L)
{
    const bool direct = (L.dlen - L.bop) >= L.max_block;
    const int32_t bits = (int32_t)((L.bsid - 4) << ST_BSID_SHIFT);
    finish(L, (direct ? (ST_GENERIC | ST_DIRECT_FLAG) : ST_DECOMPRESS_FAILED) | ST_BLOCK_FAIL_FLAG | bits);
}

// ---- items (format: lz4_split.hip Sink) --------------------------------------
__device__ __forceinline__ void qpush(Scan &L, uint32_t a, uint32_t b)
{
    // selects, not a branch: a branch here becomes a stack slot
    const uint32_t n = L.k - L.ks;
    L.q0a = n == 0 ? a : L.q0a;
    L.q0b = n == 0 ? b : L.q0b;
    L.q1a = n == 1 ? a : L.q1a;
    L.q1b = n == 1 ? b : L.q1b;
    L.q2a = n >= 2 ? a : L.q2a;
    L.q2b = n >= 2 ? b : L.q2b;
    L.k++;
}

// queue a sequence's item(s); false: the frame's slots are exhausted
__device__ __forceinline__ bool emit(Scan &L, uint32_t lsrc, uint32_t lit, uint32_t off, uint32_t ml)
{
    if (lit > 255 || ml > 258) {
        const uint32_t pad = (L.k & 63) == 63 ? 1 : 0;
        if (L.k + pad + 2 > L.cap)
            return false;
        if (pad)
            qpush(L, 0, 0);
        qpush(L, lsrc | kItemExt, off);
        qpush(L, lit, ml);
        return true;
    }
    if (L.k + 1 > L.cap)
        return false;
    qpush(L, lsrc, off | (lit << 16) | ((ml ? ml - 3 : 0) << 24));
    return true;
}

// ---- frame header (LZ4F_decodeHeader order; as parse_frame) ------------------
__device__ __forceinline__ int32_t hdr_status(Scan &L)
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

// ---- fast path: one whole sequence (the common case) -------------------------
// Leaves anything it cannot finish (bytes not in the ring yet, longer
// extensions, errors) in its phase for a later sub-step or the slow step.
// Branch-free: both halves (token, offset) are evaluated on every lane and
// committed under predicates — with one wave per SIMD, the exec-mask chains
// of an if/return version cost more than the selects.
__device__ __forceinline__ void fast(Scan &L)
{
    const bool en = L.k == L.ks && L.ph <= P_OFF;   // queue empty: items go to q0..q2
    const bool in_tok = L.ph == P_TOKEN;
    // token: literal length with at most one extension byte
    const uint32_t ip = L.ip, rem = L.iend - ip;
    const uint32_t w = r4(L, ip);
    const uint32_t tok = w & 0xFF, e = (w >> 8) & 0xFF;
    const bool lext = (tok >> 4) == 15;
    const uint32_t lit = lext ? 15 + e : tok >> 4;
    const uint32_t p = ip + (lext ? 2 : 1);
    const bool tok_ok = ip < L.iend && L.cx0 + ip + (rem < 2 ? 1 : 2) <= L.avail &&
                        !(lext && (e == 255 || rem - 1 <= 15));
    // the block's last sequence: literals only, ending the block
    const bool last = L.op + lit > L.oend - kMfLimit || L.iend - p < lit + 2 + 1 + kLastLiterals;
    const bool last_ok = en && in_tok && tok_ok && last && L.iend - p == lit && L.op + lit <= L.oend &&
                         L.op + lit <= L.dlen;
    const bool t_ok = en && in_tok && tok_ok && !last && L.op + lit <= L.dlen;
    // offset + match length with at most one extension byte (after the token
    // just parsed, or the pending one)
    const uint32_t q = in_tok ? p + lit : ip;
    const uint32_t ctok = in_tok ? tok : L.tok;
    const uint32_t clsrc = in_tok ? p : L.lsrc;
    const uint32_t cnlit = in_tok ? lit : L.nlit;
    const uint32_t cop = in_tok ? L.op + lit : L.op;
    const uint32_t o4 = r4(L, q);
    const uint32_t off = o4 & 0xFFFF, e2 = (o4 >> 16) & 0xFF;
    const bool mext = (ctok & 15) == 15;
    const uint32_t p2 = q + (mext ? 3 : 2);
    const uint32_t ml = (mext ? 15 + e2 : ctok & 15) + kMinMatch;
    const bool o_ok = (in_tok ? t_ok : en) && L.cx0 + q + 3 <= L.avail &&
                      !(mext && (q + 2 >= L.iend || e2 == 255 || p2 >= L.iend - (kLastLiterals - 1))) &&
                      off != 0 && off <= cop - L.floor_ && cop + ml <= L.oend - kLastLiterals &&
                      cop + ml <= L.dlen;
    // one sequence to emit (a match, or the literals-only last one)
    const bool em = o_ok || last_ok;
    const uint32_t esrc = o_ok ? clsrc : p, elit = o_ok ? cnlit : lit;
    const uint32_t eoff = o_ok ? off : 0, eml = o_ok ? ml : 0;
    const bool big = elit > 255 || eml > 258;
    const uint32_t pad = big && (L.k & 63) == 63 ? 1 : 0;
    const uint32_t nk = big ? 2 + pad : 1;
    const bool fits = L.k + nk <= L.cap;
    const uint32_t xa = esrc | kItemExt;
    const uint32_t small_b = eoff | (elit << 16) | ((eml ? eml - 3 : 0) << 24);
    const bool put = em && fits;
    L.q0a = put ? (big ? (pad ? 0 : xa) : esrc) : L.q0a;
    L.q0b = put ? (big ? (pad ? 0 : eoff) : small_b) : L.q0b;
    L.q1a = put ? (pad ? xa : elit) : L.q1a;
    L.q1b = put ? (pad ? eoff : eml) : L.q1b;
    L.q2a = put ? elit : L.q2a;
    L.q2b = put ? eml : L.q2b;
    L.k = put ? L.k + nk : L.k;
    // state: offset done > token done (offset waits) > last sequence
    const uint32_t nip = o_ok ? p2 : (last_ok ? L.iend : (t_ok ? p + lit : L.ip));
    const uint32_t nop = o_ok ? cop + ml : (last_ok || t_ok ? L.op + lit : L.op);
    const uint32_t nph = o_ok ? P_TOKEN : (last_ok ? P_BHDR : (t_ok ? P_OFF : L.ph));
    L.tok = t_ok ? tok : L.tok;
    L.lsrc = t_ok ? p : L.lsrc;
    L.nlit = t_ok ? lit : L.nlit;
    L.ip = nip;
    L.op = nop;
    L.ph = nph;
    if (em && !fits)
        finish(L, ST_NOT_RUN);
}

// ---- the if/return form of fast() (A/B builds: scan version 1) ---------------
// Leaves anything it cannot finish (bytes not in the ring yet, longer
// extensions, errors) in its phase for a later sub-step or the slow step.
__device__ __forceinline__ void fast_br(Scan &L)
{
    if (L.k != L.ks)
        return;
    if (L.ph == P_TOKEN) {
        const uint32_t ip = L.ip;
        if (ip >= L.iend || !have(L, ip, L.iend - ip < 2 ? 1 : 2))
            return;
        const uint32_t w = r4(L, ip);
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
            // the block's last sequence: literals only, ending the block
            if (L.iend - p != lit || L.op + lit > L.oend || L.op + lit > L.dlen)
                return;
            if (!emit(L, p, lit, 0, 0)) {
                finish(L, ST_NOT_RUN);
                return;
            }
            L.op += lit;
            L.ip = L.iend;
            L.ph = P_BHDR;
            return;
        }
        if (L.op + lit > L.dlen)
            return;
        L.tok = tok;
        L.lsrc = p;
        L.nlit = lit;
        L.op += lit;
        L.ip = p + lit;
        L.ph = P_OFF;
    }
    if (L.ph == P_OFF) {
        const uint32_t q = L.ip;
        if (!have(L, q, 3))
            return;
        const uint32_t o4 = r4(L, q);
        const uint32_t off = o4 & 0xFFFF;
        uint32_t ml = L.tok & 15, p2 = q + 2;
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
        const uint32_t op = L.op;
        if (off == 0 || off > op - L.floor_ || op + ml > L.oend - kLastLiterals || op + ml > L.dlen)
            return;
        if (!emit(L, L.lsrc, L.nlit, off, ml)) {
            finish(L, ST_NOT_RUN);
            return;
        }
        L.op = op + ml;
        L.ip = p2;
        L.ph = P_TOKEN;
    }
}

// ---- slow step: byte at a time, every rule (parse_block / parse_frame) -------
// Returns with the lane waiting (phase unchanged) when bytes are not yet in
// the ring.
__device__ __forceinline__ void slow(Scan &L)
{
    if (L.k != L.ks)
        return;
    if (L.ph == P_TOKEN) {
        uint32_t p = L.ip;
        if (p >= L.iend) {
            fail_block(L);
            return;
        }
        if (!have(L, p, 1))
            return;
        const uint32_t tok = rb(L, p++);
        uint32_t lit = tok >> 4;
        if (lit == 15) {
            if (L.iend - p <= 15) {
                fail_block(L);
                return;
            }
            uint32_t s;
            do {
                if (p >= L.iend) {
                    fail_block(L);
                    return;
                }
                if (!have(L, p, 1))
                    return;   // re-parsed from the token next time
                s = rb(L, p++);
                lit += s;
            } while (s == 255);
        }
        if (L.op + lit > L.oend - kMfLimit || L.iend - p < lit + 2 + 1 + kLastLiterals) {
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
        L.tok = tok;
        L.lsrc = p;
        L.nlit = lit;
        L.op += lit;
        L.ip = p + lit;
        L.ph = P_OFF;
        return;
    }
    if (L.ph == P_OFF) {
        uint32_t p = L.ip;
        if (!have(L, p, 2))
            return;
        const uint32_t off = rb(L, p) | (rb(L, p + 1) << 8);
        p += 2;
        uint32_t ml = L.tok & 15;
        if (ml == 15) {
            uint32_t s;
            do {
                if (p >= L.iend) {
                    fail_block(L);
                    return;
                }
                if (!have(L, p, 1))
                    return;
                s = rb(L, p++);
                ml += s;
                if (p >= L.iend - (kLastLiterals - 1)) {
                    fail_block(L);
                    return;
                }
            } while (s == 255);
        }
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
        return;
    }
    if (L.ph == P_BHDR) {
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

// One sub-step with pipeline slot S: retire S into the ring, parse, store one
// queued item, issue S's next load.  Returns true when the stream jumped (the
// caller drops the other slots' loads).
template <bool SLOW, bool BR>
__device__ __forceinline__ bool sub(Scan &L, Fill &S)
{
    if (S.x != kOff) {
        // 16-aligned coordinates: the second half may wrap to ring index 0
        lds_w128(raddr(L, S.x), S.a);
        lds_w128(raddr(L, S.x + 16), S.b);
        L.avail = S.x + 32;
    }
    if (BR) {
        if (L.ph <= P_OFF)
            fast_br(L);
    } else {
        fast(L);
    }
    if (SLOW && L.ph != P_DONE)
        slow(L);
    // one item store
    const bool st = L.ks != L.k;
    __builtin_amdgcn_raw_buffer_store_b64(
        __builtin_bit_cast(__attribute__((ext_vector_type(2))) uint32_t,
                           (__attribute__((ext_vector_type(2))) uint32_t){L.q0a, L.q0b}),
        L.irs, st ? 8 * (L.ib + L.ks) : kOff, 0, 0);
    if (st) {
        L.ks++;
        L.q0a = L.q1a;
        L.q0b = L.q1b;
        L.q1a = L.q2a;
        L.q1b = L.q2b;
    }
    // the next byte needed was never requested (a long literal run was
    // skipped): restart the stream there, dropping loads in flight
    const uint32_t need = L.cx0 + L.ip;
    const bool jump = L.ph < P_END && need >= L.fill;
    if (jump) {
        L.fill = need & ~15u;
        L.avail = L.fill;
    }
    // ring fill: 32 bytes if that leaves every byte from ip on intact
    const bool fl = L.ph < P_END && L.fill < L.cx0 + L.clen && L.fill + 32 <= need + kRing - 16;
    const uint32_t fx = fl ? L.fill : kOff;
    S.x = fx;
    S.a = bload16(L.cin, fx);
    S.b = bload16(L.cin, fl ? fx + 16 : kOff);
    if (fl)
        L.fill += 32;
    return jump;
}

template <bool BR>
__global__ __launch_bounds__(64 * kSW) __attribute__((amdgpu_waves_per_eu(4, 4))) void lz4_scan_kernel(
    const FrameDesc *__restrict__ desc, uint32_t n, const uint8_t *__restrict__ comp,
    const uint64_t *__restrict__ rec_base, uint64_t capacity, uint64_t *__restrict__ items,
    uint32_t *__restrict__ nitems, int32_t *__restrict__ status, uint32_t *__restrict__ fail_at,
    uint32_t max_csize)
{
    __shared__ __attribute__((aligned(16))) uint8_t rings[kSW * 64 * kStride];
    const uint32_t f = blockIdx.x * (64 * kSW) + threadIdx.x;
    FrameDesc d = {0, 0, 0, 0};
    if (f < n)
        d = desc[f];
    // frames of max_csize bytes and more belong to lz4_chunk_kernel
    const bool act = f < n && d.c_size < max_csize;
    uint64_t rb0 = 0;
    uint32_t cap = 0;
    if (act) {
        rb0 = rec_base[f];
        cap = slots_of(d.c_size);
    }
    const uint64_t clo = uni64(wave_min64(act ? d.c_off : ~0ull));
    const uint64_t chi = uni64(wave_max64(act ? d.c_off + d.c_size : 0ull));
    const uint64_t ilo = uni64(wave_min64(act ? rb0 : ~0ull));
    const uint64_t ihi = uni64(wave_max64(act ? rb0 + cap : 0ull));
    const uint32_t steps = (uint32_t)__builtin_amdgcn_readfirstlane(
        (int)(uint32_t)(wave_max64(act ? (uint64_t)d.c_size : 0ull) * 2 + 64 * kD + 1024));
    if (!act)
        return;
    Scan L;
    const uintptr_t cbase = reinterpret_cast<uintptr_t>(comp + clo) & ~(uintptr_t)15;
    const uint64_t cspan = reinterpret_cast<uintptr_t>(comp + chi) - cbase;
    L.cin = __builtin_amdgcn_make_buffer_rsrc((void *)cbase, 0, (int)(uint32_t)((cspan + 3) & ~3ull), kRsrcDw3);
    const uint64_t ispan = (ihi - ilo) * 8;
    L.irs = __builtin_amdgcn_make_buffer_rsrc((void *)(items + ilo), 0, (int)(uint32_t)ispan, kRsrcDw3);
    L.ib = (uint32_t)(rb0 - ilo);
    L.cx0 = (uint32_t)(reinterpret_cast<uintptr_t>(comp + d.c_off) - cbase);
    L.clen = d.c_size;
    L.dlen = d.d_size;
    L.ring = (uint32_t)(uintptr_t)(rings) + threadIdx.x * kStride;
    L.fill = L.cx0 & ~15u;
    L.avail = L.fill;
    L.ph = P_BHDR;
    L.st = ST_NOT_RUN;
    L.ip = L.op = L.fail_op = 0;
    L.csz_flag = 0;
    L.csize = 0;
    L.indep = L.bsid = L.max_block = 0;
    L.iend = L.oend = L.floor_ = L.bop = 0;
    L.tok = L.lsrc = L.nlit = 0;
    L.k = L.ks = 0;
    L.cap = cap;
    L.q0a = L.q0b = L.q1a = L.q1b = L.q2a = L.q2b = 0;
    if (cspan >= 0x7FFFFF00ull || ispan >= 0x7FFFFF00ull || d.c_size > kItemPos || rb0 + cap > capacity) {
        finish(L, ST_NOT_RUN);
    } else {
        // frame header: the first 128 bytes, synchronously
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t fx = L.fill;
            const u32x4 a = bload16(L.cin, fx), b = bload16(L.cin, fx + 16);
            lds_w128(raddr(L, fx), a);
            lds_w128(raddr(L, fx + 16), b);
            L.fill += 32;
        }
        L.avail = L.fill;
        const int32_t hs = hdr_status(L);
        if (hs >= 0)
            finish(L, hs);
    }
    Fill sl[kD];
#pragma unroll
    for (int i = 0; i < (int)kD; i++)
        sl[i].x = kOff;
    uint32_t rounds = 0;
    for (;;) {
#pragma unroll
        for (int i = 0; i < (int)kD; i++) {
            const bool jumped = i == 0 ? sub<true, BR>(L, sl[i]) : sub<false, BR>(L, sl[i]);
            // a jump restarted the stream: drop the other slots' loads
            if (jumped) {
#pragma unroll
                for (int j = 0; j < (int)kD; j++)
                    if (j != i)
                        sl[j].x = kOff;
            }
        }
        const bool busy = L.ph != P_DONE || L.k != L.ks;
        if (!__any(busy))
            break;
        if (++rounds > steps) {
            if (busy)
                L.st = ST_NOT_RUN;
            break;
        }
    }
    status[f] = L.st;
    nitems[f] = L.ks;
    if (fail_at)
        fail_at[f] = L.fail_op;
}

}   // namespace

int launch_lz4_scan(const FrameDesc *d_desc, uint32_t nframes, const uint8_t *d_comp,
                    const uint64_t *rec_base, uint64_t capacity, uint64_t *items,
                    uint32_t *nitems, int32_t *d_status, uint32_t *d_fail_at, hipStream_t stream,
                    uint32_t max_csize)
{
    if (nframes == 0)
        return 0;
    const uint32_t per = 64 * kSW;
    hipLaunchKernelGGL(lz4_scan_kernel<false>, dim3((nframes + per - 1) / per), dim3(per), 0, stream,
                       d_desc, nframes, d_comp, rec_base, capacity, items, nitems, d_status, d_fail_at,
                       max_csize);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}   // namespace zsk
