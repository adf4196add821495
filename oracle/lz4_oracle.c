/*
 * lz4_oracle.c — CPU restatement of the reference's random-access LZ4 decode.
 * TEST INFRASTRUCTURE ONLY (see oracle.h): scalar, byte-at-a-time, written for
 * obviousness, not speed.  The product never links or loads this file.
 *
 * Sources restated:
 *   seek table  /root/reference/src/seek_table.c:15-23 (constants),
 *               :62-110 (entry parse -> prefix sums), :112-176 (footer /
 *               skippable-header validation), :187-202 (frame lookup).
 *   LZ4 frame   liblz4 1.9.3 LZ4F_decompress (third-party, not in
 *               /root/reference; called at decompress.c:631,653,762): the LZ4
 *               Frame format spec v1.6.x + the 1.9.3 validation order.
 *   LZ4 block   liblz4 1.9.3 LZ4_decompress_safe(_usingDict): LZ4 Block
 *               format spec + the end-of-block parsing restrictions
 *               (MFLIMIT = 12, LASTLITERALS = 5) that decide success/error.
 */
#include <string.h>

#include "oracle.h"

#define LZ4F_MAGIC 0x184D2204U
#define LZ4F_SKIPPABLE_MASK 0xFFFFFFF0U
#define LZ4F_SKIPPABLE_START 0x184D2A50U
#define MINMATCH 4
#define MFLIMIT 12
#define LASTLITERALS 5

#define SEEK_FOOTER 9
#define SEEK_MAGIC 0x8F92EAB1U
#define SEEK_SKIPPABLE_MAGIC 0x184D2A5EU
#define SEEK_SKIPPABLE_HDR 8

static uint32_t rd32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}

static uint64_t rd64(const uint8_t *p)
{
    return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32);
}

/*
 * One LZ4 block: src[0..src_len) -> out[op0 ..), where out[0..op0) is the
 * frame's earlier output (usable as match history for linked blocks; for
 * independent blocks the history floor is op0).  Capacity of the block is
 * cap bytes (liblz4 decodes every block with dstCapacity = maxBlockSize).
 * Returns decoded size or -1.
 */
static long decode_block(const uint8_t *src, size_t src_len, uint8_t *out,
                         size_t op0, size_t cap, size_t hist_floor,
                         size_t out_limit)
{
    const uint8_t *ip = src;
    const uint8_t *const iend = src + src_len;
    size_t op = op0;
    const size_t oend = op0 + cap;   /* parsing restrictions use capacity */

    if (src_len == 0)
        return -1;

    for (;;) {
        if (ip >= iend)
            return -1;   /* block must end on a literals-only sequence */
        unsigned token = *ip++;
        size_t lit = token >> 4;
        if (lit == 15) {
            /* 1.9.3 read_variable_length(initial_check): ip < iend-15 */
            if (ip >= iend - 15 || iend - ip < 15)
                return -1;
            unsigned s;
            do {
                if (ip >= iend)
                    return -1;
                s = *ip++;
                lit += s;
            } while (s == 255);
        }
        /* literals; end-of-block restriction decides "last sequence" */
        if (op + lit > oend - MFLIMIT ||
            (size_t)(iend - ip) < lit + 2 + 1 + LASTLITERALS) {
            if ((size_t)(iend - ip) != lit || op + lit > oend)
                return -1;
            if (op + lit > out_limit)
                return -2;   /* would overflow the caller's frame slot */
            memmove(out + op, ip, lit);
            op += lit;
            return (long)(op - op0);
        }
        if (op + lit > out_limit)
            return -2;
        memcpy(out + op, ip, lit);
        ip += lit;
        op += lit;

        size_t off = (size_t)ip[0] | ((size_t)ip[1] << 8);
        ip += 2;
        size_t ml = token & 15;
        if (ml == 15) {
            unsigned s;
            do {
                if (ip >= iend)
                    return -1;
                s = *ip++;
                ml += s;
                /* 1.9.3 read_variable_length(loop_check): ip < iend-4 */
                if (ip >= iend - (LASTLITERALS - 1))
                    return -1;
            } while (s == 255);
        }
        ml += MINMATCH;
        /* offset 0 is declared invalid by the LZ4 block format spec */
        if (off == 0 || off > op - hist_floor)
            return -1;
        if (op + ml > oend - LASTLITERALS)
            return -1;
        if (op + ml > out_limit)
            return -2;
        for (size_t k = 0; k < ml; k++)   /* byte-wise: overlap-correct */
            out[op + k] = out[op + k - off];
        op += ml;
    }
}

int orc_lz4f_decode(const uint8_t *src, size_t src_len, uint8_t *dst,
                    size_t dst_cap, size_t *dst_len, size_t *src_used,
                    size_t *fail_at, int *block_fail, size_t *max_block_out)
{
    size_t ip = 0;
    size_t op = 0;
    *dst_len = 0;
    *src_used = 0;
    *fail_at = 0;
    *block_fail = 0;
    *max_block_out = 0;

    /* --- frame header (LZ4F_decodeHeader order) --- */
    if (src_len < 7)
        return ORC_ERROR_frameHeader_incomplete;
    uint32_t magic = rd32(src);
    if ((magic & LZ4F_SKIPPABLE_MASK) == LZ4F_SKIPPABLE_START)
        return ORC_ERROR_short_frame;   /* a skippable frame decodes nothing */
    if (magic != LZ4F_MAGIC)
        return ORC_ERROR_frameType_unknown;
    unsigned flg = src[4];
    unsigned version = (flg >> 6) & 3;
    unsigned block_cksum = (flg >> 4) & 1;
    unsigned block_indep = (flg >> 5) & 1;
    unsigned csize_flag = (flg >> 3) & 1;
    unsigned content_cksum = (flg >> 2) & 1;
    unsigned dictid_flag = flg & 1;
    if ((flg >> 1) & 1)
        return ORC_ERROR_reservedFlag_set;
    if (version != 1)
        return ORC_ERROR_headerVersion_wrong;
    size_t hdr = 7 + (csize_flag ? 8 : 0) + (dictid_flag ? 4 : 0);
    if (src_len < hdr)
        return ORC_ERROR_frameHeader_incomplete;
    unsigned bd = src[5];
    unsigned bsid = (bd >> 4) & 7;
    if ((bd >> 7) & 1)
        return ORC_ERROR_reservedFlag_set;
    if (bsid < 4)
        return ORC_ERROR_maxBlockSize_invalid;
    if (bd & 15)
        return ORC_ERROR_reservedFlag_set;
    if (((orc_xxh32(src + 4, hdr - 5, 0) >> 8) & 0xFF) != src[hdr - 1])
        return ORC_ERROR_headerChecksum_invalid;
    /* a dictID field is only recorded by LZ4F (no dictionary is supplied,
     * so a match reaching before the frame start fails as usual) */
    size_t max_block = (size_t)1 << (8 + 2 * bsid);   /* 64K/256K/1M/4M */
    *max_block_out = max_block;
    uint64_t content_size = csize_flag ? rd64(src + 6) : 0;
    ip = hdr;

    /* --- blocks --- */
    for (;;) {
        *fail_at = op;
        if (src_len - ip < 4)
            return ORC_ERROR_truncated;
        uint32_t bh = rd32(src + ip);
        ip += 4;
        if (bh == 0)
            break;   /* EndMark */
        size_t bsize = bh & 0x7FFFFFFFU;
        if (bsize > max_block)
            return ORC_ERROR_maxBlockSize_invalid;
        size_t need = bsize + (block_cksum ? 4 : 0);
        if (src_len - ip < need)
            return ORC_ERROR_truncated;
        if (bh & 0x80000000U) {
            if (op + bsize > dst_cap)
                return ORC_ERROR_dst_overflow;
            memcpy(dst + op, src + ip, bsize);
            if (block_cksum && orc_xxh32(src + ip, bsize, 0) !=
                                   rd32(src + ip + bsize))
                return ORC_ERROR_blockChecksum_invalid;
            op += bsize;
            ip += need;
            continue;
        }
        if (block_cksum &&
            orc_xxh32(src + ip, bsize, 0) != rd32(src + ip + bsize))
            return ORC_ERROR_blockChecksum_invalid;
        size_t floor = block_indep ? op : (op > 65536 ? op - 65536 : 0);
        long d = decode_block(src + ip, bsize, dst, op, max_block, floor,
                              dst_cap);
        if (d == -2)
            return ORC_ERROR_dst_overflow;
        if (d < 0) {
            *block_fail = 1;
            return (dst_cap - op) >= max_block ? ORC_ERROR_GENERIC
                                               : ORC_ERROR_decompressionFailed;
        }
        op += (size_t)d;
        ip += need;
    }

    /* --- suffix --- */
    *fail_at = op;
    if (csize_flag && content_size != op)
        return ORC_ERROR_frameSize_wrong;
    if (content_cksum) {
        if (src_len - ip < 4)
            return ORC_ERROR_truncated;
        if (orc_xxh32(dst, op, 0) != rd32(src + ip))
            return ORC_ERROR_contentChecksum_invalid;
        ip += 4;
    }
    *dst_len = op;
    *src_used = ip;
    return ORC_OK;
}

int64_t orc_seek_table_parse(const uint8_t *file, size_t fsize,
                             uint64_t *c_off, uint64_t *d_off,
                             uint32_t *checksum, int *checksum_flag)
{
    if (fsize < SEEK_FOOTER)
        return -1;
    const uint8_t *footer = file + fsize - SEEK_FOOTER;
    if (rd32(footer + 5) != SEEK_MAGIC)
        return -1;
    uint8_t desc = footer[4];
    if (desc & 0x7c)
        return -1;
    int ck = (desc & 0x80) != 0;
    uint32_t n = rd32(footer);
    uint64_t esize = 8 + (ck ? 4 : 0);
    uint64_t frame_size = SEEK_SKIPPABLE_HDR + (uint64_t)n * esize + SEEK_FOOTER;
    if (frame_size > fsize)
        return -1;
    const uint8_t *hdr = file + fsize - frame_size;
    if (rd32(hdr) != SEEK_SKIPPABLE_MAGIC)
        return -1;
    if (rd32(hdr + 4) != frame_size - SEEK_SKIPPABLE_HDR)
        return -1;
    if (checksum_flag)
        *checksum_flag = ck;
    const uint8_t *e = hdr + SEEK_SKIPPABLE_HDR;
    uint64_t c = 0, d = 0;
    for (uint32_t i = 0; i < n; i++, e += esize) {
        if (c_off)
            c_off[i] = c;
        if (d_off)
            d_off[i] = d;
        c += rd32(e);
        d += rd32(e + 4);
        if (ck && checksum)
            checksum[i] = rd32(e + 8);
    }
    if (c_off)
        c_off[n] = c;
    if (d_off)
        d_off[n] = d;
    return (int64_t)n;
}

int64_t orc_offset_to_frame(const uint64_t *d_off, uint64_t nframes,
                            uint64_t offset)
{
    if (offset >= d_off[nframes])
        return -1;
    uint64_t lo = 0, hi = nframes;
    while (lo + 1 < hi) {
        uint64_t mid = lo + (hi - lo) / 2;
        if (d_off[mid] <= offset)
            lo = mid;
        else
            hi = mid;
    }
    return (int64_t)lo;
}

/* SURVEY.md §8d synthetic: splitmix64 driven literal runs / back-copies. */
void orc_synth_gen(uint8_t *out, size_t n, uint64_t seed)
{
    uint64_t s = seed;
    size_t i = 0;
#define NEXT(z_)                                                   \
    do {                                                           \
        s += 0x9E3779B97F4A7C15ULL;                                \
        uint64_t z = s;                                            \
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;               \
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;               \
        (z_) = z ^ (z >> 31);                                      \
    } while (0)
    while (i < n) {
        uint64_t r;
        NEXT(r);
        if (i >= 65536 && r % 100 < 52) {
            size_t len = 4 + (size_t)((r >> 8) % 69);
            size_t off = 1 + (size_t)((r >> 24) % 8192);
            if (off > i)
                off = i;
            for (size_t k = 0; k < len && i < n; k++, i++)
                out[i] = out[i - off];
        } else {
            size_t len = 1 + (size_t)((r >> 8) % 48);
            for (size_t k = 0; k < len && i < n; k++, i++) {
                uint64_t q;
                NEXT(q);
                out[i] = (uint8_t)(0x20 + q % 64);
            }
        }
    }
#undef NEXT
}
