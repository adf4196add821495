/*
 * lz4c_oracle.c — CPU restatement of the reference writer's LZ4 frame
 * compression.  TEST INFRASTRUCTURE ONLY: never linked
 * into or called by the product.
 *
 * The reference writer compresses each seekable frame with one call
 *     LZ4F_compressFrame(dst, bound, src, n, &prefs)
 * (compress.c:750 direct frames, :483 buffered frames), prefs =
 * { compressionLevel = level, autoFlush = 1, blockSizeID = LZ4F_max64KB }
 * (compress.c:203-207) and frameInfo.contentSize = the writer's frame_uc
 * counter before the frame (compress.c:741 / :472: 0 for a direct frame,
 * the buffered byte count for a flushed one).  The compressor is liblz4
 * 1.9.3, a third-party dependency absent from /root/reference (pinned: the
 * image's /opt/conda/lib/liblz4.so.1.9.3).  Restated here from its published
 * algorithm:
 *
 *   frame   magic 0x184D2204; FLG = version 01 | B.Indep (only a single-block
 *           frame, n <= 64 KiB: larger ones are linked) | C.Size when contentSize != 0
 *           (auto-corrected to n); BD = 0x40 (64 KiB); [8-byte content size];
 *           HC = (XXH32(FLG..) >> 8) & 0xFF; 64 KiB blocks (the last one
 *           short), none when n == 0; end mark 0.  No checksums.
 *   block   LZ4F_makeBlock: compress with capacity n - 1; a result of 0
 *           (did not fit) stores the block raw with bit 31 set.
 *   encoder LZ4_compress_fast_extState_fastReset on a freshly initialised
 *           state: 16-bit position table of 2^13 entries (hash =
 *           read32 * 2654435761 >> 19), limited output, acceleration
 *           (level < 0 ? 1 - level : 1); skip trigger 6, MINMATCH 4,
 *           MFLIMIT 12, LASTLITERALS 5, inputs < 13 bytes all literals.
 *   linked  n > 64 KiB: LZ4_compress_fast_continue on one stream for every
 *           block.  The state differs from the one-block encoder: a 32-bit
 *           position table of 2^12 entries indexed by the 5-byte hash of an
 *           8-byte read ((read64 << 24) * 889523592379 >> 52, the 64-bit
 *           build's byU32 hash), positions counted from the frame start, a
 *           candidate more than 65535 back is skipped without a compare,
 *           backward extension may run into earlier blocks (down to the
 *           frame start), match lengths stop 5 bytes before the block end.
 *           The stream state (table, offsets) advances even when a block
 *           does not fit and is stored raw.
 *
 * Pinned by tests/test_lz4_compress.py against liblz4 itself (our writer
 * calls LZ4F_compressFrame) and against the compiled reference writer.
 */
#include <stdint.h>
#include <string.h>

#include "oracle.h"

enum { MINMATCH = 4, MFLIMIT = 12, LASTLITERALS = 5, MIN_LENGTH = MFLIMIT + 1,
       ML_BITS = 4, ML_MASK = 15, RUN_MASK = 15, HASH_LOG = 13, SKIP_TRIGGER = 6 };

static uint32_t rd32(const uint8_t *p)
{
    uint32_t v;
    memcpy(&v, p, 4);
    return v;
}

static uint32_t hash4(uint32_t seq)
{
    return (seq * 2654435761u) >> (32 - HASH_LOG);
}

static void wr32le(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* Equal bytes of a[] and b[] before a reaches lim. */
static uint32_t count_eq(const uint8_t *a, const uint8_t *b, const uint8_t *lim)
{
    const uint8_t *s = a;
    while (a < lim && *a == *b) { a++; b++; }
    return (uint32_t)(a - s);
}

int orc_lz4_bound(int n)
{
    return n + n / 255 + 16;
}

long long orc_lz4_compress_block(const uint8_t *src, int n, uint8_t *dst, int cap, int accel)
{
    if (n < 0 || n >= 65536 + MFLIMIT - 1)
        return -1;                        /* byU16 table only (n < LZ4_64Klimit) */
    if (accel < 1)
        accel = 1;
    if (accel > 65537)
        accel = 65537;
    const int limited = cap < orc_lz4_bound(n);
    uint16_t table[1 << HASH_LOG];
    memset(table, 0, sizeof table);

    const uint8_t *ip = src, *anchor = src;
    const uint8_t *const iend = src + n;
    const uint8_t *const mflimit1 = iend - MFLIMIT + 1;
    const uint8_t *const matchlimit = iend - LASTLITERALS;
    uint8_t *op = dst;
    uint8_t *const olimit = dst + cap;
    const uint8_t *match;
    uint8_t *token;
    uint32_t fwd_h;

    if (n < MIN_LENGTH)
        goto last_literals;

    table[hash4(rd32(ip))] = 0;
    ip++;
    fwd_h = hash4(rd32(ip));

    for (;;) {
        /* search: step grows by one every 64 misses (times accel) */
        {
            const uint8_t *fwd = ip;
            int step = 1, nb = accel << SKIP_TRIGGER;
            for (;;) {
                const uint32_t h = fwd_h;
                const uint32_t cur = (uint32_t)(fwd - src);
                const uint32_t cand = table[h];
                ip = fwd;
                fwd += step;
                step = nb++ >> SKIP_TRIGGER;
                if (fwd > mflimit1)
                    goto last_literals;
                match = src + cand;
                fwd_h = hash4(rd32(fwd));
                table[h] = (uint16_t)cur;
                if (rd32(match) == rd32(ip))
                    break;
            }
        }
        /* extend backwards */
        while (ip > anchor && match > src && ip[-1] == match[-1]) {
            ip--;
            match--;
        }
        {
            const uint32_t lit = (uint32_t)(ip - anchor);
            token = op++;
            if (limited && op + lit + (2 + 1 + LASTLITERALS) + lit / 255 > olimit)
                return 0;
            if (lit >= RUN_MASK) {
                uint32_t len = lit - RUN_MASK;
                *token = RUN_MASK << ML_BITS;
                for (; len >= 255; len -= 255)
                    *op++ = 255;
                *op++ = (uint8_t)len;
            } else {
                *token = (uint8_t)(lit << ML_BITS);
            }
            memcpy(op, anchor, lit);
            op += lit;
        }
    next_match:
        {
            const uint32_t off = (uint32_t)(ip - match);
            op[0] = (uint8_t)off;
            op[1] = (uint8_t)(off >> 8);
            op += 2;
            uint32_t mc = count_eq(ip + MINMATCH, match + MINMATCH, matchlimit);
            ip += mc + MINMATCH;
            if (limited && op + (1 + LASTLITERALS) + (mc + 240) / 255 > olimit)
                return 0;
            if (mc >= ML_MASK) {
                *token += ML_MASK;
                mc -= ML_MASK;
                for (; mc >= 255; mc -= 255)
                    *op++ = 255;
                *op++ = (uint8_t)mc;
            } else {
                *token += (uint8_t)mc;
            }
        }
        anchor = ip;
        if (ip >= mflimit1)
            break;
        table[hash4(rd32(ip - 2))] = (uint16_t)(ip - 2 - src);
        /* immediate next match: no literals, no backward extension */
        {
            const uint32_t h = hash4(rd32(ip));
            const uint32_t cand = table[h];
            match = src + cand;
            table[h] = (uint16_t)(ip - src);
            if (rd32(match) == rd32(ip)) {
                token = op++;
                *token = 0;
                goto next_match;
            }
        }
        fwd_h = hash4(rd32(++ip));
    }

last_literals:
    {
        const size_t run = (size_t)(iend - anchor);
        if (limited && op + run + 1 + (run + 255 - RUN_MASK) / 255 > olimit)
            return 0;
        if (run >= RUN_MASK) {
            size_t acc = run - RUN_MASK;
            *op++ = RUN_MASK << ML_BITS;
            for (; acc >= 255; acc -= 255)
                *op++ = 255;
            *op++ = (uint8_t)acc;
        } else {
            *op++ = (uint8_t)(run << ML_BITS);
        }
        memcpy(op, anchor, run);
        op += run;
    }
    return (long long)(op - dst);
}


static uint32_t hash5(const uint8_t *p)
{
    uint64_t v;
    memcpy(&v, p, 8);
    return (uint32_t)(((v << 24) * 889523592379ull) >> (64 - 12));
}

/* One block [base + start, base + start + n) of a linked frame on the
 * stream's table (liblz4 1.9.3 LZ4_compress_generic_validated with byU32,
 * withPrefix64k or an empty extDict, noDictIssue, limitedOutput).  Returns
 * the compressed size, 0 if it does not fit cap. */
static long long linked_block(const uint8_t *base, uint32_t start, uint32_t n, uint32_t *table,
                              uint8_t *dst, int cap, int accel)
{
    const uint8_t *const src = base + start;
    const uint8_t *ip = src, *anchor = src;
    const uint8_t *const iend = src + n;
    const uint8_t *const mflimit1 = iend - MFLIMIT + 1;
    const uint8_t *const matchlimit = iend - LASTLITERALS;
    uint8_t *op = dst;
    uint8_t *const olimit = dst + cap;
    const uint8_t *match;
    uint8_t *token;
    uint32_t fwd_h;

    if (n < MIN_LENGTH)
        goto last_literals;

    table[hash5(ip)] = (uint32_t)(ip - base);
    ip++;
    fwd_h = hash5(ip);

    for (;;) {
        {
            const uint8_t *fwd = ip;
            int step = 1, nb = accel << SKIP_TRIGGER;
            for (;;) {
                const uint32_t h = fwd_h;
                const uint32_t cur = (uint32_t)(fwd - base);
                const uint32_t cand = table[h];
                ip = fwd;
                fwd += step;
                step = nb++ >> SKIP_TRIGGER;
                if (fwd > mflimit1)
                    goto last_literals;
                match = base + cand;
                fwd_h = hash5(fwd);
                table[h] = cur;
                if (cand + 65535 < cur)
                    continue;                 /* too far: no compare */
                if (rd32(match) == rd32(ip))
                    break;
            }
        }
        while (ip > anchor && match > base && ip[-1] == match[-1]) {
            ip--;
            match--;
        }
        {
            const uint32_t lit = (uint32_t)(ip - anchor);
            token = op++;
            if (op + lit + (2 + 1 + LASTLITERALS) + lit / 255 > olimit)
                return 0;
            if (lit >= RUN_MASK) {
                uint32_t len = lit - RUN_MASK;
                *token = RUN_MASK << ML_BITS;
                for (; len >= 255; len -= 255)
                    *op++ = 255;
                *op++ = (uint8_t)len;
            } else {
                *token = (uint8_t)(lit << ML_BITS);
            }
            memcpy(op, anchor, lit);
            op += lit;
        }
    next_match:
        {
            const uint32_t off = (uint32_t)(ip - match);
            op[0] = (uint8_t)off;
            op[1] = (uint8_t)(off >> 8);
            op += 2;
            uint32_t mc = count_eq(ip + MINMATCH, match + MINMATCH, matchlimit);
            ip += mc + MINMATCH;
            if (op + (1 + LASTLITERALS) + (mc + 240) / 255 > olimit)
                return 0;
            if (mc >= ML_MASK) {
                *token += ML_MASK;
                mc -= ML_MASK;
                for (; mc >= 255; mc -= 255)
                    *op++ = 255;
                *op++ = (uint8_t)mc;
            } else {
                *token += (uint8_t)mc;
            }
        }
        anchor = ip;
        if (ip >= mflimit1)
            break;
        table[hash5(ip - 2)] = (uint32_t)(ip - 2 - base);
        {
            const uint32_t h = hash5(ip);
            const uint32_t cur = (uint32_t)(ip - base);
            const uint32_t cand = table[h];
            match = base + cand;
            table[h] = cur;
            if (cand + 65535 >= cur && rd32(match) == rd32(ip)) {
                token = op++;
                *token = 0;
                goto next_match;
            }
        }
        fwd_h = hash5(++ip);
    }

last_literals:
    {
        const size_t run = (size_t)(iend - anchor);
        if (op + run + 1 + (run + 255 - RUN_MASK) / 255 > olimit)
            return 0;
        if (run >= RUN_MASK) {
            size_t acc = run - RUN_MASK;
            *op++ = RUN_MASK << ML_BITS;
            for (; acc >= 255; acc -= 255)
                *op++ = 255;
            *op++ = (uint8_t)acc;
        } else {
            *op++ = (uint8_t)(run << ML_BITS);
        }
        memcpy(op, anchor, run);
        op += run;
    }
    return (long long)(op - dst);
}

long long orc_lz4f_compress_frame(const uint8_t *src, size_t n, uint8_t *dst, size_t cap,
                                  int level, int content_size)
{
    if (level >= 3 || n > (size_t)1 << 30)
        return -1;                        /* HC levels not restated */
    const size_t nblk = (n + 65535) / 65536;
    const size_t need = 19 + nblk * 4 + n + 4;   /* header max + block words + blocks + end mark */
    if (cap < need)
        return -1;
    const int linked = n > 65536;
    const int accel = level < 0 ? 1 - level : 1;
    content_size = content_size && n > 0;  /* auto-corrected to n: 0 means absent */
    uint8_t *op = dst;
    wr32le(op, 0x184D2204u);
    op += 4;
    uint8_t *desc = op;
    *op++ = (uint8_t)(0x40 | (linked ? 0 : 0x20) | (content_size ? 0x08 : 0));
    *op++ = 0x40;
    if (content_size) {
        for (int i = 0; i < 8; i++)
            *op++ = (uint8_t)((uint64_t)n >> (8 * i));
    }
    *op = (uint8_t)(orc_xxh32(desc, (size_t)(op - desc), 0) >> 8);
    op++;
    static uint32_t table[1 << 12];       /* linked stream state (test oracle: one caller at a time) */
    if (linked)
        memset(table, 0, sizeof table);
    for (size_t b = 0; b < nblk; b++) {
        const size_t start = b * 65536;
        const size_t m = n - start < 65536 ? n - start : 65536;
        long long c = linked ? linked_block(src, (uint32_t)start, (uint32_t)m, table, op + 4,
                                            (int)m - 1, accel)
                             : orc_lz4_compress_block(src, (int)m, op + 4, (int)m - 1, accel);
        if (c < 0)
            return -1;
        if (c == 0) {
            wr32le(op, (uint32_t)m | 0x80000000u);
            memcpy(op + 4, src + start, m);
            c = (long long)m;
        } else {
            wr32le(op, (uint32_t)c);
        }
        op += 4 + c;
    }
    wr32le(op, 0);
    op += 4;
    return (long long)(op - dst);
}
