/*
 * zstd_oracle.c — CPU restatement of the zstd frame decode the reference
 * delegates to libzstd (ZSTD_decompressDCtx at
 * /root/reference/src/decompress.c:537, ZSTD_decompressStream at :434,448).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * libzstd is a third-party dependency absent from /root/reference (pinned:
 * libzstd 1.4.9, /opt/conda/lib/libzstd.so.1.4.9).  This file restates its
 * published format (RFC 8878: frames, blocks, literals with Huffman coding,
 * sequences with FSE coding, repeat offsets, XXH64 content checksum) with the
 * decisions libzstd 1.4.9 makes where the RFC leaves room:
 *   - ZSTD_decompressDCtx semantics: concatenated frames and skippable frames
 *     in the source are all decoded / skipped, leftover bytes are an error;
 *   - error codes are ZSTD_ErrorCode values (zstd_errors.h) for the checks
 *     libzstd performs, in the order it performs them;
 *   - a repeat offset that resolves to 0 is forced to 1 (libzstd does so
 *     instead of failing); sequence FSE states are updated after the last
 *     sequence too, and the sequence bitstream must be consumed at least to
 *     its end (over-consumption is accepted), as libzstd checks.
 * Pinned by tests/test_zstd_oracle.py against libzstd itself on this host
 * (many inputs, levels, block types and entropy modes) and against the
 * reference-generated golden files.
 */
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

enum {
    ZE_GENERIC = 1,
    ZE_PREFIX_UNKNOWN = 10,
    ZE_FRAMEPARAM_UNSUPPORTED = 14,
    ZE_WINDOW_TOO_LARGE = 16,
    ZE_CORRUPTION = 20,
    ZE_CHECKSUM = 22,
    ZE_DICT_CORRUPTED = 30,
    ZE_DICT_WRONG = 32,
    ZE_TABLELOG_TOO_LARGE = 44,
    ZE_MAXSYMBOL_TOO_SMALL = 48,
    ZE_DST_TOO_SMALL = 70,
    ZE_SRC_WRONG = 72,
};

#define ZBLOCK_MAX (128u << 10)
#define ZMAGIC 0xFD2FB528u

static uint32_t rd16(const uint8_t *p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
static uint32_t rd24(const uint8_t *p) { return rd16(p) | ((uint32_t)p[2] << 16); }
static uint32_t rd32(const uint8_t *p) { return rd24(p) | ((uint32_t)p[3] << 24); }
static int highbit(uint32_t v) { return 31 - __builtin_clz(v); }

/* bits [lo, lo + nb) of the little-endian bit string p[0..n), zero outside */
static uint64_t bits_at(const uint8_t *p, size_t n, int64_t lo, int nb)
{
    if (nb == 0)
        return 0;
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) {
        const int64_t b = lo + i;
        if (b >= 0 && b < (int64_t)(8 * n) && ((p[b >> 3] >> (b & 7)) & 1))
            v |= 1ull << i;
    }
    return v;
}

/* ---- backward bitstream (RFC 8878 §4.1: read from the end, MSB first) ---- */
typedef struct {
    const uint8_t *p;
    size_t n;
    int64_t pos;   /* bits not yet consumed; < 0 once read past the start */
} BitR;

static int bitr_init(BitR *b, const uint8_t *p, size_t n)
{
    if (n == 0 || p[n - 1] == 0)
        return -1;
    b->p = p;
    b->n = n;
    b->pos = 8 * (int64_t)(n - 1) + highbit(p[n - 1]);
    return 0;
}

static uint64_t bitr_read(BitR *b, int nb)
{
    b->pos -= nb;
    return bits_at(b->p, b->n, b->pos, nb);
}

static uint64_t bitr_peek(const BitR *b, int nb)
{
    return bits_at(b->p, b->n, b->pos - nb, nb);
}

/* ---- FSE ------------------------------------------------------------------- */
typedef struct {
    uint8_t sym, nb;
    uint16_t base;
} Cell;

/* Normalized-count header (RFC 8878 §4.1.1), forward bits from p[0..n).
 * Returns bytes used or -error. */
static long read_ncount(const uint8_t *p, size_t n, int16_t *norm, int max_sym, int max_log,
                        int *tlog, int *nsym)
{
    if (n == 0)
        return -ZE_SRC_WRONG;
    int64_t pos = 0;
    const int tl = (int)bits_at(p, n, pos, 4) + 5;
    pos += 4;
    if (tl > 15)
        return -ZE_TABLELOG_TOO_LARGE;
    if (tl > max_log)
        return -ZE_CORRUPTION;
    int remaining = (1 << tl) + 1, threshold = 1 << tl, nbits = tl + 1, sym = 0, prev0 = 0;
    for (int i = 0; i <= max_sym; i++)
        norm[i] = 0;
    while (remaining > 1 && sym <= max_sym) {
        if (prev0) {
            int n0 = sym;
            while (bits_at(p, n, pos, 16) == 0xFFFF) {
                n0 += 24;
                pos += 16;
            }
            while (bits_at(p, n, pos, 2) == 3) {
                n0 += 3;
                pos += 2;
            }
            n0 += (int)bits_at(p, n, pos, 2);
            pos += 2;
            if (n0 > max_sym)
                return -ZE_MAXSYMBOL_TOO_SMALL;
            while (sym < n0)
                norm[sym++] = 0;
        }
        const int mx = 2 * threshold - 1 - remaining;
        const int v = (int)bits_at(p, n, pos, nbits);
        int count;
        if ((v & (threshold - 1)) < mx) {
            count = v & (threshold - 1);
            pos += nbits - 1;
        } else {
            count = v & (2 * threshold - 1);
            if (count >= threshold)
                count -= mx;
            pos += nbits;
        }
        count--;
        remaining -= count < 0 ? -count : count;
        norm[sym++] = (int16_t)count;
        prev0 = count == 0;
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
    }
    if (remaining != 1)
        return -ZE_CORRUPTION;
    const long used = (long)((pos + 7) >> 3);
    if ((size_t)used > n)
        return -ZE_SRC_WRONG;
    *tlog = tl;
    *nsym = sym;
    return used;
}

/* decoding table from a normalized distribution (RFC 8878 §4.1.1) */
static int fse_build(Cell *t, const int16_t *norm, int nsym, int tl)
{
    const uint32_t size = 1u << tl, mask = size - 1;
    uint32_t high = size - 1;
    uint16_t next[256];
    for (int s = 0; s < nsym; s++) {
        if (norm[s] == -1) {
            t[high--].sym = (uint8_t)s;
            next[s] = 1;
        } else {
            next[s] = (uint16_t)norm[s];
        }
    }
    const uint32_t step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0;
    for (int s = 0; s < nsym; s++) {
        for (int i = 0; i < norm[s]; i++) {
            t[pos].sym = (uint8_t)s;
            do
                pos = (pos + step) & mask;
            while (pos > high);
        }
    }
    if (pos != 0)
        return -ZE_CORRUPTION;
    for (uint32_t u = 0; u < size; u++) {
        const uint32_t s = t[u].sym, ns = next[s]++;
        const int nb = tl - highbit(ns);
        t[u].nb = (uint8_t)nb;
        t[u].base = (uint16_t)((ns << nb) - size);
    }
    return 0;
}

/* ---- Huffman literals (RFC 8878 §4.2) ------------------------------------------ */
typedef struct {
    uint8_t sym[1 << 12];
    uint8_t nb[1 << 12];
    int log;
    int valid;
} Huf;

/* Huffman tree description at p[0..n); returns bytes used or -error */
static long huf_read(Huf *h, const uint8_t *p, size_t n)
{
    uint8_t w[256];
    int nw = 0;
    if (n == 0)
        return -ZE_SRC_WRONG;
    const uint32_t hb = p[0];
    long used;
    if (hb < 128) {
        /* FSE-compressed weights: 2 interleaved states, max accuracy 6 */
        if (1 + hb > n)
            return -ZE_SRC_WRONG;
        int16_t norm[256];
        int tl = 0, nsym = 0;
        const long hs = read_ncount(p + 1, hb, norm, 255, 6, &tl, &nsym);
        if (hs < 0)
            return hs;
        Cell t[64];
        int e = fse_build(t, norm, nsym, tl);
        if (e)
            return e;
        BitR b;
        if (bitr_init(&b, p + 1 + hs, hb - hs) != 0)
            return -ZE_GENERIC;
        uint32_t s1 = (uint32_t)bitr_read(&b, tl), s2 = (uint32_t)bitr_read(&b, tl);
        for (;;) {
            if (nw > 253)
                return -ZE_DST_TOO_SMALL;
            w[nw++] = t[s1].sym;
            s1 = t[s1].base + (uint32_t)bitr_read(&b, t[s1].nb);
            if (b.pos < 0) {
                w[nw++] = t[s2].sym;
                break;
            }
            if (nw > 253)
                return -ZE_DST_TOO_SMALL;
            w[nw++] = t[s2].sym;
            s2 = t[s2].base + (uint32_t)bitr_read(&b, t[s2].nb);
            if (b.pos < 0) {
                w[nw++] = t[s1].sym;
                break;
            }
        }
        used = 1 + hb;
    } else {
        nw = (int)hb - 127;
        const size_t bytes = (size_t)(nw + 1) / 2;
        if (1 + bytes > n)
            return -ZE_SRC_WRONG;
        for (int i = 0; i < nw; i++)
            w[i] = (i & 1) ? (p[1 + i / 2] & 15) : (p[1 + i / 2] >> 4);
        used = (long)(1 + bytes);
    }
    /* weights -> code lengths; the last weight is implied */
    uint32_t total = 0, rank[16] = {0};
    for (int i = 0; i < nw; i++) {
        if (w[i] >= 12)
            return -ZE_CORRUPTION;
        rank[w[i]]++;
        total += (1u << w[i]) >> 1;
    }
    if (total == 0)
        return -ZE_CORRUPTION;
    const int log = highbit(total) + 1;
    if (log > 12)
        return -ZE_CORRUPTION;
    const uint32_t rest = (1u << log) - total;
    if (rest != (1u << highbit(rest)))
        return -ZE_CORRUPTION;
    const int lastw = highbit(rest) + 1;
    w[nw++] = (uint8_t)lastw;
    rank[lastw]++;
    if (rank[1] < 2 || (rank[1] & 1))
        return -ZE_CORRUPTION;
    /* table: weight 1 symbols first, then weight 2, ... (symbol order within) */
    uint32_t start[16], acc = 0;
    for (int k = 1; k <= log; k++) {
        start[k] = acc;
        acc += rank[k] << (k - 1);
    }
    for (int s = 0; s < nw; s++) {
        if (!w[s])
            continue;
        const uint32_t len = (1u << w[s]) >> 1;
        for (uint32_t i = 0; i < len; i++) {
            h->sym[start[w[s]] + i] = (uint8_t)s;
            h->nb[start[w[s]] + i] = (uint8_t)(log + 1 - w[s]);
        }
        start[w[s]] += len;
    }
    h->log = log;
    h->valid = 1;
    return used;
}

/* one Huffman stream p[0..n) -> out[0..cnt) */
static int huf_stream(const Huf *h, const uint8_t *p, size_t n, uint8_t *out, size_t cnt)
{
    BitR b;
    if (bitr_init(&b, p, n) != 0)
        return -ZE_CORRUPTION;
    for (size_t i = 0; i < cnt; i++) {
        const uint32_t v = (uint32_t)bitr_peek(&b, h->log);
        out[i] = h->sym[v];
        b.pos -= h->nb[v];
    }
    if (b.pos != 0)
        return -ZE_CORRUPTION;
    return 0;
}

/* ---- sequences (RFC 8878 §3.1.1.3.2) ------------------------------------------- */
static const uint32_t LL_BASE[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10,   11,
                                     12, 13, 14, 15, 16, 18, 20, 22, 24, 28, 32,   40,
                                     48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t LL_BITS[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t ML_BASE[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13,  14,  15,   16,
                                     17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27,  28,  29,   30,
                                     31, 32, 33, 34, 35, 37, 39, 41, 43, 47, 51,  59,  67,   83,
                                     99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
static const uint8_t ML_BITS[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                    2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const int16_t LL_DEF[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                   2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t ML_DEF[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t OF_DEF[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                   1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};

typedef struct {
    Cell t[512];
    int log;
    int valid;
} Table;

/* one of the three sequence tables: mode 0 predefined, 1 RLE, 2 FSE, 3 repeat */
static long seq_table(Table *T, int mode, const uint8_t *p, size_t n, int max_sym, int max_log,
                      const int16_t *def, int def_n, int def_log)
{
    switch (mode) {
    case 0:
        T->log = def_log;
        T->valid = 1;
        return fse_build(T->t, def, def_n, def_log) ? -ZE_GENERIC : 0;
    case 1:
        if (n == 0)
            return -ZE_SRC_WRONG;
        if (p[0] > max_sym)
            return -ZE_CORRUPTION;
        T->t[0].sym = p[0];
        T->t[0].nb = 0;
        T->t[0].base = 0;
        T->log = 0;
        T->valid = 1;
        return 1;
    case 2: {
        int16_t norm[64];
        int tl = 0, nsym = 0;
        const long hs = read_ncount(p, n, norm, max_sym, max_log, &tl, &nsym);
        if (hs < 0)
            return -ZE_CORRUPTION;
        if (fse_build(T->t, norm, nsym, tl))
            return -ZE_CORRUPTION;
        T->log = tl;
        T->valid = 1;
        return hs;
    }
    default:
        if (!T->valid)
            return -ZE_CORRUPTION;
        return 0;
    }
}

typedef struct {
    Huf huf;
    Table ll, of, ml;
    uint32_t rep[3];
    uint8_t *lit;   /* literal buffer of the current block */
} Dec;

/* literals section; *litn = regenerated literals; returns bytes used or -error */
static long literals(Dec *D, const uint8_t *p, size_t n, size_t *litn)
{
    if (n < 3)
        return -ZE_CORRUPTION;
    const uint32_t type = p[0] & 3, sf = (p[0] >> 2) & 3;
    if (type <= 1) {
        size_t lh, size;
        switch (sf) {
        case 0:
        case 2: lh = 1; size = p[0] >> 3; break;
        case 1: lh = 2; size = rd16(p) >> 4; break;
        default: lh = 3; size = rd24(p) >> 4; break;
        }
        if (type == 0) {
            if (lh + size > n)
                return -ZE_CORRUPTION;
            memcpy(D->lit, p + lh, size);
            *litn = size;
            return (long)(lh + size);
        }
        if (lh + 1 > n || size > ZBLOCK_MAX)
            return -ZE_CORRUPTION;
        memset(D->lit, p[lh], size);
        *litn = size;
        return (long)(lh + 1);
    }
    if (n < 5)
        return -ZE_CORRUPTION;
    size_t lh, size, csize;
    int single = 0;
    const uint32_t lhc = rd32(p);
    switch (sf) {
    case 0:
    case 1:
        single = sf == 0;
        lh = 3;
        size = (lhc >> 4) & 0x3FF;
        csize = (lhc >> 14) & 0x3FF;
        break;
    case 2:
        lh = 4;
        size = (lhc >> 4) & 0x3FFF;
        csize = lhc >> 18;
        break;
    default:
        lh = 5;
        size = (lhc >> 4) & 0x3FFFF;
        csize = (lhc >> 22) + ((size_t)p[4] << 10);
        break;
    }
    if (size > ZBLOCK_MAX)
        return -ZE_CORRUPTION;
    if (csize + lh > n)
        return -ZE_CORRUPTION;
    const uint8_t *s = p + lh;
    size_t sn = csize;
    if (type == 2) {
        const long hs = huf_read(&D->huf, s, sn);
        if (hs < 0)
            return -ZE_CORRUPTION;
        s += hs;
        sn -= (size_t)hs;
    } else if (!D->huf.valid) {
        return -ZE_DICT_CORRUPTED;
    }
    if (single) {
        if (huf_stream(&D->huf, s, sn, D->lit, size))
            return -ZE_CORRUPTION;
    } else {
        if (sn < 10)
            return -ZE_CORRUPTION;
        const size_t l1 = rd16(s), l2 = rd16(s + 2), l3 = rd16(s + 4);
        if (l1 + l2 + l3 + 6 > sn)
            return -ZE_CORRUPTION;
        const size_t l4 = sn - 6 - l1 - l2 - l3;
        const size_t seg = (size + 3) / 4;
        if (3 * seg > size)
            return -ZE_CORRUPTION;
        const uint8_t *q = s + 6;
        if (huf_stream(&D->huf, q, l1, D->lit, seg) ||
            huf_stream(&D->huf, q + l1, l2, D->lit + seg, seg) ||
            huf_stream(&D->huf, q + l1 + l2, l3, D->lit + 2 * seg, seg) ||
            huf_stream(&D->huf, q + l1 + l2 + l3, l4, D->lit + 3 * seg, size - 3 * seg))
            return -ZE_CORRUPTION;
    }
    *litn = size;
    return (long)(lh + csize);
}

/* one compressed block p[0..n) -> out (frame output, produced so far: *op) */
static int block(Dec *D, const uint8_t *p, size_t n, uint8_t *out, size_t cap, size_t *op)
{
    if (n >= ZBLOCK_MAX)
        return -ZE_SRC_WRONG;
    size_t litn = 0;
    const long ls = literals(D, p, n, &litn);
    if (ls < 0)
        return (int)ls;
    const uint8_t *q = p + ls, *qe = p + n;
    if (q >= qe)
        return -ZE_SRC_WRONG;
    uint32_t nseq = q[0];
    if (nseq == 0) {
        if (qe - q != 1)
            return -ZE_SRC_WRONG;
        q++;
    } else if (nseq == 255) {
        if (q + 3 > qe)
            return -ZE_SRC_WRONG;
        nseq = rd16(q + 1) + 0x7F00;
        q += 3;
    } else if (nseq > 127) {
        if (q + 2 > qe)
            return -ZE_SRC_WRONG;
        nseq = ((nseq - 128) << 8) + q[1];
        q += 2;
    } else {
        q++;
    }
    size_t o = *op;
    const uint8_t *lp = D->lit, *le = D->lit + litn;
    if (nseq) {
        if (q + 1 > qe)
            return -ZE_SRC_WRONG;
        const uint32_t modes = *q++;
        long r = seq_table(&D->ll, modes >> 6, q, (size_t)(qe - q), 35, 9, LL_DEF, 36, 6);
        if (r < 0)
            return (int)r;
        q += r;
        r = seq_table(&D->of, (modes >> 4) & 3, q, (size_t)(qe - q), 31, 8, OF_DEF, 29, 5);
        if (r < 0)
            return (int)r;
        q += r;
        r = seq_table(&D->ml, (modes >> 2) & 3, q, (size_t)(qe - q), 52, 9, ML_DEF, 53, 6);
        if (r < 0)
            return (int)r;
        q += r;
        BitR b;
        if (bitr_init(&b, q, (size_t)(qe - q)) != 0)
            return -ZE_CORRUPTION;
        uint32_t sll = (uint32_t)bitr_read(&b, D->ll.log);
        uint32_t sof = (uint32_t)bitr_read(&b, D->of.log);
        uint32_t sml = (uint32_t)bitr_read(&b, D->ml.log);
        for (uint32_t i = 0; i < nseq; i++) {
            const uint32_t llc = D->ll.t[sll].sym, ofc = D->of.t[sof].sym, mlc = D->ml.t[sml].sym;
            if (llc > 35 || mlc > 52 || ofc > 31)
                return -ZE_CORRUPTION;
            uint64_t ofv = (1ull << ofc) + bitr_read(&b, ofc);
            const uint32_t ml = ML_BASE[mlc] + (uint32_t)bitr_read(&b, ML_BITS[mlc]);
            const uint32_t ll = LL_BASE[llc] + (uint32_t)bitr_read(&b, LL_BITS[llc]);
            uint64_t off;
            if (ofv > 3) {
                off = ofv - 3;
                D->rep[2] = D->rep[1];
                D->rep[1] = D->rep[0];
                D->rep[0] = (uint32_t)off;
            } else {
                const uint32_t idx = (uint32_t)ofv - 1 + (ll == 0);   /* 0..3 */
                if (idx == 0) {
                    off = D->rep[0];
                } else {
                    off = idx == 3 ? D->rep[0] - 1 : D->rep[idx];
                    if (off == 0)
                        off = 1;   /* libzstd forces a 0 offset to 1 */
                    if (idx != 1)
                        D->rep[2] = D->rep[1];
                    D->rep[1] = D->rep[0];
                    D->rep[0] = (uint32_t)off;
                }
            }
            sll = D->ll.t[sll].base + (uint32_t)bitr_read(&b, D->ll.t[sll].nb);
            sml = D->ml.t[sml].base + (uint32_t)bitr_read(&b, D->ml.t[sml].nb);
            sof = D->of.t[sof].base + (uint32_t)bitr_read(&b, D->of.t[sof].nb);
            /* execute */
            if ((uint64_t)o + ll + ml > cap)
                return -ZE_DST_TOO_SMALL;
            if ((size_t)(le - lp) < ll)
                return -ZE_CORRUPTION;
            memcpy(out + o, lp, ll);
            lp += ll;
            o += ll;
            if (off > o)
                return -ZE_CORRUPTION;
            for (uint32_t k = 0; k < ml; k++)
                out[o + k] = out[o + k - off];
            o += ml;
        }
        if (b.pos > 0)
            return -ZE_CORRUPTION;
    }
    const size_t last = (size_t)(le - lp);
    if (o + last > cap)
        return -ZE_DST_TOO_SMALL;
    memcpy(out + o, lp, last);
    *op = o + last;
    return 0;
}

/* one frame at src[0..n) (magic already checked); *used = its bytes */
static int frame(const uint8_t *src, size_t n, uint8_t *out, size_t cap, size_t *produced,
                 size_t *used, uint8_t *litbuf, size_t *bstart)
{
    *bstart = 0;   /* output offset of the failing block (frame-level checks: the end) */
    if (n < 6 + 3)
        return -ZE_SRC_WRONG;
    const uint32_t fhd = src[4];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, csum = (fhd >> 2) & 1,
                   did = fhd & 3;
    const size_t hsize = 5 + !single + (did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4) +
                         (fcs_flag == 0 ? single : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
    if (n < hsize + 3)
        return -ZE_SRC_WRONG;
    if (fhd & 0x08)
        return -ZE_FRAMEPARAM_UNSUPPORTED;
    size_t ip = 5;
    uint64_t window = 0;
    if (!single) {
        const uint32_t wd = src[ip++];
        const uint32_t wlog = 10 + (wd >> 3);
        if (wlog > 31)
            return -ZE_WINDOW_TOO_LARGE;
        window = (1ull << wlog) + ((1ull << wlog) / 8) * (wd & 7);
    }
    uint32_t dict = 0;
    for (uint32_t i = 0, nb = did == 3 ? 4 : did; i < nb; i++)
        dict |= (uint32_t)src[ip++] << (8 * i);
    uint64_t fcs = ~0ull;
    switch (fcs_flag) {
    case 0:
        if (single)
            fcs = src[ip++];
        break;
    case 1: fcs = rd16(src + ip) + 256; ip += 2; break;
    case 2: fcs = rd32(src + ip); ip += 4; break;
    default: fcs = (uint64_t)rd32(src + ip) | ((uint64_t)rd32(src + ip + 4) << 32); ip += 8; break;
    }
    if (single)
        window = fcs;
    (void)window;
    if (dict)
        return -ZE_DICT_WRONG;
    Dec *D = (Dec *)calloc(1, sizeof(Dec));
    if (!D)
        return -ZE_GENERIC;
    D->rep[0] = 1;
    D->rep[1] = 4;
    D->rep[2] = 8;
    D->lit = litbuf;
    size_t o = 0;
    int rc = 0;
    for (;;) {
        if (n - ip < 3) {
            rc = -ZE_SRC_WRONG;
            break;
        }
        *bstart = o;
        const uint32_t bh = rd24(src + ip);
        const uint32_t last = bh & 1, type = (bh >> 1) & 3, bsize = bh >> 3;
        const size_t csz = type == 1 ? 1 : bsize;
        if (type == 3) {
            rc = -ZE_CORRUPTION;
            break;
        }
        ip += 3;
        if (csz > n - ip) {
            rc = -ZE_SRC_WRONG;
            break;
        }
        if (type == 0) {
            if (bsize > cap - o) {
                rc = -ZE_DST_TOO_SMALL;
                break;
            }
            memcpy(out + o, src + ip, bsize);
            o += bsize;
        } else if (type == 1) {
            if (bsize > cap - o) {
                rc = -ZE_DST_TOO_SMALL;
                break;
            }
            memset(out + o, src[ip], bsize);
            o += bsize;
        } else {
            rc = block(D, src + ip, bsize, out, cap, &o);
            if (rc)
                break;
        }
        ip += csz;
        if (last)
            break;
    }
    if (!rc)
        *bstart = o;
    if (!rc && fcs != ~0ull && o != fcs)
        rc = -ZE_CORRUPTION;
    if (!rc && csum) {
        if (n - ip < 4) {
            rc = -ZE_CHECKSUM;
        } else {
            if ((uint32_t)orc_xxh64(out, o, 0) != rd32(src + ip))
                rc = -ZE_CHECKSUM;
            ip += 4;
        }
    }
    free(D);
    *produced = o;
    *used = ip;
    return rc;
}

/*
 * ZSTD_decompressDCtx(dst, cap, src, n) restated: every frame in src
 * (skippable frames skipped).  Returns the decoded size (>= 0) or -code
 * (ZSTD_ErrorCode); on a failure *fail_at (if given) receives the output
 * offset of the failing block's start (of the failing frame's end for its
 * content-size / checksum checks, of the frame's start for its header), the
 * bytes before it decoded in dst — the position libzstd's streaming decoder
 * (decompress.c:414-454) reaches when it meets the failure.
 */
long long orc_zstd_decode_at(const uint8_t *src, size_t n, uint8_t *dst, size_t cap, size_t *fail_at)
{
    uint8_t *lit = (uint8_t *)malloc(ZBLOCK_MAX + 64);
    if (!lit)
        return -ZE_GENERIC;
    size_t o = 0, fa = 0;
    long long rc = 0;
    int frames = 0;
    while (n >= 5) {
        fa = o;
        const uint32_t magic = rd32(src);
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (n < 8) {
                rc = -ZE_SRC_WRONG;
                break;
            }
            const uint64_t sk = 8 + (uint64_t)rd32(src + 4);
            if (sk > n) {
                rc = -ZE_SRC_WRONG;
                break;
            }
            src += sk;
            n -= sk;
            continue;
        }
        if (magic != ZMAGIC) {
            rc = frames ? -ZE_SRC_WRONG : -ZE_PREFIX_UNKNOWN;
            break;
        }
        frames++;
        size_t produced = 0, used = 0, bs = 0;
        const int e = frame(src, n, dst + o, cap - o, &produced, &used, lit, &bs);
        if (e) {
            fa = o + bs;
            rc = e;
            break;
        }
        o += produced;
        src += used;
        n -= used;
    }
    if (!rc && n) {
        fa = o;
        rc = -ZE_SRC_WRONG;
    }
    free(lit);
    if (rc && fail_at)
        *fail_at = fa;
    return rc ? rc : (long long)o;
}

long long orc_zstd_decode(const uint8_t *src, size_t n, uint8_t *dst, size_t cap)
{
    return orc_zstd_decode_at(src, n, dst, cap, NULL);
}
