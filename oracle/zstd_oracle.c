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

/* ---- Huffman literals (RFC 8878 §4.2; libzstd 1.4.9 huf_decompress.c) ------------
 * libzstd has two Huffman decoders.  X1 looks up one symbol per read in a
 * table of 2^tableLog cells; X2 looks up one or two symbols per read in a
 * table of 2^12 cells (a second symbol when both codes fit in 12 bits).  A
 * 4-stream literals section picks one by HUF_selectDecoder's timing model
 * (litSize, litCSize), a 1-stream section always uses X1, and a treeless
 * section reuses the previous table with the decoder that built it.  On valid
 * streams both give the same bytes; on corrupt ones they differ, so both are
 * restated here down to libzstd's 64-bit bit container (BIT_DStream_t):
 *   - the look-ahead shifts by (bitsConsumed & 63): past 64 consumed bits it
 *     reads the container's top bits again;
 *   - X2 writes two bytes per read, and at a stream's last output byte a
 *     two-symbol cell consumes both symbols' bits, clamped to the stream end
 *     (HUF_decodeLastSymbolX2) -- so some over- and under-long streams pass;
 *   - X2's 4-stream loop runs every stream until one of them nears its start
 *     or the 4th output nears its end: an earlier stream may run past its
 *     segment (an error), or end exactly on it after a one-symbol cell whose
 *     second byte (0) lands on the next segment's first byte.
 * Pinned against libzstd 1.4.9's own HUF_* entry points in
 * tests/test_zstd_oracle.py (random and corrupted streams, every table log). */
typedef struct {
    const uint8_t *start, *ptr, *limit;
    uint64_t c;          /* bitContainer */
    uint32_t consumed;   /* bitsConsumed */
} BitD;

enum { BD_UNFINISHED = 0, BD_END_OF_BUFFER = 1, BD_COMPLETED = 2, BD_OVERFLOW = 3 };

static uint64_t rd64(const uint8_t *p) { return (uint64_t)rd32(p) | ((uint64_t)rd32(p + 4) << 32); }

/* BIT_initDStream */
static int bitd_init(BitD *b, const uint8_t *p, size_t n)
{
    memset(b, 0, sizeof *b);
    if (n < 1)
        return -1;
    b->start = p;
    b->limit = p + 8;
    const uint8_t last = p[n - 1];
    if (n >= 8) {
        b->ptr = p + n - 8;
        b->c = rd64(b->ptr);
        b->consumed = last ? 8 - (uint32_t)highbit(last) : 0;
        if (!last)
            return -1;
    } else {
        b->ptr = p;
        b->c = 0;
        for (size_t i = 0; i < n; i++)
            b->c |= (uint64_t)p[i] << (8 * i);
        b->consumed = last ? 8 - (uint32_t)highbit(last) : 0;
        if (!last)
            return -1;
        b->consumed += (uint32_t)(8 - n) * 8;
    }
    return 0;
}

/* BIT_lookBitsFast (nb >= 1) */
static uint32_t bitd_look(const BitD *b, uint32_t nb)
{
    return (uint32_t)((b->c << (b->consumed & 63)) >> ((64 - nb) & 63));
}

/* BIT_reloadDStream */
static int bitd_reload(BitD *b)
{
    if (b->consumed > 64)
        return BD_OVERFLOW;
    if (b->ptr >= b->limit) {
        b->ptr -= b->consumed >> 3;
        b->consumed &= 7;
        b->c = rd64(b->ptr);
        return BD_UNFINISHED;
    }
    if (b->ptr == b->start)
        return b->consumed < 64 ? BD_END_OF_BUFFER : BD_COMPLETED;
    uint32_t nbytes = b->consumed >> 3;
    int res = BD_UNFINISHED;
    if ((size_t)(b->ptr - b->start) < nbytes) {
        nbytes = (uint32_t)(b->ptr - b->start);
        res = BD_END_OF_BUFFER;
    }
    b->ptr -= nbytes;
    b->consumed -= nbytes * 8;
    b->c = rd64(b->ptr);
    return res;
}

/* BIT_reloadDStreamFast */
static int bitd_reload_fast(BitD *b)
{
    if (b->ptr < b->limit)
        return BD_OVERFLOW;
    b->ptr -= b->consumed >> 3;
    b->consumed &= 7;
    b->c = rd64(b->ptr);
    return BD_UNFINISHED;
}

/* BIT_endOfDStream */
static int bitd_end(const BitD *b) { return b->ptr == b->start && b->consumed == 64; }

typedef struct {
    int valid;
    int x2;                 /* table type: 0 X1, 1 X2 */
    int log;                /* lookup bits: X1 the tree's table log, X2 12 */
    int tlog;               /* the tree's table log */
    uint8_t x1s[1 << 12], x1n[1 << 12];                  /* X1 cell: byte, nbBits */
    uint16_t x2q[1 << 12];                               /* X2 cell: sequence (LE16) */
    uint8_t x2n[1 << 12], x2l[1 << 12];                  /*          nbBits, length */
    uint8_t w[256];         /* weights of the last tree read */
    int nsym;
} Huf;

/* Tree description at p[0..n) -> weights (HUF_readStats); bytes used or -error */
static long huf_weights(const uint8_t *p, size_t n, uint8_t *w, int *nsym_out, int *log_out)
{
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
    /* weights -> table log; the last weight is implied */
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
    *nsym_out = nw;
    *log_out = log;
    return used;
}

/* HUF_readDTableX1: weight-1 symbols first, then weight 2, ... (symbol order within) */
static void huf_build_x1(Huf *h, const uint8_t *w, int nsym, int log)
{
    uint32_t start[16] = {0}, acc = 0, rank[16] = {0};
    for (int s = 0; s < nsym; s++)
        rank[w[s]]++;
    for (int k = 1; k <= log; k++) {
        start[k] = acc;
        acc += rank[k] << (k - 1);
    }
    for (int s = 0; s < nsym; s++) {
        if (!w[s])
            continue;
        const uint32_t len = (1u << w[s]) >> 1;
        for (uint32_t i = 0; i < len; i++) {
            h->x1s[start[w[s]] + i] = (uint8_t)s;
            h->x1n[start[w[s]] + i] = (uint8_t)(log + 1 - w[s]);
        }
        start[w[s]] += len;
    }
    h->x2 = 0;
    h->log = h->tlog = log;
    h->valid = 1;
}

/* HUF_readDTableX2 (HUF_fillDTableX2 / HUF_fillDTableX2Level2): a 12-bit
 * table; a first symbol whose code leaves room for the shortest code gets a
 * level-2 sub-table over the next bits: two-symbol cells for the symbols
 * whose codes fit, one-symbol cells (the first symbol alone) below them */
static void huf_set2(Huf *h, uint32_t u, uint32_t seq, uint32_t nb, uint32_t len)
{
    h->x2q[u] = (uint16_t)seq;
    h->x2n[u] = (uint8_t)nb;
    h->x2l[u] = (uint8_t)len;
}

static void huf_build_x2(Huf *h, const uint8_t *w, int nsym, int tlog)
{
    enum { TL = 12 };
    uint32_t stats[13] = {0};
    for (int s = 0; s < nsym; s++)
        stats[w[s]]++;
    int maxw = tlog;
    while (stats[maxw] == 0)
        maxw--;
    /* sorted symbols by weight (weight 0 dropped); rs0[k]: first of weight k */
    uint32_t rs0[14] = {0}, *rs = rs0 + 1, next = 0;
    for (int k = 1; k <= maxw; k++) {
        rs[k] = next;
        next += stats[k];
    }
    rs[0] = next;
    const uint32_t nsort = next;
    uint8_t ssym[256], swt[256];
    for (int s = 0; s < nsym; s++) {
        const uint32_t r = rs[w[s]]++;
        ssym[r] = (uint8_t)s;
        swt[r] = w[s];
    }
    rs[0] = 0;
    /* rank values: rv[c][k] = first cell of weight k, scaled down by c bits */
    uint32_t rv[TL][13];
    memset(rv, 0, sizeof rv);
    const int rescale = (TL - tlog) - 1;
    uint32_t nrv = 0;
    for (int k = 1; k <= maxw; k++) {
        rv[0][k] = nrv;
        nrv += stats[k] << (k + rescale);
    }
    const uint32_t minbits = (uint32_t)(tlog + 1 - maxw);
    for (uint32_t c = minbits; c < TL - minbits + 1; c++)
        for (int k = 1; k <= maxw; k++)
            rv[c][k] = rv[0][k] >> c;
    /* level 1 */
    const uint32_t base = (uint32_t)tlog + 1;
    const int scale = (int)base - TL;
    uint32_t r1[13];
    memcpy(r1, rv[0], sizeof r1);
    for (uint32_t s = 0; s < nsort; s++) {
        const uint32_t sym = ssym[s], wt = swt[s], nb = base - wt;
        const uint32_t st = r1[wt], len = 1u << (TL - nb);
        if (TL - nb >= minbits) {
            int minw = (int)nb + scale;
            if (minw < 1)
                minw = 1;
            const uint32_t srank = rs0[minw];
            /* level 2 over cells [st, st + len): sub-table of TL - nb bits */
            const uint32_t slog = TL - nb;
            uint32_t r2[13];
            memcpy(r2, rv[nb], sizeof r2);
            if (minw > 1)
                for (uint32_t i = 0; i < r2[minw]; i++)
                    huf_set2(h, st + i, sym, nb, 1);
            for (uint32_t q = srank; q < nsort; q++) {
                const uint32_t sym2 = ssym[q], wt2 = swt[q], nb2 = base - wt2;
                const uint32_t l2 = 1u << (slog - nb2), s2 = r2[wt2];
                for (uint32_t i = s2; i < s2 + l2; i++)
                    huf_set2(h, st + i, sym + (sym2 << 8), nb2 + nb, 2);
                r2[wt2] += l2;
            }
        } else {
            for (uint32_t u = st; u < st + len; u++)
                huf_set2(h, u, sym, nb, 1);
        }
        r1[wt] += len;
    }
    h->x2 = 1;
    h->log = TL;
    h->tlog = tlog;
    h->valid = 1;
}

/* read a tree into h as X1 or X2 cells; bytes used or -error */
static long huf_read(Huf *h, const uint8_t *p, size_t n, int x2)
{
    int nsym = 0, log = 0;
    const long used = huf_weights(p, n, h->w, &nsym, &log);
    if (used < 0)
        return used;
    h->nsym = nsym;
    if (x2)
        huf_build_x2(h, h->w, nsym, log);
    else
        huf_build_x1(h, h->w, nsym, log);
    return used;
}

/* HUF_selectDecoder: X2 when its modelled time (+1/8, for its bigger table)
 * beats X1's, per compression ratio bucket Q and 256-byte output units */
static const uint16_t HUF_ALGO[16][2][2] = {
    {{0, 0}, {1, 1}},           {{0, 0}, {1, 1}},           {{38, 130}, {1313, 74}},
    {{448, 128}, {1353, 74}},   {{556, 128}, {1353, 74}},   {{714, 128}, {1418, 74}},
    {{883, 128}, {1437, 74}},   {{897, 128}, {1515, 75}},   {{926, 128}, {1613, 75}},
    {{947, 128}, {1729, 77}},   {{1107, 128}, {2083, 81}},  {{1177, 128}, {2379, 87}},
    {{1242, 128}, {2415, 93}},  {{1349, 128}, {2644, 106}}, {{1455, 128}, {2422, 124}},
    {{722, 128}, {1891, 145}},
};

int orc_huf_select_x2(size_t dst, size_t csrc)
{
    const uint32_t q = csrc >= dst ? 15 : (uint32_t)(csrc * 16 / dst);
    const uint32_t d256 = (uint32_t)(dst >> 8);
    const uint32_t t0 = HUF_ALGO[q][0][0] + HUF_ALGO[q][0][1] * d256;
    uint32_t t1 = HUF_ALGO[q][1][0] + HUF_ALGO[q][1][1] * d256;
    t1 += t1 >> 3;
    return t1 < t0;
}

/* X1: one symbol per read */
static void x1_sym(const Huf *h, BitD *b, uint8_t *p)
{
    const uint32_t v = bitd_look(b, (uint32_t)h->log);
    *p = h->x1s[v];
    b->consumed += h->x1n[v];
}

/* HUF_decodeStreamX1 over [p, pe) (offsets into o) */
static void x1_stream(const Huf *h, BitD *b, uint8_t *o, long p, long pe)
{
    while ((bitd_reload(b) == BD_UNFINISHED) & (p < pe - 3)) {
        for (int k = 0; k < 4; k++)
            x1_sym(h, b, o + p++);
    }
    while (p < pe)
        x1_sym(h, b, o + p++);
}

/* X2: two bytes written, 1 or 2 of them kept */
static uint32_t x2_sym(const Huf *h, BitD *b, uint8_t *p)
{
    const uint32_t v = bitd_look(b, 12);
    p[0] = (uint8_t)h->x2q[v];
    p[1] = (uint8_t)(h->x2q[v] >> 8);
    b->consumed += h->x2n[v];
    return h->x2l[v];
}

/* HUF_decodeLastSymbolX2 */
static void x2_last(const Huf *h, BitD *b, uint8_t *p)
{
    const uint32_t v = bitd_look(b, 12);
    p[0] = (uint8_t)h->x2q[v];
    if (h->x2l[v] == 1) {
        b->consumed += h->x2n[v];
    } else if (b->consumed < 64) {
        b->consumed += h->x2n[v];
        if (b->consumed > 64)
            b->consumed = 64;
    }
}

/* HUF_decodeStreamX2 over [p, pe) */
static void x2_stream(const Huf *h, BitD *b, uint8_t *o, long p, long pe)
{
    while ((bitd_reload(b) == BD_UNFINISHED) & (p < pe - 7)) {
        for (int k = 0; k < 4; k++)
            p += x2_sym(h, b, o + p);
    }
    while ((bitd_reload(b) == BD_UNFINISHED) & (p <= pe - 2))
        p += x2_sym(h, b, o + p);
    while (p <= pe - 2)
        p += x2_sym(h, b, o + p);
    if (p < pe)
        x2_last(h, b, o + p);
}

/* HUF_decompress1X{1,2}_usingDTable: one stream p[0..n) -> out[0..cnt) */
static int huf_1x(const Huf *h, const uint8_t *p, size_t n, uint8_t *out, size_t cnt)
{
    BitD b;
    if (bitd_init(&b, p, n) != 0)
        return -ZE_CORRUPTION;
    if (h->x2)
        x2_stream(h, &b, out, 0, (long)cnt);
    else
        x1_stream(h, &b, out, 0, (long)cnt);
    return bitd_end(&b) ? 0 : -ZE_CORRUPTION;
}

/* HUF_decompress4X{1,2}_usingDTable: jump table + four streams p[0..n) ->
 * out[0..cnt) (out has 32 bytes of slack past cnt, as libzstd's literal
 * buffer) */
static int huf_4x(const Huf *h, const uint8_t *p, size_t n, uint8_t *out, size_t cnt)
{
    if (n < 10)
        return -ZE_CORRUPTION;
    const size_t l1 = rd16(p), l2 = rd16(p + 2), l3 = rd16(p + 4);
    const size_t l4 = n - (l1 + l2 + l3 + 6);
    if (l4 > n)   /* (wrapped) */
        return -ZE_CORRUPTION;
    const uint8_t *q[4] = {p + 6, p + 6 + l1, p + 6 + l1 + l2, p + 6 + l1 + l2 + l3};
    const size_t ln[4] = {l1, l2, l3, l4};
    const long seg = (long)((cnt + 3) / 4), oend = (long)cnt;
    if (3 * seg > oend)
        return -ZE_CORRUPTION;
    long op[4] = {0, seg, 2 * seg, 3 * seg};
    const long ostart[5] = {0, seg, 2 * seg, 3 * seg, oend};
    BitD b[4];
    for (int k = 0; k < 4; k++)
        if (bitd_init(&b[k], q[k], ln[k]) != 0)
            return -ZE_CORRUPTION;
    if (!h->x2) {
        /* 4 symbols per stream per round, in lock step */
        for (uint32_t go = 1; go & (op[3] < oend - 3);) {
            for (int r = 0; r < 4; r++)
                for (int k = 0; k < 4; k++)
                    x1_sym(h, &b[k], out + op[k]++);
            for (int k = 0; k < 4; k++)
                go &= bitd_reload_fast(&b[k]) == BD_UNFINISHED;
        }
    } else {
        /* 4 cells per stream per round; the streams are not in lock step */
        for (uint32_t go = 1; go & (op[3] < oend - 7);) {
            for (int r = 0; r < 4; r++)
                for (int k = 0; k < 4; k++)
                    op[k] += x2_sym(h, &b[k], out + op[k]);
            uint32_t g = 1;
            for (int k = 0; k < 4; k++)
                g &= bitd_reload_fast(&b[k]) == BD_UNFINISHED;
            go = g;
        }
    }
    for (int k = 0; k < 3; k++)
        if (op[k] > ostart[k + 1])
            return -ZE_CORRUPTION;
    for (int k = 0; k < 4; k++) {
        if (h->x2)
            x2_stream(h, &b[k], out, op[k], ostart[k + 1]);
        else
            x1_stream(h, &b[k], out, op[k], ostart[k + 1]);
    }
    for (int k = 0; k < 4; k++)
        if (!bitd_end(&b[k]))
            return -ZE_CORRUPTION;
    return 0;
}

/* test hook (tests/golden/make_zstd_x2.py): 1 = decode every Huffman
 * literals section with X1, as this restatement did before round 5 -- to find
 * the inputs on which X2's rules change libzstd's result */
static int g_x1_only;
void orc_zstd_x1_only(int on) { g_x1_only = on; }

/* test hooks: libzstd's exported HUF entry points restated (tree + streams) */
static long huf_entry(int x2, int four, const uint8_t *src, size_t n, uint8_t *dst, size_t cnt, Huf **keep)
{
    Huf *h = (Huf *)calloc(1, sizeof(Huf));
    if (!h)
        return -ZE_GENERIC;
    long rc;
    const long hs = huf_read(h, src, n, x2);
    if (hs < 0)
        rc = hs;
    else if ((size_t)hs >= n)
        rc = -ZE_SRC_WRONG;
    else
        rc = four ? huf_4x(h, src + hs, n - (size_t)hs, dst, cnt) : huf_1x(h, src + hs, n - (size_t)hs, dst, cnt);
    if (keep)
        *keep = h;
    else
        free(h);
    return rc ? rc : (long)cnt;
}

/* HUF_decompress{1,4}X{1,2}_DCtx (x2: 0/1; four: 0/1); dst needs cnt + 32 bytes */
long orc_huf_decompress(int x2, int four, const uint8_t *src, size_t n, uint8_t *dst, size_t cnt)
{
    return huf_entry(x2, four, src, n, dst, cnt, NULL);
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
        /* ZSTD_decodeLiteralsBlock: 1 stream -> HUF_decompress1X1_DCtx_wksp;
         * 4 streams -> HUF_decompress4X_hufOnly_wksp (X1 or X2 by
         * HUF_selectDecoder on litSize, litCSize) */
        int x2 = 0;
        if (!single) {
            if (size == 0 || csize == 0)
                return -ZE_CORRUPTION;
            x2 = g_x1_only ? 0 : orc_huf_select_x2(size, csize);
        }
        const long hs = huf_read(&D->huf, s, sn, x2);
        if (hs < 0 || (size_t)hs >= sn)
            return -ZE_CORRUPTION;
        s += hs;
        sn -= (size_t)hs;
    } else if (!D->huf.valid) {
        return -ZE_DICT_CORRUPTED;
    }
    /* (treeless: HUF_decompress{1,4}X_usingDTable, the table's own decoder) */
    if (single ? huf_1x(&D->huf, s, sn, D->lit, size) : huf_4x(&D->huf, s, sn, D->lit, size))
        return -ZE_CORRUPTION;
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
