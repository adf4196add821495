/*
 * xxhash_oracle.c — XXH32 / XXH64 restated from the published xxHash
 * specification (https://github.com/Cyan4973/xxHash/blob/dev/doc/xxhash_spec.md).
 * TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Used by the LZ4 frame format for the header checksum byte
 * ((XXH32(descriptor, 0) >> 8) & 0xFF), block checksums and the content
 * checksum, and by the seekable format for the optional per-frame checksum
 * (low 32 bits of XXH64, /root/reference/src/seek_table.c:95-97).
 */
#include <string.h>

#include "oracle.h"

static const uint32_t P32_1 = 0x9E3779B1U, P32_2 = 0x85EBCA77U,
                      P32_3 = 0xC2B2AE3DU, P32_4 = 0x27D4EB2FU,
                      P32_5 = 0x165667B1U;
static const uint64_t P64_1 = 0x9E3779B185EBCA87ULL,
                      P64_2 = 0xC2B2AE3D27D4EB4FULL,
                      P64_3 = 0x165667B19E3779F9ULL,
                      P64_4 = 0x85EBCA77C2B2AE63ULL,
                      P64_5 = 0x27D4EB2F165667C5ULL;

static uint32_t rl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
static uint64_t rl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

static uint32_t le32(const uint8_t *p)
{
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}

static uint64_t le64(const uint8_t *p)
{
    return (uint64_t)le32(p) | ((uint64_t)le32(p + 4) << 32);
}

static uint32_t round32(uint32_t acc, uint32_t lane)
{
    acc += lane * P32_2;
    acc = rl32(acc, 13);
    return acc * P32_1;
}

uint32_t orc_xxh32(const void *data, size_t len, uint32_t seed)
{
    const uint8_t *p = data;
    const uint8_t *end = p + len;
    uint32_t acc;

    if (len >= 16) {
        uint32_t a1 = seed + P32_1 + P32_2, a2 = seed + P32_2, a3 = seed,
                 a4 = seed - P32_1;
        while ((size_t)(end - p) >= 16) {
            a1 = round32(a1, le32(p));
            a2 = round32(a2, le32(p + 4));
            a3 = round32(a3, le32(p + 8));
            a4 = round32(a4, le32(p + 12));
            p += 16;
        }
        acc = rl32(a1, 1) + rl32(a2, 7) + rl32(a3, 12) + rl32(a4, 18);
    } else {
        acc = seed + P32_5;
    }
    acc += (uint32_t)len;
    while ((size_t)(end - p) >= 4) {
        acc += le32(p) * P32_3;
        acc = rl32(acc, 17) * P32_4;
        p += 4;
    }
    while (p < end) {
        acc += (uint32_t)(*p) * P32_5;
        acc = rl32(acc, 11) * P32_1;
        p++;
    }
    acc ^= acc >> 15;
    acc *= P32_2;
    acc ^= acc >> 13;
    acc *= P32_3;
    acc ^= acc >> 16;
    return acc;
}

static uint64_t round64(uint64_t acc, uint64_t lane)
{
    acc += lane * P64_2;
    acc = rl64(acc, 31);
    return acc * P64_1;
}

static uint64_t merge64(uint64_t acc, uint64_t a)
{
    acc ^= round64(0, a);
    return acc * P64_1 + P64_4;
}

uint64_t orc_xxh64(const void *data, size_t len, uint64_t seed)
{
    const uint8_t *p = data;
    const uint8_t *end = p + len;
    uint64_t acc;

    if (len >= 32) {
        uint64_t a1 = seed + P64_1 + P64_2, a2 = seed + P64_2, a3 = seed,
                 a4 = seed - P64_1;
        while ((size_t)(end - p) >= 32) {
            a1 = round64(a1, le64(p));
            a2 = round64(a2, le64(p + 8));
            a3 = round64(a3, le64(p + 16));
            a4 = round64(a4, le64(p + 24));
            p += 32;
        }
        acc = rl64(a1, 1) + rl64(a2, 7) + rl64(a3, 12) + rl64(a4, 18);
        acc = merge64(acc, a1);
        acc = merge64(acc, a2);
        acc = merge64(acc, a3);
        acc = merge64(acc, a4);
    } else {
        acc = seed + P64_5;
    }
    acc += (uint64_t)len;
    while ((size_t)(end - p) >= 8) {
        acc ^= round64(0, le64(p));
        acc = rl64(acc, 27) * P64_1 + P64_4;
        p += 8;
    }
    if ((size_t)(end - p) >= 4) {
        acc ^= (uint64_t)le32(p) * P64_1;
        acc = rl64(acc, 23) * P64_2 + P64_3;
        p += 4;
    }
    while (p < end) {
        acc ^= (uint64_t)(*p) * P64_5;
        acc = rl64(acc, 11) * P64_1;
        p++;
    }
    acc ^= acc >> 33;
    acc *= P64_2;
    acc ^= acc >> 29;
    acc *= P64_3;
    acc ^= acc >> 32;
    return acc;
}
