// lz4_dev.h — device helpers shared by the LZ4 kernels (lz4_split.hip,
// lz4_lane.hip): byte picking from 16-byte register vectors, range-checked
// aligned buffer loads, exact-length stores, wave reductions.
#ifndef ZSK_LZ4_DEV_H
#define ZSK_LZ4_DEV_H

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zsk {
namespace lz4d {

constexpr uint32_t kRsrcDw3 = 0x00020000u;   // gfx9-family raw buffer, 32-bit data
constexpr uint32_t kLz4Magic = 0x184D2204u;
constexpr uint32_t kMinMatch = 4;
constexpr uint32_t kMfLimit = 12;
constexpr uint32_t kLastLiterals = 5;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_u __attribute__((aligned(1)));
typedef uint64_t u64_u __attribute__((aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));

__device__ __forceinline__ uint32_t uni(uint32_t v)
{
    return __builtin_amdgcn_readfirstlane(v);
}

// byte i (0..15) of a 16-byte register vector
__device__ __forceinline__ uint32_t vbyte(const u32x4 &w, uint32_t i)
{
    uint32_t d = (i & 8) ? ((i & 4) ? w.w : w.z) : ((i & 4) ? w.y : w.x);
    return (d >> ((i & 3) * 8)) & 0xFF;
}

// 32 bits starting at byte i (0..12) of a 16-byte register vector
__device__ __forceinline__ uint32_t vword(const u32x4 &w, uint32_t i)
{
    uint32_t k = i >> 2;
    uint32_t lo = (k & 2) ? ((k & 1) ? w.w : w.z) : ((k & 1) ? w.y : w.x);
    uint32_t hi = (k & 2) ? w.w : ((k & 1) ? w.z : w.y);
    return __builtin_amdgcn_alignbyte(hi, lo, i & 3);
}

// 16 bytes at byte coordinate x of a buffer resource whose base is 4-byte
// aligned.  Loads are dword-aligned: the hardware range-checks every dword
// of a buffer load on its own (a dword straddling num_records reads as 0), so
// unaligned 16-byte loads would lose the last bytes of a range; aligned
// dwords with num_records rounded up to 4 never do.
__device__ __forceinline__ u32x4 load16u(__amdgpu_buffer_rsrc_t r, uint32_t x)
{
    const uint32_t a = x & ~3u, sh = x & 3;
    const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, a, 0, 0));
    const uint32_t e = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(r, a + 16, 0, 0);
    u32x4 o;
    o.x = __builtin_amdgcn_alignbyte(v.y, v.x, sh);
    o.y = __builtin_amdgcn_alignbyte(v.z, v.y, sh);
    o.z = __builtin_amdgcn_alignbyte(v.w, v.z, sh);
    o.w = __builtin_amdgcn_alignbyte(e, v.w, sh);
    return o;
}

// A byte range [p0, p0+len) of device memory as (aligned resource, bias):
// frame offset p lives at resource coordinate p + s0.
struct Span {
    __amdgpu_buffer_rsrc_t r;
    uint32_t s0;
};

__device__ __forceinline__ Span make_span(const uint8_t *p0, uint64_t len)
{
    const uintptr_t a = reinterpret_cast<uintptr_t>(p0);
    Span s;
    s.s0 = (uint32_t)(a & 3);
    s.r = __builtin_amdgcn_make_buffer_rsrc((void *)(a & ~(uintptr_t)3), 0,
                                            (int)(uint32_t)((s.s0 + len + 3) & ~3ull), kRsrcDw3);
    return s;
}

// store the first n (1..16) bytes of v at p, never touching p[n..]
__device__ __forceinline__ void store_exact(uint8_t *p, u32x4 v, uint32_t n)
{
    if (n >= 16) {
        *reinterpret_cast<u32x4_u *>(p) = v;
        return;
    }
    if (n & 8) {
        *reinterpret_cast<u64_u *>(p) = ((uint64_t)v.y << 32) | v.x;
        p += 8;
        v.x = v.z;
        v.y = v.w;
    }
    if (n & 4) {
        *reinterpret_cast<u32_u *>(p) = v.x;
        p += 4;
        v.x = v.y;
    }
    if (n & 2) {
        p[0] = (uint8_t)v.x;
        p[1] = (uint8_t)(v.x >> 8);
        p += 2;
        v.x >>= 16;
    }
    if (n & 1)
        p[0] = (uint8_t)v.x;
}

// ---- DPP lane exchange (no LDS, a few cycles each; pinned by
// scripts/microtests/dpp_scan.hip and dpp_shift.hip)

// lane i receives lane i+1's x (lane 63 receives `fill`)
__device__ __forceinline__ uint32_t dpp_next(uint32_t x, uint32_t fill)
{
    return __builtin_amdgcn_update_dpp(fill, x, 0x130, 0xf, 0xf, false);   // wave_shl:1
}

// lane i receives lane i-1's x (lane 0 receives `fill`)
__device__ __forceinline__ uint32_t dpp_prev(uint32_t x, uint32_t fill)
{
    return __builtin_amdgcn_update_dpp(fill, x, 0x138, 0xf, 0xf, false);   // wave_shr:1
}

// inclusive prefix sum over the wave: row shifts, then row broadcasts
__device__ __forceinline__ uint32_t wave_incl_add(uint32_t v)
{
    uint32_t x = v;
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);   // row_shr:1
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);   // row_shr:2
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);   // row_shr:4
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);   // row_shr:8
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);   // row_bcast:15
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);   // row_bcast:31
    return x;
}

// Order LDS writes of some lanes before LDS reads of others in the same
// wave.  The hardware already does (a wave's DS ops execute in order; no
// instruction is emitted), but the compiler treats lanes as threads: without
// a fence it may forward a lane's own earlier store to a load of a location
// another lane wrote meanwhile.
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
}

// inclusive prefix max over the wave (0 is the identity)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v)
{
    uint32_t x = v;
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false));   // row_shr:1
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false));   // row_shr:2
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false));   // row_shr:4
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false));   // row_shr:8
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false));   // row_bcast:15
    x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false));   // row_bcast:31
    return x;
}

__device__ __forceinline__ uint32_t lane_val(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}

__device__ __forceinline__ uint64_t uni64(uint64_t v)
{
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t wave_min64(uint64_t v)
{
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t o = __shfl_xor(v, m, 64);
        v = o < v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint64_t wave_max64(uint64_t v)
{
    for (int m = 32; m >= 1; m >>= 1) {
        uint64_t o = __shfl_xor(v, m, 64);
        v = o > v ? o : v;
    }
    return v;
}

}   // namespace lz4d
}   // namespace zsk

#endif
