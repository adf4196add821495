"""libzstd 1.4.9 (the reference's zstd dependency, /opt/conda) through ctypes,
for the tests only: compressing inputs with chosen parameters and decoding
them with the library itself as a second checker beside oracle/."""
from __future__ import annotations

import ctypes as C
import os

ZSTD_SO = "/opt/conda/lib/libzstd.so.1.4.9"

# ZSTD_cParameter values (zstd.h, 1.4.9)
P_LEVEL, P_WLOG, P_HLOG, P_CLOG, P_SLOG, P_MINMATCH, P_TLEN, P_STRAT = 100, 101, 102, 103, 104, 105, 106, 107
P_CSIZE, P_CHECKSUM = 200, 201


def load():
    if not os.path.exists(ZSTD_SO):
        return None
    z = C.CDLL(ZSTD_SO)
    z.ZSTD_createCCtx.restype = C.c_void_p
    z.ZSTD_CCtx_setParameter.argtypes = [C.c_void_p, C.c_int, C.c_int]
    z.ZSTD_CCtx_setParameter.restype = C.c_size_t
    z.ZSTD_compress2.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
    z.ZSTD_compress2.restype = C.c_size_t
    z.ZSTD_compressBound.argtypes = [C.c_size_t]
    z.ZSTD_compressBound.restype = C.c_size_t
    z.ZSTD_isError.argtypes = [C.c_size_t]
    z.ZSTD_isError.restype = C.c_uint
    z.ZSTD_getErrorCode.argtypes = [C.c_size_t]
    z.ZSTD_getErrorCode.restype = C.c_int
    z.ZSTD_freeCCtx.argtypes = [C.c_void_p]
    z.ZSTD_createDCtx.restype = C.c_void_p
    z.ZSTD_freeDCtx.argtypes = [C.c_void_p]
    z.ZSTD_decompressDCtx.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
    z.ZSTD_decompressDCtx.restype = C.c_size_t
    z.ZSTD_compressStream2.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    z.ZSTD_compressStream2.restype = C.c_size_t
    return z


def compress(z, data: bytes, params: dict) -> bytes:
    """one frame, ZSTD_compress2 with the given parameters"""
    cctx = z.ZSTD_createCCtx()
    try:
        for k, v in params.items():
            assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cctx, k, v)), (k, v)
        cap = z.ZSTD_compressBound(len(data))
        out = C.create_string_buffer(cap)
        n = z.ZSTD_compress2(cctx, out, cap, data, len(data))
        assert not z.ZSTD_isError(n)
        return out.raw[:n]
    finally:
        z.ZSTD_freeCCtx(cctx)


class _InBuf(C.Structure):
    _fields_ = [("src", C.c_void_p), ("size", C.c_size_t), ("pos", C.c_size_t)]


class _OutBuf(C.Structure):
    _fields_ = [("dst", C.c_void_p), ("size", C.c_size_t), ("pos", C.c_size_t)]


def compress_stream(z, data: bytes, chunk: int) -> bytes:
    """Streaming compression without a pledged size: no content size in the
    header, a window descriptor, one or more blocks flushed per chunk."""
    cctx = z.ZSTD_createCCtx()
    out = bytearray()
    try:
        dst = C.create_string_buffer(1 << 20)
        src = C.create_string_buffer(data, len(data))
        pos = 0
        while True:
            end = min(len(data), pos + chunk)
            ib = _InBuf(C.addressof(src) + pos, end - pos, 0)
            mode = 2 if end == len(data) else 1   # ZSTD_e_end / ZSTD_e_flush
            while True:
                ob = _OutBuf(C.addressof(dst), len(dst), 0)
                r = z.ZSTD_compressStream2(cctx, C.byref(ob), C.byref(ib), mode)
                assert not z.ZSTD_isError(r)
                out += dst.raw[: ob.pos]
                if r == 0 and ib.pos == ib.size:
                    break
            pos = end
            if end == len(data):
                break
        return bytes(out)
    finally:
        z.ZSTD_freeCCtx(cctx)


def decode(z, src: bytes, cap: int):
    """ZSTD_decompressDCtx -> (bytes, 0) or (b"", ZSTD_ErrorCode)"""
    d = z.ZSTD_createDCtx()
    try:
        out = C.create_string_buffer(max(cap, 1))
        r = z.ZSTD_decompressDCtx(d, out, cap, src, len(src))
        if z.ZSTD_isError(r):
            return b"", z.ZSTD_getErrorCode(r)
        return out.raw[:r], 0
    finally:
        z.ZSTD_freeDCtx(d)


# -- libzstd 1.4.9's Huffman entry points (exported by the shared library):
#    the oracle's X1 / X2 restatement is pinned against these directly
def load_huf(z):
    z.HUF_selectDecoder.argtypes = [C.c_size_t, C.c_size_t]
    z.HUF_selectDecoder.restype = C.c_uint32
    for n in ("HUF_compress2", "HUF_compress1X"):
        f = getattr(z, n)
        f.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_uint, C.c_uint]
        f.restype = C.c_size_t
    for n in ("HUF_decompress1X1_DCtx", "HUF_decompress1X2_DCtx", "HUF_decompress4X1_DCtx",
              "HUF_decompress4X2_DCtx", "HUF_decompress4X_hufOnly"):
        f = getattr(z, n)
        f.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        f.restype = C.c_size_t
    return z


def huf_compress(z, data: bytes, four: bool, max_log: int = 11) -> bytes | None:
    """HUF_compress2 (4 streams) / HUF_compress1X: tree description + streams,
    None when libzstd declines (incompressible or a single symbol)."""
    out = C.create_string_buffer(len(data) + 1024)
    f = z.HUF_compress2 if four else z.HUF_compress1X
    n = f(out, len(out), data, len(data), 255, max_log)
    if z.ZSTD_isError(n) or n <= 1:
        return None
    return out.raw[:n]


def huf_decompress(z, x2: bool, four: bool, src: bytes, cnt: int):
    """HUF_decompress{1,4}X{1,2}_DCtx on a fresh 12-bit DTable ->
    (ok, the cnt output bytes)."""
    dt = (C.c_uint32 * (1 + 4096))()
    dt[0] = 12 * 0x01000001
    out = C.create_string_buffer(cnt + 64)
    f = getattr(z, "HUF_decompress%dX%d_DCtx" % (4 if four else 1, 2 if x2 else 1))
    r = f(dt, out, cnt, src, len(src))
    return (not z.ZSTD_isError(r)), out.raw[:cnt]
