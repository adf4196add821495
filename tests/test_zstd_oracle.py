"""Pins oracle/zstd_oracle.c (the CPU restatement of libzstd 1.4.9's frame
decoder, the third-party code the reference calls at decompress.c:434-538)
against libzstd 1.4.9 itself on this host: frames compressed by libzstd with
many parameter sets must decode to the original bytes, and corrupted frames
must fail with the error code libzstd reports.  CPU only."""
import ctypes as C
import os

import numpy as np
import pytest

from oracle.oracle import Oracle

ZSTD_SO = "/opt/conda/lib/libzstd.so.1.4.9"

# ZSTD_cParameter values (zstd.h, 1.4.9)
P_LEVEL, P_WLOG, P_HLOG, P_CLOG, P_SLOG, P_MINMATCH, P_TLEN, P_STRAT = 100, 101, 102, 103, 104, 105, 106, 107
P_CSIZE, P_CHECKSUM = 200, 201


@pytest.fixture(scope="module")
def zstd():
    if not os.path.exists(ZSTD_SO):
        pytest.skip("libzstd 1.4.9 not present")
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
    z.ZSTD_decompressDCtx.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
    z.ZSTD_decompressDCtx.restype = C.c_size_t
    z.ZSTD_CCtx_reset.argtypes = [C.c_void_p, C.c_int]
    z.ZSTD_compressStream2.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    z.ZSTD_compressStream2.restype = C.c_size_t
    return z


@pytest.fixture(scope="module")
def orc():
    return Oracle()


class _InBuf(C.Structure):
    _fields_ = [("src", C.c_void_p), ("size", C.c_size_t), ("pos", C.c_size_t)]


class _OutBuf(C.Structure):
    _fields_ = [("dst", C.c_void_p), ("size", C.c_size_t), ("pos", C.c_size_t)]


def compress_stream(z, data: bytes, chunk: int) -> bytes:
    """Streaming compression without a pledged size: no content size in the
    header, window descriptor present, blocks flushed per chunk."""
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


def libzstd_decode(z, src: bytes, cap: int):
    d = z.ZSTD_createDCtx()
    out = C.create_string_buffer(max(cap, 1))
    r = z.ZSTD_decompressDCtx(d, out, cap, src, len(src))
    if z.ZSTD_isError(r):
        return b"", z.ZSTD_getErrorCode(r)
    return out.raw[:r], 0


def datasets():
    rng = np.random.default_rng(5)
    from oracle.oracle import Oracle as _O
    synth = _O().synth(300_000, 3).tobytes()
    words = [b"seek", b"frame", b"table", b"zstd", b"lz4", b"gpu", b"wave", b"lane", b"the", b"of"]
    text = b" ".join(words[i] for i in rng.integers(0, len(words), 60_000))
    return {
        "synth": synth,
        "text": text,
        "random": rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes(),
        "zeros": bytes(150_000),
        "periodic": (bytes(range(7)) * 40_000),
        "small": b"abc",
        "one": b"x",
        "mixed": synth[:50_000] + bytes(70_000) + rng.integers(0, 256, 40_000, dtype=np.uint8).tobytes() + text[:80_000],
    }


DATA = datasets()
LEVELS = [-5, 1, 3, 9, 19]


@pytest.mark.parametrize("name", sorted(DATA))
@pytest.mark.parametrize("level", LEVELS)
def test_oracle_matches_libzstd(zstd, orc, name, level):
    data = DATA[name]
    comp = _compress(zstd, data, {P_LEVEL: level})
    out, err = orc.zstd_decode(comp, len(data))
    assert err == 0
    assert out == data


def _compress(z, data, params):
    cctx = z.ZSTD_createCCtx()
    try:
        for k, v in params.items():
            assert not z.ZSTD_isError(z.ZSTD_CCtx_setParameter(cctx, k, v))
        cap = z.ZSTD_compressBound(len(data))
        out = C.create_string_buffer(cap)
        n = z.ZSTD_compress2(cctx, out, cap, data, len(data))
        assert not z.ZSTD_isError(n)
        return out.raw[:n]
    finally:
        z.ZSTD_freeCCtx(cctx)


@pytest.mark.parametrize("name", ["synth", "text", "mixed"])
@pytest.mark.parametrize("chunk", [1000, 40_000])
def test_oracle_streamed_frames(zstd, orc, name, chunk):
    """unknown content size, window descriptor, many flushed blocks (treeless
    literals and repeat-mode tables across blocks)"""
    data = DATA[name]
    comp = compress_stream(zstd, data, chunk)
    out, err = orc.zstd_decode(comp, len(data))
    assert err == 0 and out == data


@pytest.mark.parametrize("name", ["synth", "text", "zeros", "random"])
def test_oracle_checksum_and_strategies(zstd, orc, name):
    data = DATA[name]
    for params in ({P_LEVEL: 3, P_CHECKSUM: 1}, {P_LEVEL: 3, P_STRAT: 1},
                   {P_LEVEL: 7, P_WLOG: 10}, {P_LEVEL: 12, P_MINMATCH: 3},
                   {P_LEVEL: 3, P_CSIZE: 0}):
        comp = _compress(zstd, data, params)
        out, err = orc.zstd_decode(comp, len(data))
        assert err == 0 and out == data, params


def test_oracle_concatenated_and_skippable(zstd, orc):
    a, b = DATA["synth"][:70_000], DATA["text"][:50_000]
    ca, cb = _compress(zstd, a, {P_LEVEL: 3}), _compress(zstd, b, {P_LEVEL: 1})
    skip = (0x184D2A5E).to_bytes(4, "little") + (5).to_bytes(4, "little") + b"12345"
    src = ca + skip + cb
    assert orc.zstd_decode(src, len(a) + len(b)) == libzstd_decode(zstd, src, len(a) + len(b))
    assert orc.zstd_decode(src, len(a) + len(b))[0] == a + b


def test_oracle_errors_match_libzstd(zstd, orc):
    """Single-byte corruptions and truncations of a few frames: the oracle
    must agree with libzstd on success/failure and on the error code."""
    rng = np.random.default_rng(9)
    checked = lenient = 0
    for name, level in (("synth", 3), ("text", 19), ("mixed", 1)):
        data = DATA[name][:60_000]
        comp = bytearray(_compress(zstd, data, {P_LEVEL: level}))
        cases = []
        for pos in rng.integers(0, len(comp), 120):
            c = bytearray(comp)
            c[pos] ^= int(rng.integers(1, 256))
            cases.append(bytes(c))
        for cut in (1, 3, 7, 20, len(comp) // 2, len(comp) - 1):
            cases.append(bytes(comp[:cut]))
        for c in cases:
            ref = libzstd_decode(zstd, c, len(data))
            got = orc.zstd_decode(c, len(data))
            if ref[1] == 0 and got[1] == 20:
                # documented divergence: libzstd's double-symbol
                # Huffman decoder clamps an over-read at a stream's last
                # symbol, so some corrupted literal streams decode to garbage
                # without an error; the restatement reports corruption there
                lenient += 1
                continue
            assert got[1] == ref[1], (name, level)
            if ref[1] == 0:
                assert got[0] == ref[0]
            checked += 1
    assert checked > 300
    assert lenient <= 3


# ---------------------------------------------------------------------------
# the restatement against the reference-generated golden zstd files
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["zstd_64k_direct", "zstd_64k_buffered"])
def test_oracle_decodes_golden_zstd_files(orc, name):
    import hashlib
    import json

    from conftest import GOLDEN, golden_file
    g = json.load(open(os.path.join(GOLDEN, "golden.json")))["files"][name]
    img = golden_file(name)
    st = orc.seek_table(img)
    out = bytearray()
    for i in range(len(st["c_off"]) - 1):
        c0, c1 = int(st["c_off"][i]), int(st["c_off"][i + 1])
        n = int(st["d_off"][i + 1] - st["d_off"][i])
        frame, err = orc.zstd_decode(img[c0:c1], n)
        assert err == 0 and len(frame) == n, i
        out += frame
    assert hashlib.sha256(bytes(out)).hexdigest() == g["payload_sha256"]
