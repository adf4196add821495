"""The LZ4 frame compressor restatement (oracle/lz4c_oracle.c, SURVEY §8f
row 4) pinned on CPU: byte-identical to liblz4 1.9.3's LZ4F_compressFrame
(the third-party compressor the reference writer calls, compress.c:750 /
:483 with the prefs of :203-207) and to the frames the compiled reference
writer produces, direct (compress_frame_lz4, no content size) and buffered
(end_frame_lz4, content size in the header)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest


class _FrameInfo(C.Structure):
    _fields_ = [("block_size_id", C.c_int), ("block_mode", C.c_int), ("content_checksum", C.c_int),
                ("frame_type", C.c_int), ("content_size", C.c_ulonglong), ("dict_id", C.c_uint),
                ("block_checksum", C.c_int)]


class _Prefs(C.Structure):
    _fields_ = [("frame_info", _FrameInfo), ("compression_level", C.c_int), ("auto_flush", C.c_uint),
                ("favor_dec_speed", C.c_uint), ("reserved", C.c_uint * 3)]


@pytest.fixture(scope="module")
def liblz4():
    L = C.CDLL("liblz4.so.1")
    L.LZ4_versionNumber.restype = C.c_int
    assert L.LZ4_versionNumber() == 10903, "pinned against liblz4 1.9.3"
    L.LZ4F_compressFrame.restype = C.c_size_t
    L.LZ4F_compressFrame.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.POINTER(_Prefs)]

    def frame(data: bytes, level: int, content_size: int) -> bytes:
        p = _Prefs()
        p.frame_info.block_size_id = 4            # LZ4F_max64KB, compress.c:207
        p.frame_info.content_size = content_size  # compress.c:741 / :472
        p.compression_level = level               # compress.c:203
        p.auto_flush = 1                          # compress.c:205
        out = C.create_string_buffer(len(data) + 4 * (len(data) // 65536) + 64)
        r = L.LZ4F_compressFrame(out, len(out), data, len(data), C.byref(p))
        assert r < (1 << 63)
        return out.raw[:r]
    return frame


def _cases(oracle, count: int):
    rng = np.random.default_rng(7)
    syn = oracle.synth_buffer(1 << 22).tobytes()
    out = []
    for n in (0, 1, 4, 5, 11, 12, 13, 14, 15, 16, 19, 20, 64, 270, 1000, 4096, 65534, 65535, 65536):
        out += [bytes(rng.integers(0, 256, n, dtype=np.uint8)), b"\0" * n,
                bytes(rng.integers(0, 3, n, dtype=np.uint8)), syn[:n], syn[(1 << 21):][:n]]
    for _ in range(count):
        n = int(rng.integers(0, 65537))
        o = int(rng.integers(0, len(syn) - n))
        out.append(syn[o: o + n])
        out.append(bytes(rng.integers(0, int(rng.integers(1, 257)), n, dtype=np.uint8)))
    # long literal runs / long matches around the 15 / 255 length-byte edges
    for k in (14, 15, 16, 269, 270, 271, 525):
        out.append(bytes(rng.integers(0, 256, k, dtype=np.uint8)) * 3 + b"x" * k)
    return out


@pytest.mark.parametrize("level", [0, 1, 2, -1, -7])
def test_restatement_matches_liblz4(oracle, liblz4, level):
    for i, b in enumerate(_cases(oracle, 60)):
        for cs in (0, 1):
            want = liblz4(b, level, cs)
            got = oracle.lz4f_compress_frame(b, level, bool(cs))
            assert got == want, (i, len(b), level, cs)


@pytest.mark.parametrize("level", [0, -2])
def test_linked_restatement_matches_liblz4(oracle, liblz4, level):
    """Frames above 64 KiB: linked 64 KiB blocks on one stream (the reference
    example's 1 MiB frames, test/example.c), with stored blocks in between
    (whose stream state still advances) and a short last block."""
    rng = np.random.default_rng(11)
    syn = oracle.synth_buffer(1 << 22).tobytes()
    noise = bytes(rng.integers(0, 256, 1 << 20, dtype=np.uint8))
    cases = [syn[:1 << 20], syn[12345:12345 + (1 << 20)], syn[:65537], syn[:65536 + 12],
             syn[:65536 + 13], syn[:3 * 65536 + 999], noise[:200000],
             noise[:65536] + syn[:65536] + noise[:70000] + syn[5:65536 * 2],
             syn[:100000] * 3, b"\0" * 300000, bytes(rng.integers(0, 4, 400000, dtype=np.uint8))]
    # a pattern repeating at 65535 / 65536 / 65537 bytes: distance-limit edge
    blk = bytes(rng.integers(0, 256, 65536, dtype=np.uint8))
    cases += [blk[:65535] * 3, blk * 3, blk + b"z" + blk + b"zz" + blk]
    for i, b in enumerate(cases):
        for cs in (0, 1):
            want = liblz4(b, level, cs)
            assert want[4] & 0x20 == 0, "linked"
            assert oracle.lz4f_compress_frame(b, level, bool(cs)) == want, (i, len(b), cs)


def test_incompressible_frame_is_stored(oracle, liblz4):
    b = bytes(np.random.default_rng(3).integers(0, 256, 65536, dtype=np.uint8))
    f = oracle.lz4f_compress_frame(b, 0, False)
    assert f == liblz4(b, 0, 0)
    assert f[:7].hex() == "04224d18604082"
    assert int.from_bytes(f[7:11], "little") == 0x80000000 | 65536
    assert f[11:-4] == b and f[-4:] == b"\0\0\0\0"


@pytest.mark.parametrize("min_frame,write,level", [(65536, 65536, 0), (4096, 4096, 0), (4096, 1000, 0),
                                                   (60000, 7000, 0), (20000, 20000, -3),
                                                   (1 << 20, 1 << 16, 0), (1 << 20, 1 << 20, 0),
                                                   (300000, 300000, -1)])
def test_restatement_matches_reference_writer(oracle, ref, min_frame, write, level):
    """Every frame of a file the compiled reference writer made: direct frames
    (write >= min_frame) without content size, buffered ones with it."""
    size = 1 << 20 if min_frame <= 65536 else 5 << 20
    data = oracle.synth_buffer(size).tobytes() + b"tail" * 333
    img = ref.compress(data, 1, min_frame, write, level=level)   # ZSEEK_LZ4
    st = oracle.seek_table(img)
    n, c_off, d_off = st["frames"], [int(x) for x in st["c_off"]], [int(x) for x in st["d_off"]]
    assert n > 3
    for f in range(n):
        frame = img[c_off[f]: c_off[f + 1]]
        chunk = data[d_off[f]: d_off[f + 1]]
        has_size = bool(frame[4] & 0x08)
        assert has_size == (write < min_frame or f == n - 1 and len(chunk) < min_frame), f
        assert oracle.lz4f_compress_frame(chunk, level, has_size) == frame, f


def test_writer_gpu_mode_refused_without_device(zs):
    """zsk_writer_set_gpu_compress reports false (and the writer stays on the
    host) where no HIP device is visible, for zstd writers and for HC levels."""
    from conftest import gpu_available
    data = bytes(zs.synth_buffer(300000))
    w = zs.Writer(zs.ZSEEK_LZ4, 65536)
    if not gpu_available():
        assert not w.set_gpu_compress(0)
    w.write(data)
    img = w.close()
    h = zs.Writer(zs.ZSEEK_LZ4, 65536)
    h.write(data)
    assert img == h.close()
    z = zs.Writer(zs.ZSEEK_ZSTD, 65536)
    assert not z.set_gpu_compress(0)
    z.close()
    hc = zs.Writer(zs.ZSEEK_LZ4, 65536, level=3)
    assert not hc.set_gpu_compress(0)
    hc.close()
