"""Pins oracle/zstd_oracle.c (the CPU restatement of libzstd 1.4.9's frame
decoder, the third-party code the reference calls at decompress.c:434-538)
against libzstd 1.4.9 itself on this host: frames compressed by libzstd with
many parameter sets must decode to the original bytes, and corrupted frames
must fail with the error code libzstd reports.  CPU only."""
import os

import numpy as np
import pytest

from oracle.oracle import Oracle

from zstd_util import (P_CHECKSUM, P_CSIZE, P_LEVEL, P_MINMATCH, P_STRAT, P_WLOG, compress,
                       compress_stream, decode, load)


@pytest.fixture(scope="module")
def zstd():
    z = load()
    if z is None:
        pytest.skip("libzstd 1.4.9 not present")
    return z


@pytest.fixture(scope="module")
def orc():
    return Oracle()


def _compress(z, data, params):
    return compress(z, data, params)


def libzstd_decode(z, src, cap):
    return decode(z, src, cap)


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
