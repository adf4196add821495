"""Generate tests/golden/zstd_x2.{bin,json}: corrupted zstd frames on which
libzstd 1.4.9's double-symbol Huffman decoder (X2) decides the result.

Run in the build container (needs /opt/conda's libzstd 1.4.9 and, for the
seekable-file answers, oracle/_ref built by `make -C oracle ref`):

    python tests/golden/make_zstd_x2.py

For deterministic payloads it compresses one zstd frame with libzstd itself,
sweeps single-byte corruptions, and keeps those where decoding every Huffman
literals section with the single-symbol decoder (X1 -- what the oracle and
the GPU did before round 5) gives a different result from libzstd's own
ZSTD_decompressDCtx (X1 or X2 per HUF_selectDecoder, HUF_decodeLastSymbolX2's
clamp...).  For each kept frame it records libzstd's return code and output
hash, and the compiled REFERENCE reader's answers (oracle/_ref) on a seekable
file holding the frame between two intact ones: a caller's loop of
zseek_pread (test/example.c) with cache 0 and 1 -- bytes delivered, their
SHA-256, the last return value and its error string.  One payload is a
streamed multi-block frame, so treeless literal sections reuse an X2 table.

Only data is written (the corrupted frames and the expected answers).
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle.oracle import Oracle, RefZseek  # noqa: E402
from zstd_util import P_LEVEL, compress, compress_stream, decode, load  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MAX_CASES = 40


def payloads():
    """literal-heavy inputs (few matches), so blocks carry big Huffman
    literal sections -- the ones HUF_selectDecoder gives to X2"""
    rng = np.random.default_rng(2025)
    p = 1.0 / np.arange(1, 257) ** 1.2
    p /= p.sum()
    zipf = rng.choice(256, 40_000, p=p).astype(np.uint8).tobytes()
    q = np.exp(-np.arange(60) / 9.0)
    q /= q.sum()
    expo = rng.choice(60, 30_000, p=q).astype(np.uint8).tobytes()
    vocab = [bytes(rng.integers(97, 123, int(rng.integers(2, 9)), dtype=np.uint8)) for _ in range(3000)]
    text = b" ".join(vocab[i] for i in rng.integers(0, len(vocab), 6000))[:36_000]
    return [("zipf", zipf, 1), ("expo", expo, 3), ("text", text, 19), ("zipf", zipf[:20_000], 9),
            ("zipf-streamed", zipf, None)]


def seekable(frames: list[bytes], sizes: list[int]) -> bytes:
    """the frames + a seek table (zseek's skippable frame, no checksums)"""
    n = len(frames)
    table = bytearray((0x184D2A5E).to_bytes(4, "little") + (8 * n + 9).to_bytes(4, "little"))
    for f, s in zip(frames, sizes):
        table += len(f).to_bytes(4, "little") + s.to_bytes(4, "little")
    table += n.to_bytes(4, "little") + bytes([0]) + (0x8F92EAB1).to_bytes(4, "little")
    return b"".join(frames) + bytes(table)


def neighbours(z):
    """the intact frames around each corrupted one in its seekable file"""
    a = bytes(range(256)) * 24
    b = b"seekable zstd neighbour frame " * 150
    return [(compress(z, a, {P_LEVEL: 3}), len(a)), (compress(z, b, {P_LEVEL: 1}), len(b))]


def ref_answers(ref, img: bytes, total: int):
    """the reference reader under a caller's loop (test/example.c): zseek_pread
    from where the last call ended until it returns <= 0 -> bytes delivered,
    their SHA-256, the last return value and its error string"""
    out = {}
    for cache in (0, 1):
        r = ref.open(img, cache)
        got, pos = b"", 0
        while True:
            rv, b = r.pread(total - pos if total > pos else 1, pos)
            if rv <= 0:
                break
            got += b
            pos += rv
        out[f"cache{cache}"] = {"bytes": len(got), "sha": hashlib.sha256(got).hexdigest(), "last": int(rv),
                                "error": r.error if rv < 0 else ""}
        r.close()
    return out


def main():
    z = load()
    assert z is not None, "libzstd 1.4.9 missing"
    orc = Oracle()
    ref = RefZseek()
    assert ref.versions["zstd"] == 10409, ref.versions
    rng = np.random.default_rng(7)
    (fa, sa), (fb, sb) = neighbours(z)
    blob = bytearray()
    cases = []
    for name, data, level in payloads():
        # (level None: streamed in 13,000-byte flushes -- blocks after the
        # first may send treeless literals)
        comp = compress(z, data, {P_LEVEL: level}) if level is not None else compress_stream(z, data, 13_000)
        found = 0
        for pos in rng.permutation(len(comp))[:3000]:
            if len(cases) >= MAX_CASES or found >= MAX_CASES // 5:
                break
            c = bytearray(comp)
            x = int(rng.integers(1, 256))
            c[int(pos)] ^= x
            c = bytes(c)
            lib = decode(z, c, len(data))
            exact = orc.zstd_decode(c, len(data))
            assert exact[1] == lib[1] and (lib[1] or exact[0] == lib[0]), (name, int(pos))
            orc.lib.orc_zstd_x1_only(1)
            x1 = orc.zstd_decode(c, len(data))
            orc.lib.orc_zstd_x1_only(0)
            if x1[1] == lib[1] and (lib[1] or x1[0] == lib[0]):
                continue
            img = seekable([fa, c, fb], [sa, len(data), sb])
            total = sa + len(data) + sb
            cases.append({
                "payload": name, "level": level, "pos": int(pos), "xor": x, "off": len(blob), "len": len(c),
                "dsize": len(data),
                "libzstd": {"code": int(lib[1]), "sha": hashlib.sha256(lib[0]).hexdigest() if not lib[1] else ""},
                "x1_code": int(x1[1]),
                "reference": ref_answers(ref, img, total),
            })
            blob += c
            found += 1
    with open(os.path.join(OUT, "zstd_x2.bin"), "wb") as f:
        f.write(bytes(blob))
    meta = {"neighbours": {"a": {"len": len(fa), "dsize": sa}, "b": {"len": len(fb), "dsize": sb}},
            "neighbour_frames_hex": [fa.hex(), fb.hex()], "cases": cases}
    with open(os.path.join(OUT, "zstd_x2.json"), "w") as f:
        json.dump(meta, f, indent=1)
    print(f"{len(cases)} cases, {len(blob)} bytes;",
          sum(1 for c in cases if c["libzstd"]["code"] == 0), "decode without error in libzstd")


if __name__ == "__main__":
    main()
