"""GPU parity for zstd: zsk_zstd_decode_frames and the
reader's zstd preads vs the reference's own outputs (golden files made by
oracle/_ref), libzstd 1.4.9 itself, and the oracle (oracle/zstd_oracle.c) on
corrupt frames.  Bit-exact outputs; per-frame statuses equal the libzstd
error code the oracle restates."""
from __future__ import annotations

import numpy as np
import pytest

from conftest import golden_file, sha
from zstd_util import (P_CHECKSUM, P_CSIZE, P_LEVEL, P_MINMATCH, P_STRAT, P_WLOG, compress,
                       compress_stream, load)

pytestmark = pytest.mark.gpu

ZSTD_FILES = ["zstd_64k_direct", "zstd_64k_buffered"]
ZSK_STATUS_ZSTD = 0x4000000


@pytest.fixture(scope="module")
def zstd():
    z = load()
    if z is None:
        pytest.skip("libzstd 1.4.9 not present")
    return z


def device_decode(zs, gpu, frames, sizes, pad=0):
    """decode a list of compressed frames (bytes) with decoded sizes via the
    device API -> (list of decoded bytes, status array)"""
    import torch
    n = len(frames)
    desc = np.zeros(n, zs.FRAME_DESC_DTYPE)
    c = d = 0
    for i, (f, s) in enumerate(zip(frames, sizes)):
        desc[i]["c_off"], desc[i]["d_off"] = c, d
        desc[i]["c_size"], desc[i]["d_size"] = len(f), s
        c += len(f) + pad
        d += s
    blob = bytearray()
    for f in frames:
        blob += f + bytes(pad)
    comp = torch.zeros(len(blob) + 64, dtype=torch.uint8, device=gpu)
    if blob:
        comp[: len(blob)].copy_(torch.frombuffer(bytearray(blob), dtype=torch.uint8))
    out = torch.zeros(max(d, 1), dtype=torch.uint8, device=gpu)
    status = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    dt = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    zs.zstd_decode_frames(dt, comp, out, status)
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    res, p = [], 0
    for s in sizes:
        res.append(o[p: p + s])
        p += s
    return res, status.cpu().numpy()


def datasets(oracle):
    rng = np.random.default_rng(7)
    synth = oracle.synth(400_000, 5).tobytes()
    words = [b"seek", b"frame", b"table", b"zstd", b"lz4", b"gpu", b"wave", b"lane", b"the", b"of"]
    text = b" ".join(words[i] for i in rng.integers(0, len(words), 50_000))
    return {
        "synth": synth,
        "text": text,
        "random": rng.integers(0, 256, 150_000, dtype=np.uint8).tobytes(),
        "zeros": bytes(140_000),
        "periodic": bytes(range(13)) * 9000,
        "mixed": synth[:60_000] + bytes(50_000) + rng.integers(0, 256, 30_000, dtype=np.uint8).tobytes() + text[:60_000],
        "tiny": b"zseek",
    }


@pytest.mark.parametrize("level", [-5, 1, 3, 9, 19])
def test_device_zstd_levels(gpu, zs, oracle, zstd, level):
    """every dataset, one frame each, compressed by libzstd at several levels"""
    data = datasets(oracle)
    names = sorted(data)
    frames = [compress(zstd, data[k], {P_LEVEL: level}) for k in names]
    out, st = device_decode(zs, gpu, frames, [len(data[k]) for k in names])
    for k, o, s in zip(names, out, st):
        assert s == 0, (k, hex(int(s)))
        assert o == data[k], k


def test_device_zstd_frame_variants(gpu, zs, oracle, zstd):
    """unknown content size + multi-block streamed frames (treeless literals,
    repeat-mode tables, window descriptors), checksums, other strategies and
    parameters, concatenated and skippable frames in one entry"""
    data = datasets(oracle)
    frames, sizes = [], []
    for k in ("synth", "text", "mixed"):
        for chunk in (1000, 30_000):
            frames.append(compress_stream(zstd, data[k], chunk))
            sizes.append(len(data[k]))
        for params in ({P_LEVEL: 3, P_CHECKSUM: 1}, {P_LEVEL: 3, P_STRAT: 1},
                       {P_LEVEL: 7, P_WLOG: 10}, {P_LEVEL: 12, P_MINMATCH: 3},
                       {P_LEVEL: 3, P_CSIZE: 0}):
            frames.append(compress(zstd, data[k], params))
            sizes.append(len(data[k]))
    a, b = data["synth"][:70_000], data["text"][:40_000]
    skip = (0x184D2A5E).to_bytes(4, "little") + (3).to_bytes(4, "little") + b"abc"
    frames.append(compress(zstd, a, {P_LEVEL: 3}) + skip + compress(zstd, b, {P_LEVEL: 1}))
    sizes.append(len(a) + len(b))
    want = [data[k] for k in ("synth", "text", "mixed") for _ in range(7)] + [a + b]
    out, st = device_decode(zs, gpu, frames, sizes, pad=3)
    for i, (o, s) in enumerate(zip(out, st)):
        assert s == 0, (i, hex(int(s)))
        assert o == want[i], i


@pytest.mark.parametrize("frame", [4096, 65536, 1 << 20, 100_000])
def test_device_zstd_synthetic(gpu, zs, frame):
    """the §8d synthetic as the reference writer compresses it (level 3,
    strategy 1), several frame sizes, through the device API"""
    data = zs.synth_buffer(24 << 20)
    img = zs.zstd_seekable(data, frame)
    c_off, d_off = zs.seek_table_of(img)
    n = len(c_off) - 1
    frames = [img[c_off[i]: c_off[i + 1]].tobytes() for i in range(n)]
    sizes = [int(d_off[i + 1] - d_off[i]) for i in range(n)]
    out, st = device_decode(zs, gpu, frames, sizes)
    assert int((st != 0).sum()) == 0
    assert b"".join(out) == data.tobytes()


@pytest.mark.parametrize("nframes", [16384, 20001])
def test_device_zstd_three_chunk_pipeline(gpu, zs, nframes):
    """batches of >= 16,384 frames decode in three pipelined chunks (ragged
    at 20,001): every frame OK, bytes == the source"""
    data = zs.synth_buffer(nframes * 4096)
    img = zs.zstd_seekable(data, 4096)
    c_off, d_off = zs.seek_table_of(img)
    n = len(c_off) - 1
    assert n == nframes
    frames = [img[c_off[i]: c_off[i + 1]].tobytes() for i in range(n)]
    sizes = [int(d_off[i + 1] - d_off[i]) for i in range(n)]
    out, st = device_decode(zs, gpu, frames, sizes)
    assert int((st != 0).sum()) == 0
    assert b"".join(out) == data.tobytes()


@pytest.mark.parametrize("batch", [0, 40])
def test_device_zstd_corrupt_status(gpu, zs, oracle, zstd, batch):
    """single-byte corruptions and truncations: every frame's status is the
    libzstd error code the oracle gives, intact frames decode bit-exact --
    all 198 frames in one batch (a lane per frame), and in batches of 40 (the
    one-frame route: a wave per frame's sequences, a workgroup per frame's
    execute)"""
    rng = np.random.default_rng(3)
    data = datasets(oracle)
    frames, sizes = [], []
    for k, level in (("synth", 3), ("text", 19), ("mixed", 1)):
        src = data[k][:60_000]
        comp = compress(zstd, src, {P_LEVEL: level})
        for pos in rng.integers(0, len(comp), 60):
            c = bytearray(comp)
            c[pos] ^= int(rng.integers(1, 256))
            frames.append(bytes(c))
            sizes.append(len(src))
        for cut in (1, 5, 9, 20, len(comp) // 2, len(comp) - 1):
            frames.append(comp[:cut])
            sizes.append(len(src))
    if batch:
        out, st = [], []
        for b in range(0, len(frames), batch):
            o, t = device_decode(zs, gpu, frames[b: b + batch], sizes[b: b + batch])
            out += o
            st += list(t)
    else:
        out, st = device_decode(zs, gpu, frames, sizes)
    for i, (f, n) in enumerate(zip(frames, sizes)):
        want, err = oracle.zstd_decode(f, n)
        if err:
            assert st[i] == ZSK_STATUS_ZSTD | err, (i, hex(int(st[i])), err)
        else:
            ok = len(want) == n
            assert st[i] == (0 if ok else 101), (i, hex(int(st[i])))
            if ok:
                assert out[i] == want, i


# ---------------------------------------------------------------------------
# the reader (zseek_pread) on the reference-generated golden files
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", ZSTD_FILES)
@pytest.mark.parametrize("cache", [0, 1])
def test_zstd_full_range_pread(gpu, zs, golden, payloads, name, cache):
    data = payloads[name]
    with zs.Reader(golden_file(name), cache) as r:
        got = r.pread(len(data) + 17, 0)
        assert len(got) == len(data)
        assert sha(got) == golden["files"][name]["payload_sha256"]


@pytest.mark.parametrize("name", ZSTD_FILES)
def test_zstd_reference_queries(gpu, zs, golden, payloads, name):
    """every query the reference answered: our (possibly longer, multi-frame)
    answer starts with exactly its bytes; the cache ends in its state"""
    entry = golden["files"][name]
    data = payloads[name]
    readers = {c: zs.Reader(golden_file(name), c) for c in (0, 1)}
    try:
        for q in entry["reads"]:
            r = readers[q["cache"]]
            off, cnt, ref_ret = q["offset"], q["count"], q["ret"]
            out = np.empty(max(cnt, 1), np.uint8)
            ret = r.pread_raw(out.ctypes.data, cnt, off)
            assert ret == max(0, min(cnt, len(data) - off)), q
            assert ret >= ref_ret
            assert sha(out[:ref_ret]) == q["sha256"], q
        assert readers[1].stats()["cached_frames"] == entry["stats_cache1"]["cached_frames"]
    finally:
        for r in readers.values():
            r.close()


def test_zstd_writer_roundtrip(gpu, zs, payloads):
    data = payloads["zstd_64k_direct"]
    w = zs.Writer(zs.ZSEEK_ZSTD, 65536, nb_workers=1)
    for s in range(0, len(data), 65536):
        w.write(data[s: s + 65536])
    img = w.close()
    with zs.Reader(img, 0) as r:
        assert r.read_all(len(data), 0) == data


def test_cache_lru_matches_reference(gpu, zs, ref):
    """Frame-cache semantics (ref src/cache.c): capacity in frames, LRU
    eviction, find promotes — cached_frames after single-frame zstd reads
    equals the reference library's."""
    img = golden_file("zstd_64k_direct")
    seq = [0, 65536, 0, 131072, 200000, 0, 70000, 300000, 5, 400000]
    for cap in (1, 2, 3):
        ours = zs.Reader(img, cap)
        theirs = ref.open(img, cap)
        for off in seq:
            a = ours.pread(100, off)
            rb, b = theirs.pread(100, off)
            assert a == b
            assert ours.stats()["cached_frames"] == theirs.stats()[1]["cached_frames"]
        ours.close()
        theirs.close()


@pytest.mark.parametrize("cache", [0, 1])
def test_zstd_corrupt_frame_error_text(gpu, zs, oracle, cache):
    """a corrupt frame: the bytes before it, then -1 with libzstd's wording
    (the corruption is one libzstd detects, found with the oracle)"""
    data = zs.synth_buffer(5 * 65536)
    img = bytearray(zs.zstd_seekable(data, 65536).tobytes())
    c_off, d_off = zs.seek_table_of(np.frombuffer(bytes(img), np.uint8))
    f0, f1 = int(c_off[2]), int(c_off[3])
    for pos in range(f0 + 20, f1):
        frame = bytearray(img[f0:f1])
        frame[pos - f0] ^= 0xFF
        if oracle.zstd_decode(bytes(frame), 65536)[1] == 20:   # corruption_detected
            img[pos] ^= 0xFF
            break
    else:
        pytest.fail("no detectable corruption found")
    with zs.Reader(np.frombuffer(bytes(img), np.uint8), cache) as r:
        got = r.pread(5 * 65536, 0)
        assert got == data[: 2 * 65536].tobytes()
        with pytest.raises(zs.ZseekError) as e:
            r.pread(100, 2 * 65536)
        msg = str(e.value)
        assert msg == ("decompress frame: " if cache else "decompress user data: ") + \
            "Corrupted block detected"
        # a request starting inside the corrupt frame: libzstd's streaming
        # decoder meets the damage while discarding the prefix
        if not cache:
            with pytest.raises(zs.ZseekError) as e:
                r.pread(100, 2 * 65536 + 1000)
            assert str(e.value) == "decompress discard data: Corrupted block detected"


@pytest.mark.parametrize("case", ["zstd1m_block4_first", "zstd1m_block4_type"])
def test_zstd_partial_reads_golden(gpu, zs, golden, case):
    """A corrupt 5th block of a 1 MiB frame (golden, made by the compiled
    reference): without a cache a request ending before the bad block gets its
    bytes, one reaching it gets libzstd's user/discard-data error; with a
    cache every read of the frame fails."""
    rec = golden["corrupt"][case]
    base = bytearray(golden_file(rec["base"]))
    for at, v in rec["mutations"]:
        base[at] = v
    for q in rec["results"]:
        with zs.Reader(bytes(base), q["cache"]) as r:
            out = np.empty(max(q["count"], 1), np.uint8)
            ret = r.pread_raw(out.ctypes.data, q["count"], q["offset"])
            if q["ret"] < 0:
                assert ret == -1, q
                assert r.error == q["error"], q
            else:
                assert ret == q["ret"], q
                assert sha(out[: q["ret"]]) == q["sha256"], q


def test_device_zstd_partial_waves(gpu, zs, oracle, zstd):
    """Batches that leave lanes of the kernels' last wave idle (1, 2, 31, 33
    and 65 frames), each decoded right after a 64-frame batch, so idle lanes
    hold another launch's registers: every frame bit-exact (the sequence
    kernel once reduced its item span over idle lanes)."""
    data = datasets(oracle)["synth"]
    frames, sizes = [], []
    for k in range(96):
        src = data[(k * 4096) % 300_000:][:4096]
        frames.append(compress(zstd, src, {P_LEVEL: 3}))
        sizes.append(len(src))
    full, st = device_decode(zs, gpu, frames, sizes)
    assert (st == 0).all()
    for n in (1, 2, 31, 33, 65):
        device_decode(zs, gpu, frames[:64], sizes[:64])
        out, st = device_decode(zs, gpu, frames[:n], sizes[:n])
        assert (st == 0).all(), n
        assert out == full[:n], n


def test_zstd_readers_concurrent(gpu, zs):
    """Readers opened, read and closed from several threads at once, and one
    reader shared by them (the reader serialises its own preads): every read
    bit-exact.  Exercises the pooled Huffman side stream (zstd_decode.hip
    side_acquire / side_release) under interleaved open/close."""
    import threading
    data = zs.synth_buffer(48 * 65536 + 1234)
    img = bytes(zs.zstd_seekable(data, 65536).tobytes())
    shared = zs.Reader(img, 0)
    errors = []

    def work(seed):
        rng = np.random.default_rng(seed)
        try:
            for rnd in range(3):
                r = zs.Reader(img, int(rng.integers(0, 3)))
                for _ in range(6):
                    off = int(rng.integers(0, len(data)))
                    cnt = int(rng.integers(1, 5 * 65536))
                    src = r if rng.integers(0, 2) else shared
                    got = src.pread(cnt, off)
                    if got != data[off: off + cnt].tobytes():
                        errors.append((seed, rnd, off, cnt))
                r.close()
        except Exception as e:   # reported below, not lost in the thread
            errors.append((seed, repr(e)))

    ts = [threading.Thread(target=work, args=(s,)) for s in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=100)
    shared.close()
    assert not any(t.is_alive() for t in ts)
    assert not errors, errors[:4]


@pytest.mark.parametrize("nframes", [4095, 4096, 4099, 8197])
def test_zstd_many_small_frames(gpu, zs, nframes):
    """Batches across the item-bound scan's 4,096-frame tiles (zstd_scan_kernel),
    ragged at the end: a full-range read of 1 KiB frames, bit-exact."""
    data = zs.synth_buffer(nframes * 1024 - 17)
    img = bytes(zs.zstd_seekable(data, 1024).tobytes())
    with zs.Reader(img, 0) as r:
        assert r.read_all(data.size, 0) == data.tobytes()


# ---------------------------------------------------------------------------
# libzstd's double-symbol Huffman decoder (X2) on corrupted literal streams
# ---------------------------------------------------------------------------
def _x2_fixtures():
    import json
    import os
    g = os.path.join(os.path.dirname(__file__), "golden")
    meta = json.load(open(os.path.join(g, "zstd_x2.json")))
    blob = open(os.path.join(g, "zstd_x2.bin"), "rb").read()
    frames = [blob[c["off"]: c["off"] + c["len"]] for c in meta["cases"]]
    return meta, frames


def _x2_seekable(meta, frame, dsize):
    """the case between its two intact neighbours, with a seek table (as
    tests/golden/make_zstd_x2.py built it for the reference)"""
    fa, fb = (bytes.fromhex(h) for h in meta["neighbour_frames_hex"])
    sa, sb = meta["neighbours"]["a"]["dsize"], meta["neighbours"]["b"]["dsize"]
    sizes = [sa, dsize, sb]
    table = bytearray((0x184D2A5E).to_bytes(4, "little") + (8 * 3 + 9).to_bytes(4, "little"))
    for f, s in zip((fa, frame, fb), sizes):
        table += len(f).to_bytes(4, "little") + s.to_bytes(4, "little")
    table += (3).to_bytes(4, "little") + bytes([0]) + (0x8F92EAB1).to_bytes(4, "little")
    return fa + frame + fb + bytes(table), sum(sizes)


@pytest.mark.parametrize("repeat", [1, 700])
def test_device_zstd_x2_fixtures(gpu, zs, repeat):
    """tests/golden/zstd_x2.* (corrupted frames whose literal streams
    libzstd's X2 decoder accepts and an X1 decode rejects) through
    zsk_zstd_decode_frames: libzstd's status and bytes for every frame; at
    700 copies (22,400 frames) the launch runs as the 3-chunk pipeline"""
    import hashlib
    meta, frames = _x2_fixtures()
    cases = meta["cases"]
    out, st = device_decode(zs, gpu, frames * repeat, [c["dsize"] for c in cases] * repeat)
    for i, (o, s) in enumerate(zip(out, st)):
        c = cases[i % len(cases)]
        code = c["libzstd"]["code"]
        if code:
            assert s == ZSK_STATUS_ZSTD | code, (i, hex(int(s)))
        else:
            assert s == 0, (i, hex(int(s)))
            assert hashlib.sha256(o).hexdigest() == c["libzstd"]["sha"], i


@pytest.mark.parametrize("cache", [0, 1])
def test_zstd_x2_fixtures_pread(gpu, zs, cache):
    """the same frames inside seekable files through zseek_pread under a
    caller's loop: the compiled reference's recorded answers (bytes
    delivered, their hash, the last return value and its error string)"""
    import hashlib
    meta, frames = _x2_fixtures()
    for c, frame in zip(meta["cases"], frames):
        img, total = _x2_seekable(meta, frame, c["dsize"])
        want = c["reference"][f"cache{cache}"]
        with zs.Reader(img, cache) as r:
            out = np.empty(total + 1, np.uint8)
            pos = 0
            while True:
                n = r.pread_raw(out.ctypes.data + pos, max(total - pos, 1), pos)
                if n <= 0:
                    break
                pos += n
            assert (pos, n) == (want["bytes"], want["last"]), c["pos"]
            assert hashlib.sha256(out[:pos].tobytes()).hexdigest() == want["sha"]
            if n < 0:
                assert r.error == want["error"]


def _seekable(frames, sizes):
    """a seekable image of the given compressed frames (seek table without
    checksums: entries of compressed / decompressed size, then the footer)"""
    import struct
    table = b"".join(struct.pack("<II", len(f), s) for f, s in zip(frames, sizes))
    table += struct.pack("<IBI", len(frames), 0, 0x8F92EAB1)
    return b"".join(frames) + struct.pack("<II", 0x184D2A5E, len(table)) + table


@pytest.mark.parametrize("cache", [0, 1])
def test_zstd_content_checksum_like_reference(gpu, zs, zstd, ref, cache):
    """Frames carrying a content checksum, one of them wrong: every query,
    read the way callers read (pread again after a short read, until the
    count, EOF or an error), gives the reference library's bytes and then its
    error text -- through the one-frame route (its host plan sees the
    checksum flags and runs the check kernel; a no-cache read that stops
    before the frame's end never reaches the checksum, as libzstd's
    streaming decoder does not).  (One pread may return more than the
    reference's -- several frames, not one -- a legal short-read difference.)"""
    data = zs.synth_buffer(5 * 65536).tobytes()
    frames = [compress(zstd, data[i * 65536:(i + 1) * 65536], {P_LEVEL: 3, P_CHECKSUM: 1}) for i in range(5)]
    bad = bytearray(frames[2])
    bad[-1] ^= 0x5A   # the checksum's last byte
    frames[2] = bytes(bad)
    img = _seekable(frames, [65536] * 5)

    def drive(pread, count, off):
        got, err = b"", None
        while len(got) < count:
            rc, b, e = pread(count - len(got), off + len(got))
            if rc < 0:
                err = e
                break
            if rc == 0:
                break
            got += b
        return got, err

    def ours_pread(r):
        def f(n, o):
            try:
                b = r.pread(n, o)
                return len(b), b, None
            except zs.ZseekError as e:
                return -1, b"", str(e)
        return f

    def ref_pread(r):
        def f(n, o):
            rc, b = r.pread(n, o)
            return rc, b, (r.error if rc < 0 else None)
        return f

    queries = [(100, 2 * 65536), (65536, 2 * 65536), (3 * 65536, 65536), (65536 - 10, 2 * 65536 + 10),
               (10, 3 * 65536 - 10), (5 * 65536, 0), (200, 4 * 65536)]
    for count, off in queries:
        ours = zs.Reader(np.frombuffer(img, np.uint8), cache)
        theirs = ref.open(img, cache)
        try:
            assert drive(ours_pread(ours), count, off) == drive(ref_pread(theirs), count, off), (count, off)
        finally:
            ours.close()
            theirs.close()


@pytest.mark.parametrize("cache", [0, 1])
def test_zstd_content_checksum_many_frames_like_reference(gpu, zs, zstd, ref, cache):
    """a request over more than kOneMaxFrames (64) frames takes the
    device-planned path (zstd_decode_frames), which now passes the no-cache
    stop too: a read ending inside a frame whose content checksum is wrong
    returns the reference's bytes (libzstd's streaming decoder stops before the
    checksum), one running to that frame's end its error."""
    n, fs = 80, 16384
    data = zs.synth_buffer(n * fs).tobytes()
    frames = [compress(zstd, data[i * fs:(i + 1) * fs], {P_LEVEL: 3, P_CHECKSUM: 1}) for i in range(n)]
    bad = bytearray(frames[75])
    bad[-1] ^= 0x5A
    frames[75] = bytes(bad)
    img = _seekable(frames, [fs] * n)
    queries = [(75 * fs + 100, 0), (70 * fs + 5000, 5 * fs), (76 * fs, 0), (fs * 74 - 3, fs + 7)]
    for count, off in queries:
        ours = zs.Reader(np.frombuffer(img, np.uint8), cache)
        theirs = ref.open(img, cache)
        try:
            got, err = b"", None
            while len(got) < count:
                try:
                    b = ours.pread(count - len(got), off + len(got))
                except zs.ZseekError as e:
                    err = str(e)
                    break
                if not b:
                    break
                got += b
            want, werr = b"", None
            while len(want) < count:
                rc, b = theirs.pread(count - len(want), off + len(want))
                if rc < 0:
                    werr = theirs.error
                    break
                if rc == 0:
                    break
                want += b
            assert (got, err) == (want, werr), (count, off)
        finally:
            ours.close()
            theirs.close()


def _literal_sections(frame: bytes):
    """[start, end) of every compressed block's literals section in one zstd
    frame (frame header, block headers and literals headers as RFC 8878
    lays them out)"""
    B = lambda p: frame[p] if p < len(frame) else 0   # noqa: E731
    fhd = B(4)
    fcs, single, did = fhd >> 6, (fhd >> 5) & 1, fhd & 3
    ip = 5 + (0 if single else 1) + (4 if did == 3 else did) + (single if fcs == 0 else (2, 4, 8)[fcs - 1])
    out = []
    while ip + 3 <= len(frame):
        bh = B(ip) | B(ip + 1) << 8 | B(ip + 2) << 16
        typ, size = (bh >> 1) & 3, bh >> 3
        ip += 3
        if typ == 2:
            b0 = B(ip)
            lt, sf = b0 & 3, (b0 >> 2) & 3
            if lt <= 1:
                lh = 2 if sf == 1 else 3 if sf == 3 else 1
                sz = ((b0 | B(ip + 1) << 8) >> 4) if sf == 1 else \
                    ((b0 | B(ip + 1) << 8 | B(ip + 2) << 16) >> 4) if sf == 3 else b0 >> 3
                sec = lh + (sz if lt == 0 else 1)
            else:
                lhc = b0 | B(ip + 1) << 8 | B(ip + 2) << 16 | B(ip + 3) << 24
                sec = (3 + ((lhc >> 14) & 0x3FF)) if sf <= 1 else (4 + (lhc >> 18)) if sf == 2 else \
                    (5 + (lhc >> 22) + (B(ip + 4) << 10))
            out.append((ip, ip + min(sec, size)))
        ip += 1 if typ == 1 else size
        if bh & 1:
            break
    return out


@pytest.mark.parametrize("batch", [0, 40])
def test_device_zstd_x2_corruption_sweep(gpu, zs, oracle, zstd, batch):
    """verdict r05 item 5: >= 1,000 single-byte corruptions inside the Huffman
    literals sections of make_zstd_x2.py's literal-heavy payloads (the
    sections HUF_selectDecoder gives to X2), through zsk_zstd_decode_frames
    in one launch (a lane per frame) and in batches of 40 (the one-frame
    route): every frame's status and bytes are libzstd 1.4.9's own.  Pins on
    the GPU that a stream the X1 walk accepts decodes the same under X2 and
    that x2_rescue re-walks exactly the streams it rejects; the
    oracle's X1-only mode counts the frames where X2 decides the result."""
    import importlib.util
    import os
    from zstd_util import decode
    spec = importlib.util.spec_from_file_location(
        "make_zstd_x2", os.path.join(os.path.dirname(__file__), "golden", "make_zstd_x2.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    rng = np.random.default_rng(11)
    frames, sizes, want = [], [], []
    for name, data, level in mk.payloads():
        comp = compress(zstd, data, {P_LEVEL: level}) if level is not None else compress_stream(zstd, data, 13_000)
        spans = _literal_sections(comp)
        assert spans, name
        pos = np.concatenate([np.arange(a, b) for a, b in spans])
        for p in rng.choice(pos, 260, replace=len(pos) < 260):
            c = bytearray(comp)
            c[int(p)] ^= int(rng.integers(1, 256))
            frames.append(bytes(c))
            sizes.append(len(data))
            want.append(decode(zstd, bytes(c), len(data)))
    assert len(frames) >= 1000
    decisive = 0
    oracle.lib.orc_zstd_x1_only(1)
    try:
        for f, n, (wb, wc) in zip(frames, sizes, want):
            x1 = oracle.zstd_decode(f, n)
            decisive += not (x1[1] == wc and (wc or x1[0] == wb))
    finally:
        oracle.lib.orc_zstd_x1_only(0)
    assert decisive >= 10, decisive   # the sweep reaches frames X2 decides
    if batch:
        out, st = [], []
        for b in range(0, len(frames), batch):
            o, t = device_decode(zs, gpu, frames[b: b + batch], sizes[b: b + batch])
            out += o
            st += list(t)
    else:
        out, st = device_decode(zs, gpu, frames, sizes)
    for i, (n, (wb, wc)) in enumerate(zip(sizes, want)):
        if wc:
            assert st[i] == ZSK_STATUS_ZSTD | wc, (i, hex(int(st[i])), wc)
        else:
            ok = len(wb) == n
            assert st[i] == (0 if ok else 101), (i, hex(int(st[i])))
            if ok:
                assert out[i] == wb, i
