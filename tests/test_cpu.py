"""CPU-side checks (no GPU): the oracle against the reference's golden
vectors, the C-ABI library's exports and its host logic (seek table, open /
stats / error conventions, writer)."""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT, golden_file, sha

# LZ4F-option fixtures: frames the reference writer never makes (checksums,
# dictID, linked / bigger blocks) that its reader accepts, read by it
LZ4F = ["lz4f_content_checksum", "lz4f_block_checksum_linked", "lz4f_dictid_1m_blocks",
        "lz4f_all_flags_256k"]
LZ4 = [n for n in ["lz4_64k_direct", "lz4_64k_buffered", "lz4_4k_direct", "lz4_1m_direct",
                   "lz4_1m_buffered", "lz4_odd_frames", "lz4_zeros", "lz4_random",
                   "lz4_periodic", "lz4_text_hc", "lz4_single_byte"]] + LZ4F
LZ4F_CORRUPT = ["lz4f_content_checksum__content_checksum",
                "lz4f_block_checksum_linked__block_checksum",
                "lz4f_all_flags_256k__content_checksum", "lz4f_all_flags_256k__block_checksum"]
ZSTD = ["zstd_64k_direct", "zstd_64k_buffered"]


# ---------------------------------------------------------------------------
# the synthetic generator (SURVEY §8d check values)
# ---------------------------------------------------------------------------
def test_synthetic_check_values(oracle, zs):
    a = oracle.synth(4 << 20, 1)
    assert hashlib.sha256(a.tobytes()).hexdigest().startswith("33244cb45799614f")
    b = zs.synth_buffer(4 << 20)
    assert (a == b).all()
    c = zs.synth_buffer((64 << 20) + 12345)
    assert (c[: 64 << 20] == oracle.synth(64 << 20, 1)).all()
    assert (c[64 << 20:] == oracle.synth(12345, 2)).all()


# ---------------------------------------------------------------------------
# oracle pinned against the reference's own outputs (golden.json)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("name", LZ4)
def test_oracle_decodes_golden_files(oracle, golden, payloads, name):
    img = golden_file(name)
    assert sha(img) == golden["files"][name]["file_sha256"]
    assert oracle.decode_file(img) == payloads[name]


@pytest.mark.parametrize("name", LZ4)
def test_oracle_pread_model_matches_reference(oracle, golden, name):
    img = golden_file(name)
    for q in golden["files"][name]["reads"]:
        got = oracle.pread_model(img, q["count"], q["offset"])
        assert len(got) == q["ret"] and sha(got) == q["sha256"], q


@pytest.mark.parametrize("name", LZ4 + ZSTD)
def test_oracle_seek_table_matches_reference(oracle, golden, name):
    st = oracle.seek_table(golden_file(name))
    ref = golden["files"][name]["stats_cache1"]
    assert st["frames"] == ref["frames"]
    assert int(st["d_off"][-1]) == ref["decompressed_size"]


# failures liblz4's LZ4F_decompress meets while reading a block header or the
# end mark, which it does as soon as the block before has filled the request
HEADER_LEVEL = {"ERROR_maxBlockSize_invalid", "ERROR_frameSize_wrong",
                "ERROR_contentChecksum_invalid"}


def _oracle_error(oracle, img, cache, off, cnt):
    """What the reference reader reports, derived from the oracle's decode:
    None (success) or the error string.  Without a cache the reference
    decodes a frame only as far as the request reaches (decompress.c:614-669)."""
    st = oracle.seek_table(img)
    i = int(np.searchsorted(st["d_off"], np.uint64(off), side="right") - 1)
    c0, c1 = int(st["c_off"][i]), int(st["c_off"][i + 1])
    dsz = int(st["d_off"][i + 1] - st["d_off"][i])
    code, data, _, info = oracle.decode_frame(img[c0:c1], dsz)
    if code == 0:
        return None
    rel = off - int(st["d_off"][i])
    hdr = oracle.error_name(code) in HEADER_LEVEL
    fa = info["fail_at"]
    if not cache:
        end_in = min(rel + cnt, dsz)
        if (end_in < fa) if hdr else (end_in <= fa):
            return None
    if cache:
        prefix, room = "decompress frame", dsz - info["fail_at"]
    elif rel > 0 and ((fa <= rel) if hdr else (fa < rel)):
        prefix, room = "decompress discard data", rel - info["fail_at"]
    else:
        prefix = "decompress user data"
        room = min(cnt, dsz - rel) - (info["fail_at"] - rel)
    name = oracle.error_name(code)
    if info["block_fail"]:
        name = "ERROR_GENERIC" if room >= info["max_block"] else "ERROR_decompressionFailed"
    return f"{prefix}: {name}"


@pytest.mark.parametrize("case", ["block_byte", "block_size_huge", "first_token_offset",
                                  "frame_magic", "flg_version", "flg_reserved", "bd_reserved",
                                  "bd_blocksize", "header_checksum", "1m_block4_offset0",
                                  "1m_block4_size_huge"] + LZ4F_CORRUPT)
def test_oracle_errors_match_reference(oracle, golden, case):
    """Every corruption fixture: the restatement's result (error string, or the
    bytes a partial no-cache read gets) equals the reference's.  1m_block4_offset0
    pins liblz4 1.9.3's zero-offset match (zeros, no error)."""
    rec = golden["corrupt"][case]
    img = bytearray(golden_file(rec.get("base", "lz4_64k_direct")))
    for at, v in rec["mutations"]:
        img[at] = v
    img = bytes(img)
    st = oracle.seek_table(img)
    for q in rec["results"]:
        err = _oracle_error(oracle, img, q["cache"], q["offset"], q["count"])
        if q["ret"] == -1:
            assert err == q["error"], q
        else:
            assert err is None, q
            i = int(np.searchsorted(st["d_off"], np.uint64(q["offset"]), side="right") - 1)
            c0, c1 = int(st["c_off"][i]), int(st["c_off"][i + 1])
            dsz = int(st["d_off"][i + 1] - st["d_off"][i])
            _, data, _, _ = oracle.decode_frame(img[c0:c1], dsz)
            rel = q["offset"] - int(st["d_off"][i])
            got = data[rel: rel + min(q["count"], dsz - rel)]
            assert len(got) == q["ret"] and sha(got) == q["sha256"], q


ZSTD_NAMES = {20: "Corrupted block detected", 22: "Restored data doesn't match checksum"}


def _oracle_zstd_error(oracle, img, cache, off, cnt):
    """The reference's zstd read restated on the oracle's decode: None or the
    error string.  Without a cache libzstd's streaming decoder (decompress.c:
    414-454) decodes a block as soon as the previous one is flushed, so a
    request fails iff it ends at or past the failing block's start, and it
    fails in the discard pass iff that block starts at or before the request."""
    st = oracle.seek_table(img)
    i = int(np.searchsorted(st["d_off"], np.uint64(off), side="right") - 1)
    c0, c1 = int(st["c_off"][i]), int(st["c_off"][i + 1])
    dsz = int(st["d_off"][i + 1] - st["d_off"][i])
    _, code, fa = oracle.zstd_decode_at(img[c0:c1], dsz)
    if code == 0:
        return None
    rel = off - int(st["d_off"][i])
    if cache:
        prefix = "decompress frame"
    elif rel + min(cnt, dsz - rel) < fa:
        return None
    elif rel > 0 and fa <= rel:
        prefix = "decompress discard data"
    else:
        prefix = "decompress user data"
    return f"{prefix}: {ZSTD_NAMES[code]}"


@pytest.mark.parametrize("case", ["zstd1m_block4_first", "zstd1m_block4_type"])
def test_oracle_zstd_partial_reads_match_reference(oracle, golden, case):
    """A corrupt 5th block of a 1 MiB zstd frame (golden, made by the compiled
    reference): the oracle's failing-block offset and the streaming rule give
    the reference's result for every query, bytes included."""
    rec = golden["corrupt"][case]
    img = bytearray(golden_file(rec["base"]))
    for at, v in rec["mutations"]:
        img[at] = v
    img = bytes(img)
    st = oracle.seek_table(img)
    for q in rec["results"]:
        err = _oracle_zstd_error(oracle, img, q["cache"], q["offset"], q["count"])
        if q["ret"] == -1:
            assert err == q["error"], q
            continue
        assert err is None, q
        i = int(np.searchsorted(st["d_off"], np.uint64(q["offset"]), side="right") - 1)
        c0, c1 = int(st["c_off"][i]), int(st["c_off"][i + 1])
        dsz = int(st["d_off"][i + 1] - st["d_off"][i])
        data, _, _ = oracle.zstd_decode_at(img[c0:c1], dsz)
        rel = q["offset"] - int(st["d_off"][i])
        got = data[rel: rel + min(q["count"], dsz - rel)]
        assert len(got) == q["ret"] and sha(got) == q["sha256"], q


def test_oracle_truncated_block_is_an_error(oracle, golden):
    """The reference spins forever here (golden: 'hang'); the restatement
    (and the GPU path) report an error instead."""
    rec = golden["corrupt"]["block_size_short"]
    assert any(q["ret"] == "hang" for q in rec["results"])
    img = bytearray(golden_file("lz4_64k_direct"))
    for at, v in rec["mutations"]:
        img[at] = v
    st = oracle.seek_table(bytes(img))
    c0, c1 = int(st["c_off"][1]), int(st["c_off"][2])
    code, _, _, _ = oracle.decode_frame(bytes(img[c0:c1]), 65536)
    assert code != 0


def test_xxhash_known_answers(oracle):
    # published xxHash test vectors (empty input, seed 0)
    assert oracle.xxh32(b"", 0) == 0x02CC5D05
    assert oracle.xxh64(b"", 0) == 0xEF46DB3751D8E999
    # the LZ4 frame header checksum byte of every golden frame verifies
    img = golden_file("lz4_64k_buffered")
    st = oracle.seek_table(img)
    for i in range(st["frames"]):
        c0 = int(st["c_off"][i])
        flg = img[c0 + 4]
        hdr = 7 + (8 if flg & 8 else 0) + (4 if flg & 1 else 0)
        assert (oracle.xxh32(img[c0 + 4: c0 + hdr - 1]) >> 8) & 0xFF == img[c0 + hdr - 1]


def test_reference_runs_its_pinned_dependencies(zs, ref):
    """The reference runs against the liblz4 1.9.3 / libzstd 1.4.9 it was
    compiled for even with our library -- which links the
    system libzstd 1.4.8 under the same SONAME -- loaded first; and the zstd
    inputs our tools make come from the same libzstd."""
    from oracle.oracle import REF_LZ4_VERSION, REF_ZSTD_VERSION, RefBench
    zs.lib()
    assert ref.versions == {"zstd": REF_ZSTD_VERSION, "lz4": REF_LZ4_VERSION}
    assert RefBench().versions == ref.versions
    assert zs.zstd_tool_version() == "1.4.9"


def test_zstd_tool_image_equals_reference_writer(zs, oracle, ref):
    """Config 5's input path: zstd_seekable (frames compressed in parallel by
    the tools library) writes the file the reference writer writes for
    frame-sized zseek_write calls (level 3, strategy 1, compress.c:58-91)."""
    data = oracle.synth_buffer(3 << 20)
    img = zs.zstd_seekable(data, 65536, 3, 1)
    assert img.tobytes() == ref.compress(data.tobytes(), 0, 65536, 65536)


def test_oracle_vs_reference_roundtrip(oracle, ref):
    """Fresh inputs through the reference writer, decoded by the oracle."""
    rng = np.random.default_rng(11)
    for frame, wsize in [(65536, 65536), (65536, 1000), (1 << 20, 1 << 20), (5000, 7000)]:
        data = oracle.synth(700000, int(rng.integers(1, 1000))).tobytes()
        img = ref.compress(data, 1, frame, wsize)
        assert oracle.decode_file(img) == data


# ---------------------------------------------------------------------------
# the C-ABI library: exports, host logic (no GPU compute)
# ---------------------------------------------------------------------------
def _declared_symbols():
    names = []
    for h in ("zseek.h", "zseek_hip.h"):
        text = "\n".join(ln for ln in open(os.path.join(ROOT, "include", h))
                         if not ln.lstrip().startswith("#"))
        names += re.findall(r"ZSEEK_EXPORT[^;(]*?\b(\w+)\s*\(", text, re.S)
    return names


def test_library_exports_every_declared_symbol(zs):
    declared = _declared_symbols()
    assert len(declared) == len(set(declared)) == len(zs.EXPORTED)
    for n in ("zseek_reader_open_full", "zseek_pread", "zseek_writer_close",
              "zsk_lz4_decode_frames"):
        assert n in declared
    L = zs.lib()
    for n in declared:
        assert hasattr(L, n), n
    assert set(declared) == set(zs.EXPORTED)


def test_library_hides_internals(zs):
    """Only the API is exported (the reference's meson.build:25 hidden visibility):
    every defined dynamic symbol of any type (T, D, B, W, V, i, ...) is one of the
    functions include/*.h declares -- no STL instantiations, kernel handles or
    __hip_cuid_* (the linker version script csrc/libzseek.map)."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", zs.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {}
    for ln in out.splitlines():
        parts = ln.split()
        syms[parts[-1]] = parts[-2]
    assert set(syms) == set(_declared_symbols()), sorted(set(syms) ^ set(_declared_symbols()))
    assert set(syms.values()) == {"T"}


def test_null_handles(zs):
    L = zs.lib()
    err = C.create_string_buffer(80)
    buf = C.create_string_buffer(16)
    assert L.zseek_pread(None, buf, 16, 0, None, err) == 0
    assert err.value == b"invalid reader"
    assert L.zseek_reader_close(None, None, err)
    assert not L.zseek_reader_stats(None, None, err)
    assert L.zseek_write(None, buf, 1, None, err) is False
    assert err.value == b"invalid writer"
    assert L.zseek_writer_close(None, None, err)


@pytest.mark.parametrize("name", LZ4 + ZSTD)
def test_reader_open_and_stats(zs, golden, name):
    entry = golden["files"][name]
    if "open_error" in entry:
        with pytest.raises(zs.ZseekError) as e:
            zs.Reader(golden_file(name), 1)
        assert str(e.value) == entry["open_error"]
        return
    with zs.Reader(golden_file(name), 1) as r:
        st = r.stats()
        assert st["frames"] == entry["stats_cache1"]["frames"]
        assert st["decompressed_size"] == entry["stats_cache1"]["decompressed_size"]
        assert st["cached_frames"] == 0
        assert r.type == (zs.ZSEEK_LZ4 if entry["codec"] == "lz4" else zs.ZSEEK_ZSTD)
        c_off, d_off = r.frames()
        assert int(d_off[-1]) == entry["stats_cache1"]["decompressed_size"]
        # a read past EOF returns 0 without touching the GPU
        assert r.pread(10, int(d_off[-1]) + 5) == b""


def test_empty_file_open_error(zs, golden):
    """Zero-frame file: the reference says 'unrecognized file format'."""
    with pytest.raises(zs.ZseekError) as e:
        zs.Reader(golden_file("lz4_empty"), 1)
    assert str(e.value) == golden["files"]["lz4_empty"]["open_error"]


@pytest.mark.parametrize("case", ["seek_magic", "seek_descriptor", "file_magic", "truncated",
                                  "zero_bytes", "three_bytes"])
def test_open_errors_match_reference(zs, golden, case):
    rec = golden["corrupt"][case]
    base = golden_file("lz4_64k_direct")
    if "truncate" in rec:
        img = base[: rec["truncate"]]
    else:
        b = bytearray(base)
        for at, v in rec["mutations"]:
            b[at] = v
        img = bytes(b)
    if len(img) == 0:
        img = b""
    with pytest.raises(zs.ZseekError) as e:
        zs.Reader(img if img else b"\0"[:0], 1)
    assert str(e.value) == rec["open_error"]


@pytest.mark.parametrize("name", [n for n in LZ4 if n != "lz4_text_hc" and n not in LZ4F])
def test_writer_byte_identical_to_reference(zs, golden, payloads, name):
    entry = golden["files"][name]
    data = payloads[name]
    w = zs.Writer(zs.ZSEEK_LZ4, entry["min_frame_size"], level=entry["level"])
    for s in range(0, len(data), entry["write_size"]):
        w.write(data[s: s + entry["write_size"]])
    assert sha(w.close()) == entry["file_sha256"]


def test_writer_stats(zs):
    w = zs.Writer(zs.ZSEEK_LZ4, 65536)
    w.write(bytes(100000))          # >= min_frame_size: one direct frame
    st = w.stats()
    assert st["frames"] == 1 and st["seek_table_size"] == 8 + 8 * 1 + 9
    w.write(bytes(1000))            # buffered: counted as a pending frame
    st = w.stats()
    assert st["frames"] == 2 and st["seek_table_size"] == 8 + 8 * 1 + 9 + 8
    img = w.close()
    with zs.Reader(img, 0) as r:
        assert r.stats()["frames"] == 2


def test_tools_image_equals_writer(zs):
    data = zs.synth_buffer(3 << 20)
    for frame in (4096, 65536, 1 << 20, 100000):
        w = zs.Writer(zs.ZSEEK_LZ4, frame)
        for s in range(0, data.size, frame):
            w.write(data[s: s + frame].tobytes())
        assert zs.lz4_seekable(data, frame).tobytes() == w.close()


def test_seek_table_with_checksums(zs, oracle):
    """Descriptor bit 7 (per-frame XXH64 low-32 checksums, ref
    seek_table.c:95-97): parsed, entries 12 bytes wide."""
    data = zs.synth_buffer(200000)
    img = bytearray(zs.lz4_seekable(data, 65536).tobytes())
    st = oracle.seek_table(bytes(img))
    n = st["frames"]
    body = img[: int(st["c_off"][-1])]
    table = bytearray()
    table += (0x184D2A5E).to_bytes(4, "little") + (12 * n + 9).to_bytes(4, "little")
    for i in range(n):
        c = int(st["c_off"][i + 1] - st["c_off"][i])
        d = int(st["d_off"][i + 1] - st["d_off"][i])
        ck = oracle.xxh64(data[int(st["d_off"][i]): int(st["d_off"][i + 1])].tobytes()) & 0xFFFFFFFF
        table += c.to_bytes(4, "little") + d.to_bytes(4, "little") + ck.to_bytes(4, "little")
    table += n.to_bytes(4, "little") + bytes([0x80]) + (0x8F92EAB1).to_bytes(4, "little")
    img2 = bytes(body + table)
    st2 = oracle.seek_table(img2)
    assert st2["checksum_flag"] and st2["frames"] == n
    with zs.Reader(img2, 0) as r:
        c_off, d_off = r.frames()
        assert (d_off == st["d_off"]).all() and (c_off == st["c_off"]).all()


def test_oracle_xxh64_matches_xxhash_package(oracle):
    """The oracle's XXH64 (the checker of the GPU frame checksums) against the
    independent xxhash package: every tail length and a few frame sizes."""
    xxhash = pytest.importorskip("xxhash")
    rng = np.random.default_rng(5)
    for n in list(range(0, 80)) + [1000, 4096, 65536, 65537, 100003]:
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.xxh64(b) == xxhash.xxh64_intdigest(b, seed=0), n


def test_with_frame_checksums_layout(zs, oracle):
    """zs.with_frame_checksums writes the table the oracle's restatement of
    seek_table.c:62-176 parses, checksums included, and the library opens."""
    data = zs.synth_buffer(300000)
    img = zs.lz4_seekable(data, 65536)
    st = oracle.seek_table(img.tobytes())
    cks = [oracle.xxh64(data[int(st["d_off"][i]): int(st["d_off"][i + 1])].tobytes()) & 0xFFFFFFFF
           for i in range(st["frames"])]
    img2 = zs.with_frame_checksums(img, cks)
    st2 = oracle.seek_table(img2.tobytes())
    assert st2["checksum_flag"] and st2["frames"] == st["frames"]
    assert (st2["checksum"] == np.array(cks, np.uint32)).all()
    assert (st2["c_off"] == st["c_off"]).all() and (st2["d_off"] == st["d_off"]).all()
    with zs.Reader(img2, 0) as r:
        r.set_verify_checksums(True)
        c_off, d_off = r.frames()
        assert (d_off == st["d_off"]).all()


def test_checksum_table_read_by_reference(zs, oracle, ref):
    """The reference itself opens and decodes a with_frame_checksums image
    (12-byte entries, descriptor 0x80)."""
    data = zs.synth_buffer(300000)
    img = zs.lz4_seekable(data, 65536)
    n = oracle.seek_table(img.tobytes())["frames"]
    img2 = zs.with_frame_checksums(img, [0x01234567 * (i + 1) for i in range(n)]).tobytes()
    r = ref.open(img2, 0)
    try:
        assert r.h, r.error
        ok, st = r.stats()
        assert ok and st["frames"] == n
        got, b = r.pread(1000, 70000)
        assert got == 1000 and b == data[70000:71000].tobytes()
    finally:
        r.close()


def test_gpu_stats_respects_caller_struct_size(zs):
    """zsk_reader_gpu_stats writes only the round-4 layout (through
    `device`), so a caller built against the shorter struct is never written
    past it; zsk_reader_gpu_stats_ex writes exactly the bytes it is given."""
    import ctypes as C
    L = zs.lib()
    full = C.sizeof(zs.GpuStatsC)
    old = zs.GpuStatsC.copy_threads.offset
    with zs.Reader(golden_file("lz4_64k_direct"), 1) as r:
        buf = (C.c_uint8 * (full + 16))(*([0xAB] * (full + 16)))
        assert L.zsk_reader_gpu_stats(r._h, C.cast(buf, C.POINTER(zs.GpuStatsC)))
        assert bytes(buf[old:]) == b"\xab" * (full + 16 - old)
        assert int.from_bytes(bytes(buf[old - 4:old]), "little", signed=True) == -1   # device: no lane yet
        buf = (C.c_uint8 * (full + 16))(*([0xAB] * (full + 16)))
        assert L.zsk_reader_gpu_stats_ex(r._h, C.cast(buf, C.POINTER(zs.GpuStatsC)), full)
        assert bytes(buf[full:]) == b"\xab" * 16
        s = zs.GpuStatsC.from_buffer(buf)
        assert s.copy_threads >= 2 and s.io_parts >= 1
        buf = (C.c_uint8 * 8)(*([0xAB] * 8))
        assert L.zsk_reader_gpu_stats_ex(r._h, C.cast(buf, C.POINTER(zs.GpuStatsC)), 4)
        assert bytes(buf[4:]) == b"\xab" * 4
        assert not L.zsk_reader_gpu_stats_ex(r._h, C.cast(buf, C.POINTER(zs.GpuStatsC)), 0)
