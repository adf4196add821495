"""Seek-table frame checksums checked on the GPU (SURVEY §8f row 3;
csrc/frame_check.hip).  Expected values come from the oracle's XXH64
(pinned against the published vectors and the xxhash package in
test_cpu.py), low 32 bits, as seek_table.c:95-97 stores them.  The reference
parses these tables but never checks them, so the reader only does when
asked (zsk_reader_set_verify_checksums)."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _checksums(oracle, data, d_off) -> np.ndarray:
    return np.array([oracle.xxh64(data[int(d_off[i]): int(d_off[i + 1])].tobytes()) & 0xFFFFFFFF
                     for i in range(len(d_off) - 1)], np.uint32)


def _decode(zs, img, gpu, zstd=False):
    import torch
    c_off, d_off = zs.seek_table_of(img)
    n = len(c_off) - 1
    b = zs.frame_batch(c_off, d_off, 0, n)
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(gpu)
    comp = torch.zeros(b.comp_end + 256, dtype=torch.uint8, device=gpu)
    comp[: b.comp_end].copy_(torch.from_numpy(np.asarray(img[: b.comp_end]).copy()))
    out = torch.zeros(max(b.out_bytes, 1), dtype=torch.uint8, device=gpu)
    status = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    (zs.zstd_decode_frames if zstd else zs.decode_frames)(desc, comp, out, status)
    torch.cuda.synchronize()
    return desc, out, status, d_off


def _dev(want, gpu):
    import torch
    return torch.from_numpy(np.ascontiguousarray(want, np.uint32).view(np.int32)).to(gpu)


@pytest.mark.parametrize("frame,size", [(65536, 3 << 20), (4096, 1 << 20), (65537, 2 << 20),
                                        (3000, 1 << 20), (1 << 20, 3 << 20), (40, 20000),
                                        (31, 5000), (7, 700)])
def test_device_checksums(gpu, zs, oracle, frame, size):
    """Every frame size class: whole stripes, ragged tails, frames < 32 B."""
    import torch
    data = zs.synth_buffer(size)
    img = zs.lz4_seekable(data, frame)
    desc, out, status, d_off = _decode(zs, img, gpu)
    assert int((status != 0).sum()) == 0
    want = _checksums(oracle, data, d_off)
    zs.verify_frame_checksums(desc, out, _dev(want, gpu), status)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    # one bit off in a few expected values: exactly those frames fail
    n = len(want)
    bad = sorted({0, n // 2, n - 1})
    want[bad] ^= 1
    status.zero_()
    zs.verify_frame_checksums(desc, out, _dev(want, gpu), status)
    got = status.cpu().numpy()
    assert list(np.nonzero(got)[0]) == bad
    assert (got[bad] == zs.ZSK_ERR_SEEK_CHECKSUM).all()


def test_failed_frames_are_left_alone(gpu, zs, oracle):
    data = zs.synth_buffer(1 << 20)
    img = zs.lz4_seekable(data, 65536)
    desc, out, status, d_off = _decode(zs, img, gpu)
    want = _checksums(oracle, data, d_off)
    want[3] ^= 0xFF
    status[3] = 16   # a decode failure already recorded
    zs.verify_frame_checksums(desc, out, _dev(want, gpu), status)
    got = status.cpu().numpy()
    assert got[3] == 16 and int(np.count_nonzero(np.delete(got, 3))) == 0


def test_zstd_frames(gpu, zs, oracle):
    data = zs.synth_buffer(2 << 20)
    img = zs.zstd_seekable(data, 65536)
    desc, out, status, d_off = _decode(zs, img, gpu, zstd=True)
    assert int((status != 0).sum()) == 0
    want = _checksums(oracle, data, d_off)
    want[7] ^= 1
    zs.verify_frame_checksums(desc, out, _dev(want, gpu), status)
    got = status.cpu().numpy()
    assert list(np.nonzero(got)[0]) == [7]


@pytest.mark.parametrize("codec", ["lz4", "zstd"])
@pytest.mark.parametrize("cache", [0, 1])
def test_reader_checks_when_asked(gpu, zs, oracle, codec, cache):
    data = zs.synth_buffer(2 << 20)
    img = zs.lz4_seekable(data, 65536) if codec == "lz4" else zs.zstd_seekable(data, 65536)
    c_off, d_off = zs.seek_table_of(img)
    want = _checksums(oracle, data, d_off)
    with zs.Reader(zs.with_frame_checksums(img, want), cache) as r:
        r.set_verify_checksums(True)
        assert r.read_all(data.size, 0) == data.tobytes()
        assert r.pread(1000, 70000) == data[70000:71000].tobytes()
    want[5] ^= 1
    bad = zs.with_frame_checksums(img, want)
    with zs.Reader(bad, cache) as r:   # default off: the reference never checks
        assert r.read_all(data.size, 0) == data.tobytes()
    with zs.Reader(bad, cache) as r:
        r.set_verify_checksums(True)
        # a range read stops before the bad frame; a read inside it fails
        assert r.pread(data.size, 0) == data[: int(d_off[5])].tobytes()
        with pytest.raises(zs.ZseekError) as e:
            r.pread(100, int(d_off[5]) + 7)
        assert str(e.value).endswith(": frame checksum mismatch")
        d6 = int(d_off[6])
        assert r.pread(100, d6) == data[d6: d6 + 100].tobytes()
