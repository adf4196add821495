"""GPU: the reader's batch pipeline and its device lanes (reader.cpp).

A read runs as a pipeline of batches (user pread / upload + decode +
download / copy into the caller's buffer overlapping, kSlots in flight) on
one lane per entry of the reader's device list.  These tests drive many
small batches and two lanes on one GPU (the device list may repeat a device),
and check every byte, the short read at a corrupt frame in a later batch, the
error of the next call, and the cache contents against the reference library
(oracle/_ref) running the same call loop.
"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FRAME = 65536


@pytest.fixture(scope="module")
def synth_img(zs):
    data = zs.synth_buffer(8 << 20)                    # 128 frames of 64 KiB
    tail = np.frombuffer(b"ragged-tail" * 1000, np.uint8)
    data = np.concatenate([data, tail])                # + one short frame
    img = zs.lz4_seekable(data, FRAME)
    return data, img


def corrupt(zs, img, frame):
    """Frame `frame` of the image with a broken FLG byte (version bits: liblz4
    says ERROR_headerVersion_wrong; the file's magic stays intact)."""
    c_off, _ = zs.seek_table_of(img)
    bad = img.copy()
    bad[int(c_off[frame]) + 4] ^= 0xFF
    return bad


@pytest.mark.parametrize("batch", [4096, 3 * FRAME + 7, 1 << 20, 64 << 20])
@pytest.mark.parametrize("lanes", [1, 2, 3])
def test_pipeline_full_and_partial_reads(gpu, zs, synth_img, batch, lanes):
    data, img = synth_img
    with zs.Reader(img, 0) as r:
        r.set_batch_bytes(batch)
        r.set_devices([0] * lanes)
        assert r.pread(len(data) + 100, 0) == data.tobytes()
        for off, cnt in [(1, len(data) - 1), (FRAME - 3, 5 * FRAME), (777777, 3 << 20),
                         (len(data) - 20000, 1 << 20), (12345, 7)]:
            assert r.pread(cnt, off) == data[off: off + cnt].tobytes(), (off, cnt)
        assert r.devices() == [0] * lanes


@pytest.mark.parametrize("lanes", [1, 2])
def test_pread_device_lanes(gpu, zs, synth_img, lanes):
    import torch
    data, img = synth_img
    with zs.Reader(img, 0) as r:
        r.set_batch_bytes(1 << 20)
        r.set_devices([0] * lanes)
        out = torch.zeros(len(data), dtype=torch.uint8, device=gpu)
        assert r.pread_device(out.data_ptr(), len(data), 0) == len(data)
        assert out.cpu().numpy().tobytes() == data.tobytes()
        part = torch.zeros(3 << 20, dtype=torch.uint8, device=gpu)
        n = r.pread_device(part.data_ptr(), 3 << 20, 1000001)
        assert part[:n].cpu().numpy().tobytes() == data[1000001: 1000001 + n].tobytes()


@pytest.mark.parametrize("bad_frame", [0, 5, 50, 120])
@pytest.mark.parametrize("lanes", [1, 2])
@pytest.mark.parametrize("cache", [0, 3])
def test_corrupt_frame_in_later_batch(gpu, zs, ref, synth_img, bad_frame, lanes, cache):
    """A corrupt frame in batch k+1 while batches k+2.. are already in flight:
    the read returns exactly the bytes before it, the next call starting there
    fails with the reference's error text, and the cache holds what the
    reference's frame-by-frame loop over the same range leaves (the last good
    frames before the failure)."""
    data, img = synth_img
    bad = corrupt(zs, img, bad_frame)
    start = bad_frame * FRAME
    with zs.Reader(bad, cache) as r:
        r.set_batch_bytes(4 * FRAME)
        r.set_devices([0] * lanes)
        out = np.empty(len(data), np.uint8)
        n = r.pread_raw(out.ctypes.data, len(data), 0)
        if bad_frame == 0:
            assert n == -1
        else:
            assert n == start
            assert out[:n].tobytes() == data[:n].tobytes()
        assert r.pread_raw(out.ctypes.data, 1 << 20, start) == -1
        ours_err = r.error
        ours_cached = r.stats()["cached_frames"]
    theirs = ref.open(bad.tobytes(), cache)
    pos = 0
    while True:   # the reference's caller loop until the error
        rb, got = theirs.pread(1 << 20, pos)
        if rb <= 0:
            break
        pos += rb
    assert pos == start
    rb, _ = theirs.pread(1 << 20, start)
    assert rb == -1
    assert ours_err == theirs.error
    assert ours_cached == theirs.stats()[1]["cached_frames"]
    theirs.close()


def test_cache_after_multi_lane_read(gpu, zs, ref, synth_img):
    """cache_size 5, a full read over two lanes, then single-frame reads: the
    frames the cache holds are served without a GPU batch, as many as the
    reference holds after its loop."""
    data, img = synth_img
    with zs.Reader(img, 5) as r:
        r.set_batch_bytes(8 * FRAME)
        r.set_devices([0, 0])
        assert r.pread(len(data), 0) == data.tobytes()
        assert r.stats()["cached_frames"] == 5
        b0 = r.gpu_stats()["batches"]
        last = len(data) // FRAME   # the short frame's index
        for f in range(last - 4, last + 1):
            off = f * FRAME + 10
            assert r.pread(100, off) == data[off: off + 100].tobytes()
        assert r.gpu_stats()["batches"] == b0          # all hits
        r.pread(100, 3 * FRAME)                         # a miss: one batch
        assert r.gpu_stats()["batches"] == b0 + 1
    theirs = ref.open(img.tobytes(), 5)
    pos = 0
    while pos < len(data):
        rb, _ = theirs.pread(1 << 20, pos)
        pos += rb
    assert theirs.stats()[1]["cached_frames"] == 5
    theirs.close()


def test_devices_env_single_lane(gpu, zs, synth_img, monkeypatch):
    """ZSEEK_HIP_DEVICES=0: the single-device path, one lane."""
    data, img = synth_img
    monkeypatch.setenv("ZSEEK_HIP_DEVICES", "0")
    with zs.Reader(img, 0) as r:
        assert r.pread(len(data), 0) == data.tobytes()
        assert r.devices() == [0]
    monkeypatch.setenv("ZSEEK_HIP_DEVICES", "0,0")
    with zs.Reader(img, 0) as r:
        assert r.pread(len(data), 0) == data.tobytes()
        assert r.devices() == [0, 0]


def test_set_devices_rejects_invalid(gpu, zs, synth_img):
    import torch
    _, img = synth_img
    with zs.Reader(img, 0) as r:
        with pytest.raises(zs.ZseekError):
            r.set_devices([torch.cuda.device_count()])
        with pytest.raises(zs.ZseekError):
            r.set_devices([-1])


def test_zstd_pipeline_lanes(gpu, zs):
    data = zs.synth_buffer(6 << 20)
    img = zs.zstd_seekable(data, FRAME)
    with zs.Reader(img, 2) as r:
        r.set_batch_bytes(5 * FRAME)
        r.set_devices([0, 0])
        assert r.pread(len(data), 0) == data.tobytes()
        assert r.pread(300000, 1234567) == data[1234567: 1234567 + 300000].tobytes()


def test_single_frame_reads_one_batch_each(gpu, zs, synth_img):
    """Small reads inside one frame (the latency path): one batch of one
    frame per read without a cache, hits with one."""
    data, img = synth_img
    rng = np.random.default_rng(3)
    for cache in (0, 1):
        with zs.Reader(img, cache) as r:
            for _ in range(50):
                off = int(rng.integers(0, len(data) - 4096))
                if off // FRAME != (off + 4095) // FRAME:
                    continue
                b0 = r.gpu_stats()["batches"]
                assert r.pread(4096, off) == data[off: off + 4096].tobytes()
                assert r.gpu_stats()["batches"] - b0 <= 1


@pytest.mark.parametrize("io", [2, 4, 8])
def test_parallel_pread_callbacks(gpu, zs, io):
    """zsk_reader_set_io_threads: a batch's compressed span read by concurrent
    pread calls on disjoint pieces (the in-memory callback is safe for it):
    every byte exact, multi-batch, ragged, and a read past the end."""
    data = zs.synth_buffer(40 << 20)
    img = zs.lz4_seekable(data, FRAME)
    with zs.Reader(img, 0) as r:
        r.set_io_threads(io)
        r.set_batch_bytes(24 << 20)
        assert r.pread(len(data), 0) == data.tobytes()
        assert r.pread(len(data), 12345) == data[12345:].tobytes()
    with zs.Reader(img, 0) as r:
        with pytest.raises(zs.ZseekError):
            r.set_io_threads(0)


def test_concurrent_cache_hits_and_stats_during_read(gpu, zs, synth_img):
    """The reference's reader concurrency (decompress.c:699-706, :850-875):
    cache hits run under a shared lock, so several threads read one warm
    frame at once; and zseek_reader_stats answers while a large GPU read on
    the same reader is in flight."""
    import threading
    data, img = synth_img
    with zs.Reader(img, 4) as r:
        base = 5 * FRAME
        assert r.pread(4096, base) == data[base: base + 4096].tobytes()   # warm
        b0 = r.gpu_stats()["batches"]
        errors = []

        def hits(seed):
            rng = np.random.default_rng(seed)
            for _ in range(300):
                o = base + int(rng.integers(0, FRAME - 512))
                n = int(rng.integers(1, 513))
                if r.pread(n, o) != data[o: o + n].tobytes():
                    errors.append((o, n))

        th = [threading.Thread(target=hits, args=(s,)) for s in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors
        assert r.gpu_stats()["batches"] == b0          # every read a hit
        assert r.stats()["cached_frames"] == 1
    with zs.Reader(img, 0) as r:
        r.set_batch_bytes(FRAME)                        # one frame per batch: a long read
        out = {}
        t = threading.Thread(target=lambda: out.setdefault("got", r.pread(len(data), 0)))
        t.start()
        during = 0
        while t.is_alive():
            st = r.stats()
            assert st["frames"] == 129 and st["decompressed_size"] == len(data)
            during += t.is_alive()
        t.join()
        assert out["got"] == data.tobytes()
        assert during > 0   # stats calls returned while the read was in flight


def test_two_lanes_one_gib_into_host_buffer(gpu, zs):
    """zsk_reader_set_devices([0, 0]): a 1 GiB zseek_pread into a host buffer
    over two lanes (each its own host thread, slots and streams) is bit-exact,
    and both lanes decoded half the frames (lane_plan.h's split)."""
    data = zs.synth_buffer(1 << 30)
    img = zs.lz4_seekable(data, FRAME)
    out = np.empty(data.size, np.uint8)
    with zs.Reader(img, 0) as r:
        r.set_devices([0, 0])
        assert r.pread_raw(out.ctypes.data, data.size, 0) == data.size
        st = r.gpu_stats()
    assert np.array_equal(out, data)
    assert st["frames_decoded"] == data.size // FRAME
