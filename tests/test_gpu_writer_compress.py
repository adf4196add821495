"""The writer's GPU mode (zsk_writer_set_gpu_compress):
files byte-identical to host compression and to the compiled reference
writer for direct, buffered and mixed write sequences, linked frames above
64 KiB (the reference example's 1 MiB frames), frames > 4 MiB on the host in
order, per-frame call_data, stats, callback failures, and the
file decoding back through the reader."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _writes(data: bytes, sizes):
    out, at, i = [], 0, 0
    while at < len(data):
        n = sizes[i % len(sizes)]
        out.append(data[at: at + n])
        at += n
        i += 1
    return out


def _file(zs, chunks, min_frame, level=0, gpu_batch=None, **kw):
    w = zs.Writer(zs.ZSEEK_LZ4, min_frame, level=level, **kw)
    if gpu_batch is not None:
        assert w.set_gpu_compress(gpu_batch)
    for i, c in enumerate(chunks):
        w.write(c, call_data=i + 1)
    return w.close(), w


CASES = [
    (65536, [65536], 0, 0),               # direct frames (config 2's writer)
    (4096, [4096], 0, 65536),             # small direct frames, batch flushed every 16
    (4096, [1000], 0, 0),                 # buffered frames (content size)
    (60000, [7000, 300, 65536], -2, 0),   # mixed buffered / direct, negative level
    (20000, [30000, 200000, 100], 0, 0),  # linked frames > 64 KiB on the GPU
    (1 << 20, [1 << 20], 0, 0),           # the reference example's 1 MiB frames
    (20000, [30000, 5 << 20, 100], 0, 0), # frames > 4 MiB go to the host, in order
    (1, [1, 2, 3], 0, 65536),             # tiny frames
]


@pytest.mark.parametrize("min_frame,sizes,level,batch", CASES)
def test_gpu_writer_matches_host(gpu, zs, min_frame, sizes, level, batch):
    data = bytes(zs.synth_buffer((12 if max(sizes) > 1 << 20 else 3) << 20)) + b"end" * 1000
    if min_frame == 1:
        data = data[:20000]
    chunks = _writes(data, sizes)
    host, hw = _file(zs, chunks, min_frame, level)
    dev, dw = _file(zs, chunks, min_frame, level, gpu_batch=batch)
    assert dev == host
    assert dw.call_data_seen == hw.call_data_seen
    with zs.Reader(dev, 1) as r:
        assert r.read_all(len(data), 0) == data


@pytest.mark.parametrize("min_frame,write", [(65536, 65536), (4096, 1000), (1 << 20, 1 << 16),
                                             (1 << 20, 1 << 20)])
def test_gpu_writer_matches_reference(gpu, zs, ref, min_frame, write):
    """Byte-identical to the compiled reference writer, including the
    reference example's 1 MiB frames (test/example.c)."""
    data = bytes(zs.synth_buffer((6 if min_frame > 65536 else 2) << 20)) + b"tail" * 333
    dev, _ = _file(zs, _writes(data, [write]), min_frame, gpu_batch=0)
    assert dev == ref.compress(data, zs.ZSEEK_LZ4, min_frame, write)


def test_gpu_writer_stats_flush_queue(gpu, zs):
    data = bytes(zs.synth_buffer(1 << 20))
    h = zs.Writer(zs.ZSEEK_LZ4, 65536)
    g = zs.Writer(zs.ZSEEK_LZ4, 65536)
    assert g.set_gpu_compress(0)
    for w in (h, g):
        for f in range(5):
            w.write(data[f * 65536: (f + 1) * 65536])
        w.write(data[5 * 65536: 5 * 65536 + 1000])
    sh, sg = h.stats(), g.stats()
    for k in ("frames", "compressed_size", "seek_table_size"):
        assert sh[k] == sg[k], k
    assert g.callbacks == 5
    assert h.close() == g.close()


def test_gpu_writer_callback_failure(gpu, zs):
    """A failing write callback fails the call that flushed its frame; what
    reached the sink before it is the host writer's prefix."""
    data = bytes(zs.synth_buffer(1 << 20))
    chunks = _writes(data, [65536])
    host, _ = _file(zs, chunks, 65536)
    w = zs.Writer(zs.ZSEEK_LZ4, 65536, fail_on_callback=4)
    assert w.set_gpu_compress(0)
    for c in chunks:
        w.write(c)
    with pytest.raises(zs.ZseekError, match="end_frame_lz4 failed|write to file failed"):
        w.close()
    got = bytes(w._out)
    c_off, _ = zs.seek_table_of(host)
    c3 = int(c_off[3])
    assert got[:c3] == host[:c3]            # frames 1-3 written, the 4th refused
    assert int.from_bytes(got[-9:-5], "little") == 3   # close's seek table: 3 frames


def test_gpu_writer_mode_switch(gpu, zs):
    """GPU mode on mid-stream and off again: the file is unchanged."""
    data = bytes(zs.synth_buffer(2 << 20))
    chunks = _writes(data, [65536, 1000])
    host, _ = _file(zs, chunks, 65536)
    w = zs.Writer(zs.ZSEEK_LZ4, 65536)
    for i, c in enumerate(chunks):
        if i == 3:
            assert w.set_gpu_compress(131072)
        if i == len(chunks) // 2:
            assert w.set_gpu_compress(-1)
        if i == len(chunks) - 3:
            assert w.set_gpu_compress(0)
        w.write(c)
    assert w.close() == host
    np.testing.assert_equal(len(host) > 0, True)


def test_gpu_writer_failure_latches(gpu, zs):
    """Deferred writes (zseek_hip.h): a queued frame's callback failure is
    reported by the later zseek_write that flushed it, and every call after
    it fails too -- the frames queued behind it are never written."""
    data = bytes(zs.synth_buffer(1 << 20))
    chunks = _writes(data, [65536])
    w = zs.Writer(zs.ZSEEK_LZ4, 65536, fail_on_callback=2)
    assert w.set_gpu_compress(2 * 65536)   # a flush every second frame
    w.write(chunks[0])
    with pytest.raises(zs.ZseekError):
        w.write(chunks[1])                 # flushes frames 1-2; frame 2's callback fails
    with pytest.raises(zs.ZseekError):
        w.write(chunks[2])
    with pytest.raises(zs.ZseekError):
        w.close()
    assert w.callbacks == 3                # frames 1, 2 (refused), then close's seek table


def test_gpu_writer_empty_first_write(gpu, zs):
    """An empty zseek_write first (min_frame_size 0: a frame per write) needs
    an output slot although it has no input bytes: the GPU mode allocates its
    first staging for it and the file equals the host writer's."""
    data = bytes(zs.synth_buffer(1 << 20))
    chunks = [b"", b"abc" * 100, b"", data[:70000], b""]
    host, _ = _file(zs, chunks, 0)
    dev, _ = _file(zs, chunks, 0, gpu_batch=0)
    assert dev == host
