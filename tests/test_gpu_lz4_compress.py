"""GPU LZ4 frame compression (csrc/lz4_compress.hip)
against the oracle restatement (pinned to liblz4 1.9.3 and the reference
writer in test_lz4_compress.py): byte-identical frames for edge sizes and
contents, levels, the content-size flag, stored (incompressible) blocks and
refused descriptors; linked frames above 64 KiB (the reference example's
1 MiB frames); at full size, 64 KiB- and 1 MiB-frame seekable files identical
to the ones liblz4 makes, and a round trip through the GPU decoder."""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(zs, gpu, src: np.ndarray, sizes, offsets=None, flags=None, level=0):
    import torch
    desc, dst_bytes = zs.lz4_compress_layout(sizes, offsets, flags)
    n = len(sizes)
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    d_src = torch.from_numpy(np.ascontiguousarray(src)).to(gpu) if src.size else \
        torch.zeros(16, dtype=torch.uint8, device=gpu)
    d_dst = torch.full((max(dst_bytes, 16),), 0xA5, dtype=torch.uint8, device=gpu)
    csize = torch.full((max(n, 1),), -1, dtype=torch.int32, device=gpu)[:n]
    zs.lz4_compress_frames(d_desc, d_src, d_dst, csize, level)
    torch.cuda.synchronize()
    dst = d_dst.cpu().numpy()
    cs = csize.cpu().numpy()
    return [dst[int(desc["dst_off"][f]):][: int(cs[f])].tobytes() for f in range(n)], cs


def _edge_batch(oracle):
    rng = np.random.default_rng(11)
    syn = oracle.synth_buffer(1 << 21)
    chunks = []
    for n in (0, 1, 4, 5, 11, 12, 13, 14, 15, 16, 20, 64, 270, 1000, 4096, 65534, 65535, 65536):
        chunks += [rng.integers(0, 256, n, dtype=np.uint8), np.zeros(n, np.uint8),
                   rng.integers(0, 3, n, dtype=np.uint8), syn[:n], syn[(1 << 20):][:n]]
    for _ in range(120):
        n = int(rng.integers(0, 65537))
        o = int(rng.integers(0, syn.size - n))
        chunks.append(syn[o: o + n])
        chunks.append(rng.integers(0, int(rng.integers(1, 257)), n, dtype=np.uint8))
    for k in (14, 15, 16, 269, 270, 271, 525):
        b = rng.integers(0, 256, k, dtype=np.uint8)
        chunks.append(np.concatenate([b, b, b, np.full(k, ord("x"), np.uint8)]))
    return chunks


@pytest.mark.parametrize("level", [0, -1, -7])
def test_gpu_frames_match_oracle(gpu, zs, oracle, level):
    chunks = _edge_batch(oracle)
    sizes = [c.size for c in chunks]
    flags = np.arange(len(chunks), dtype=np.uint32) % 2   # content size on every other frame
    src = np.concatenate(chunks)
    got, cs = _run(zs, gpu, src, sizes, flags=flags, level=level)
    for f, c in enumerate(chunks):
        want = oracle.lz4f_compress_frame(c.tobytes(), level, bool(flags[f]))
        assert got[f] == want, (f, c.size, level, int(flags[f]), int(cs[f]), len(want))


def test_gpu_frames_unaligned_sources(gpu, zs, oracle):
    """Frames starting at odd offsets of the input (buffered writer frames)."""
    syn = oracle.synth_buffer(1 << 21)
    rng = np.random.default_rng(5)
    offs = np.sort(rng.integers(0, (1 << 21) - 65536, 64)).astype(np.uint64)
    sizes = rng.integers(1, 65537, 64).astype(np.uint64)
    got, _ = _run(zs, gpu, syn, sizes, offsets=offs, flags=np.ones(64, np.uint32))
    for f in range(64):
        chunk = syn[int(offs[f]):][: int(sizes[f])].tobytes()
        assert got[f] == oracle.lz4f_compress_frame(chunk, 0, True), f


def _linked_batch(oracle):
    rng = np.random.default_rng(12)
    syn = oracle.synth_buffer(1 << 22)
    noise = rng.integers(0, 256, 1 << 20, dtype=np.uint8)
    blk = rng.integers(0, 256, 65536, dtype=np.uint8)
    chunks = [syn[:1 << 20], syn[777:777 + (1 << 20)], syn[:65537], syn[:65536 + 12], syn[:65536 + 13],
              syn[:3 * 65536 + 999], noise[:200000],
              np.concatenate([noise[:65536], syn[:65536], noise[:70000], syn[5:5 + 2 * 65536]]),
              np.tile(syn[:100000], 3), np.zeros(300000, np.uint8), rng.integers(0, 4, 400000, dtype=np.uint8),
              np.tile(blk[:65535], 3), np.tile(blk, 3),
              np.concatenate([blk, [122], blk, [122, 122], blk]).astype(np.uint8),
              syn[: 4 << 20]]   # ZSK_LZ4_COMPRESS_MAX_FRAME
    for _ in range(12):
        n = int(rng.integers(65537, 1 << 21))
        o = int(rng.integers(0, syn.size - n))
        chunks.append(syn[o: o + n])
    return chunks


@pytest.mark.parametrize("level", [0, -2])
def test_gpu_linked_frames_match_oracle(gpu, zs, oracle, level):
    """Frames above 64 KiB: linked 64 KiB blocks on one stream, stored blocks
    in between, short last blocks, the 65535 distance limit, 4 MiB frames."""
    chunks = _linked_batch(oracle)
    sizes = [c.size for c in chunks]
    flags = np.arange(len(chunks), dtype=np.uint32) % 2
    got, cs = _run(zs, gpu, np.concatenate(chunks), sizes, flags=flags, level=level)
    for f, c in enumerate(chunks):
        want = oracle.lz4f_compress_frame(c.tobytes(), level, bool(flags[f]))
        assert got[f] == want, (f, c.size, level, int(cs[f]), len(want))


def test_gpu_1mib_frames_match_liblz4(gpu, zs):
    """256 MiB in the reference example's 1 MiB frames (test/example.c): every
    GPU frame equals the one liblz4 wrote into the writer-identical image, and
    the frames decode back to the input on the GPU."""
    import torch
    data = zs.synth_buffer(256 << 20)
    img = np.asarray(zs.lz4_seekable(data, 1 << 20))
    c_off, d_off = zs.seek_table_of(img)
    n = len(c_off) - 1
    got, cs = _run(zs, gpu, data, np.diff(d_off))
    for f in range(n):
        assert got[f] == img[c_off[f]: c_off[f + 1]].tobytes(), f
    ddesc = np.zeros(n, zs.FRAME_DESC_DTYPE)
    ddesc["c_off"] = c_off[:-1]
    ddesc["d_off"] = d_off[:-1]
    ddesc["c_size"] = np.diff(c_off)
    ddesc["d_size"] = np.diff(d_off)
    out = torch.empty(data.size, dtype=torch.uint8, device=gpu)
    status = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    zs.decode_frames(torch.from_numpy(ddesc.view(np.uint8).copy()).to(gpu),
                     torch.from_numpy(np.concatenate([img, np.zeros(16, np.uint8)])).to(gpu), out, status)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert np.array_equal(out.cpu().numpy(), data)


def test_gpu_refused_descriptors(gpu, zs):
    import torch
    desc, _ = zs.lz4_compress_layout([100, (4 << 20) + 1, 100])
    desc["dst_off"][2] += 4   # not 16-byte aligned
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    src = torch.zeros(1 << 18, dtype=torch.uint8, device=gpu)
    dst = torch.zeros(1 << 18, dtype=torch.uint8, device=gpu)
    cs = torch.full((3,), -1, dtype=torch.int32, device=gpu)
    zs.lz4_compress_frames(d_desc, src, dst, cs, 0)
    torch.cuda.synchronize()
    assert cs.cpu().tolist()[1:] == [0, 0]
    assert cs.cpu().tolist()[0] > 0
    with pytest.raises(zs.ZseekError):
        zs.lz4_compress_frames(d_desc, src, dst, cs, 3)   # HC levels: not on this path


def test_gpu_seekable_file_matches_liblz4(gpu, zs):
    """64 MiB of §8d synthetic input in 64 KiB frames: every GPU frame equals
    the frame liblz4 wrote into the writer-identical seekable image."""
    data = zs.synth_buffer(64 << 20)
    img = np.asarray(zs.lz4_seekable(data, 65536))
    c_off, d_off = zs.seek_table_of(img)
    n = len(c_off) - 1
    got, cs = _run(zs, gpu, data, np.diff(d_off))
    for f in range(n):
        assert got[f] == img[c_off[f]: c_off[f + 1]].tobytes(), f


def test_gpu_full_size_round_trip(gpu, zs, oracle):
    """1 GiB in 64 KiB frames: compress on the GPU, decode the frames with the
    GPU decoder, compare with the input; 64 sampled frames against the oracle."""
    import torch
    n_bytes = 1 << 30
    data = zs.synth_buffer(n_bytes)
    sizes = np.full(n_bytes // 65536, 65536, np.uint64)
    desc, dst_bytes = zs.lz4_compress_layout(sizes)
    n = sizes.size
    d_src = torch.from_numpy(data).to(gpu)
    d_dst = torch.empty(dst_bytes, dtype=torch.uint8, device=gpu)
    cs = torch.empty(n, dtype=torch.int32, device=gpu)
    zs.lz4_compress_frames(torch.from_numpy(desc.view(np.uint8).copy()).to(gpu), d_src, d_dst, cs, 0)
    torch.cuda.synchronize()
    csz = cs.cpu().numpy().astype(np.uint64)
    assert (csz > 0).all()
    ddesc = np.zeros(n, zs.FRAME_DESC_DTYPE)
    ddesc["c_off"] = desc["dst_off"]
    ddesc["d_off"] = np.arange(n, dtype=np.uint64) * 65536
    ddesc["c_size"] = csz
    ddesc["d_size"] = 65536
    out = torch.empty(n_bytes, dtype=torch.uint8, device=gpu)
    status = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    zs.decode_frames(torch.from_numpy(ddesc.view(np.uint8).copy()).to(gpu), d_dst, out, status)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert torch.equal(out, d_src)
    host = d_dst.cpu().numpy()
    for f in np.random.default_rng(2).integers(0, n, 64):
        frame = host[int(desc["dst_off"][f]):][: int(csz[f])].tobytes()
        assert frame == oracle.lz4f_compress_frame(data[f * 65536:][:65536].tobytes(), 0, False), f
