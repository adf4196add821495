"""Block route of the two-phase LZ4 decoder (lz4_split.hip block plan,
lz4_lean.hip block lanes, lz4_chunk.hip accept / re-parse, seq_exec.hip job
segments): one parse lane per LZ4 block of each multi-block frame at the
output offset the block starts at when every earlier block is full-size.

Frames built here by splicing LZ4F blocks — reordered independent blocks,
short stored blocks before the last (the speculation fails and the chunk
parse takes the frame), corrupt blocks mid-frame, trailing bytes, more blocks
than the route takes, seek-table sizes that disagree — go through the forced
route (ZSK_DECODER_BLOCK: any batch, any job count) -- and the one-frame
route's big-frame path (ZSK_DECODER_ONE: its jobs of <= 64 KiB blocks parsed a
workgroup each, lz4_job_parse_kernel, and executed through the sliding
window, seq_exec_big_kernel) -- and must give the CPU restatement's status
and bytes (oracle/lz4_oracle.c decode_frame, liblz4
1.9.3 LZ4F_decompress semantics) and the wave kernel's status codes."""
import numpy as np
import pytest
import xxhash

from conftest import golden_file

pytestmark = pytest.mark.gpu


def _frames_of(zs, img):
    c_off, d_off = zs.seek_table_of(img)
    return [bytes(img[int(c_off[i]): int(c_off[i + 1])]) for i in range(len(c_off) - 1)], \
        [int(d_off[i + 1] - d_off[i]) for i in range(len(d_off) - 1)]


def _split(frame: bytes):
    """-> (FLG, BD, header length, [(block header u32, payload)])"""
    flg, bd = frame[4], frame[5]
    hdr = 7 + (8 if flg & 8 else 0) + (4 if flg & 1 else 0)
    p, blocks = hdr, []
    while True:
        h = int.from_bytes(frame[p: p + 4], "little")
        p += 4
        if h == 0:
            break
        n = h & 0x7FFFFFFF
        blocks.append((h, frame[p: p + n]))
        p += n + (4 if flg & 0x10 else 0)
    return flg, bd, hdr, blocks


def _frame(blocks, flg=0x60, bd=0x40, content_size=None, dict_id=None, tail=b""):
    """An LZ4F frame (magic, descriptor, header checksum) of the given blocks:
    bytes payloads are stored blocks, (h, payload) pairs are copied."""
    if content_size is not None:
        flg |= 8
    if dict_id is not None:
        flg |= 1
    desc = bytes([flg, bd])
    if content_size is not None:
        desc += int(content_size).to_bytes(8, "little")
    if dict_id is not None:
        desc += int(dict_id).to_bytes(4, "little")
    out = bytearray(b"\x04\x22\x4d\x18" + desc + bytes([(xxhash.xxh32(desc).intdigest() >> 8) & 0xFF]))
    for b in blocks:
        if isinstance(b, (bytes, bytearray)):
            out += (len(b) | 0x80000000).to_bytes(4, "little") + bytes(b)
        else:
            out += b[0].to_bytes(4, "little") + b[1]
    out += b"\0\0\0\0" + tail
    return bytes(out)


def _decode(zs, gpu, frames, dsizes, engine):
    import torch
    n = len(frames)
    c = np.cumsum([0] + [len(f) for f in frames])
    d = np.cumsum([0] + list(dsizes))
    desc = np.zeros(n, dtype=[("c_off", "<u8"), ("d_off", "<u8"), ("c_size", "<u4"), ("d_size", "<u4")])
    desc["c_off"], desc["d_off"] = c[:-1], d[:-1]
    desc["c_size"], desc["d_size"] = np.diff(c), np.asarray(dsizes)
    td = torch.from_numpy(desc.view(np.uint8).copy()).to(gpu)
    comp = torch.zeros(int(c[-1]) + 256, dtype=torch.uint8, device=gpu)
    comp[: int(c[-1])].copy_(torch.from_numpy(np.frombuffer(b"".join(frames), np.uint8).copy()))
    out = torch.zeros(max(int(d[-1]), 1), dtype=torch.uint8, device=gpu)
    status = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    zs.decode_frames(td, comp, out, status, engine=engine)
    torch.cuda.synchronize()
    o = out.cpu().numpy().tobytes()
    return [o[int(d[i]): int(d[i + 1])] for i in range(n)], status.cpu().tolist()


def _check(zs, oracle, gpu, frames, dsizes, engine="block"):
    """block route == oracle (status, bytes of OK frames) and == wave statuses"""
    got, st = _decode(zs, gpu, frames, dsizes, engine)
    _, st_w = _decode(zs, gpu, frames, dsizes, "wave")
    assert st == st_w
    for i, (f, ds) in enumerate(zip(frames, dsizes)):
        ost, obytes, _, _ = oracle.decode_frame(f, ds)
        if ost == 0 and len(obytes) == ds:
            assert st[i] == 0, (i, zs.status_string(st[i]))
            assert got[i] == obytes, i
        else:
            assert st[i] != 0, i
    return st


@pytest.fixture(scope="module")
def indep(zs):
    """1 MiB frames with independent 64 KiB blocks (block route eligible)"""
    data = zs.synth_buffer(4 << 20)
    img = zs.lz4_seekable_ex(data, 1 << 20, independent=True)
    frames, _ = _frames_of(zs, img)
    return [_split(f)[3] for f in frames]


@pytest.mark.parametrize("engine", ["block", "one"])
def test_block_route_reordered_independent_blocks(gpu, zs, oracle, indep, engine):
    """Independent blocks reordered and mixed across frames: accepted by the
    route (every block but the last full-size), bytes == oracle."""
    b = indep
    frames = [_frame([b[0][3], b[1][0], b[2][7], b[3][15]], flg=0x60 | 0x20),
              _frame([b[1][5], b[0][0]], flg=0x60 | 0x20),
              _frame([b[2][i] for i in range(16)][::-1][1:] + [b[2][15]], flg=0x60 | 0x20)]
    dsizes = [len(oracle.decode_frame(f, 1 << 24)[1]) for f in frames]
    st = _check(zs, oracle, gpu, frames, dsizes, engine)
    assert st == [0, 0, 0]


@pytest.mark.parametrize("engine", ["block", "one"])
def test_block_route_short_blocks_reparsed(gpu, zs, oracle, indep, engine):
    """A stored block shorter than the maximum before the last: the
    speculative offsets are wrong for the blocks after it; the chunk parse
    re-parses the frame (bytes == oracle).  Also all-stored frames (accepted),
    a final short stored block (accepted) and an empty stored block."""
    b = indep
    rng = np.random.default_rng(5)
    raw = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in (1000, 65536, 65536, 10, 300)]
    frames = [_frame([raw[0], b[0][1], b[0][2]], flg=0x60 | 0x20),
              _frame([b[1][4], raw[3], b[1][5]], flg=0x60 | 0x20),
              _frame([raw[1], raw[2], raw[4]]),
              _frame([b[2][0], b[2][1], raw[3]], flg=0x60 | 0x20)]
    dsizes = [len(oracle.decode_frame(f, 1 << 24)[1]) for f in frames]
    st = _check(zs, oracle, gpu, frames, dsizes, engine)
    assert st == [0, 0, 0, 0]


@pytest.mark.parametrize("engine", ["block", "one"])
def test_block_route_corrupt_and_odd_frames(gpu, zs, oracle, indep, engine):
    """Failures inside the route's frames give the exact statuses: a corrupt
    block mid-frame, a block size over the maximum, a zero-size compressed
    block, trailing bytes after the end mark, a truncated frame, a seek-table
    dSize larger and smaller than the frame's, 65 blocks (more than the route
    takes), a content size that disagrees, dictID and content-size frames."""
    b = indep
    blocks = list(b[0])
    bad = bytearray(blocks[5][1])
    bad[len(bad) // 2] ^= 0xFF
    bad[len(bad) // 2 + 1] = 0xF0
    corrupt = blocks[:5] + [(blocks[5][0], bytes(bad))] + blocks[6:]
    full = _frame(blocks, flg=0x60 | 0x20)
    rng = np.random.default_rng(9)
    many = [bytes(rng.integers(0, 4, 65536, dtype=np.uint8)) for _ in range(65)]
    frames = [_frame(corrupt, flg=0x60 | 0x20),
              _frame(blocks[:3] + [(0x7FFFFFF0, b"")], flg=0x60 | 0x20)[:-4],
              _frame(blocks[:2] + [(0, b"")] + blocks[2:4], flg=0x60 | 0x20),
              _frame(blocks[:4], flg=0x60 | 0x20, tail=b"xyz"),
              full[: len(full) - 9],
              full, full,
              _frame(many),
              _frame(blocks[:4], flg=0x60 | 0x20, content_size=4 * 65536 + 1),
              _frame(blocks[:4], flg=0x60 | 0x20, content_size=4 * 65536, dict_id=77)]
    dsizes = [1 << 20, 3 * 65536, 4 * 65536, 4 * 65536, 1 << 20,
              (1 << 20) + 100, (1 << 20) - 100, 65 * 65536, 4 * 65536, 4 * 65536]
    st = _check(zs, oracle, gpu, frames, dsizes, engine)
    # (the corrupt block may still decode: _check holds it to the oracle)
    assert st[-1] == 0 and st[1] != 0 and st[7] == 0


@pytest.mark.parametrize("engine", ["block", "one"])
def test_block_route_linked_and_big_blocks(gpu, zs, oracle, engine):
    """Linked 64 KiB blocks (the reference writer's frames), 256 KiB blocks,
    frames of 64 blocks (the route's maximum) and 65 (the chunk parse), and a
    frame one byte past a block boundary: bytes == the generator."""
    data = zs.synth_buffer((8 << 20) + 1)
    for img in (zs.lz4_seekable(data, 1 << 20), zs.lz4_seekable_ex(data, 1 << 20, bsid=5),
                zs.lz4_seekable(data, 4 << 20), zs.lz4_seekable(data, (4 << 20) + 65536),
                zs.lz4_seekable(data, 65537)):
        frames, dsizes = _frames_of(zs, img)
        got, st = _decode(zs, gpu, frames, dsizes, engine)
        assert all(s == 0 for s in st)
        assert b"".join(got) == data.tobytes()


@pytest.mark.parametrize("engine", ["block", "one"])
@pytest.mark.parametrize("case", ["1m_block4_offset0", "1m_block4_size_huge"])
def test_block_route_reference_corruptions(gpu, zs, golden, case, engine):
    """The reference fixtures' corruptions in block 4 of a 1 MiB frame (a
    zero match offset, which liblz4 decodes and the route hands to the wave
    kernel; a block size over the maximum): the route's statuses == the wave
    kernel's, the frames either decodes equal."""
    rec = golden["corrupt"][case]
    img = bytearray(golden_file(rec["base"]))
    for at, v in rec["mutations"]:
        img[at] = v
    frames, dsizes = _frames_of(zs, np.frombuffer(bytes(img), np.uint8))
    got, st = _decode(zs, gpu, frames, dsizes, engine)
    got_w, st_w = _decode(zs, gpu, frames, dsizes, "wave")
    assert st == st_w
    for i, s in enumerate(st):
        if s == 0:
            assert got[i] == got_w[i], i


def test_block_route_auto_at_scale(gpu, zs):
    """The library's own routing takes the block route for 1,024 frames of
    1 MiB (16,384 jobs, config 3's shape at 1 GiB): decoded == generator."""
    import torch
    data = zs.synth_buffer(1 << 30)
    img = zs.lz4_seekable(data, 1 << 20)
    c_off, d_off = zs.seek_table_of(img)
    n = len(c_off) - 1
    bt = zs.frame_batch(c_off, d_off, 0, n)
    desc = torch.from_numpy(bt.desc.view(np.uint8).copy()).to(gpu)
    comp = torch.zeros(bt.comp_end + 256, dtype=torch.uint8, device=gpu)
    comp[: bt.comp_end].copy_(torch.from_numpy(img[: bt.comp_end].copy()))
    out = torch.zeros(bt.out_bytes, dtype=torch.uint8, device=gpu)
    status = torch.full((n,), -1, dtype=torch.int32, device=gpu)
    zs.decode_frames(desc, comp, out, status)
    torch.cuda.synchronize()
    assert int((status != 0).sum()) == 0
    assert torch.equal(out, torch.from_numpy(data).to(gpu))


_FIRST_CALL = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1])
import libzseek_amd as z
data = z.synth_buffer(64 << 20)
img = z.lz4_seekable(data, 1 << 20)
c_off, d_off = z.seek_table_of(img)
b = z.frame_batch(c_off, d_off, 0, len(c_off) - 1)
dev = torch.device("cuda", 0)
desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
comp = torch.zeros(b.comp_end + 256, dtype=torch.uint8, device=dev)
comp[: b.comp_end].copy_(torch.from_numpy(img[: b.comp_end].copy()))
out = torch.empty(b.out_bytes, dtype=torch.uint8, device=dev)
status = torch.full((len(b.desc),), -1, dtype=torch.int32, device=dev)
z.kernel_timing(True)
z.decode_frames(desc, comp, out, status)      # this process's FIRST device-API call
torch.cuda.synchronize()
n, ms = z.kernel_times()
z.kernel_timing(False)
assert int((status != 0).sum()) == 0
assert out.cpu().numpy().tobytes() == data.tobytes()
print("STAGES", ms)
assert ms["hand-off"] < 0.25 * ms["execute"], ms
"""


def test_device_api_first_call_big_frames(gpu):
    """The device API's first call in a process on 1 MiB frames sizes its
    item scratch from the compressed span, so no frame is handed to the
    (6x slower) wave kernel: the hand-off stage stays an empty launch."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", _FIRST_CALL, root], capture_output=True, text=True,
                       timeout=110, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
