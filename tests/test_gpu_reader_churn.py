"""Reader open / read / close churn (regression for round 3's host heap
corruption): the zstd writer round trip and cached single-frame reads beside
the compiled reference, 30 cycles in one process.  Before HIP streams and
events were recycled instead of destroyed, this sequence
corrupted the host heap within 2-24 cycles (a later free() hung or faulted);
scripts/hang_probe.py is the long form."""
import pytest

from conftest import golden_file

pytestmark = pytest.mark.gpu

SEQ = [0, 65536, 0, 131072, 200000, 0, 70000, 300000, 5, 400000]


def test_reader_churn_beside_reference(gpu, zs, ref):
    img = golden_file("zstd_64k_direct")
    data = bytes(zs.synth_buffer(1 << 20))
    for cycle in range(30):
        w = zs.Writer(zs.ZSEEK_ZSTD, 65536, nb_workers=1)
        for s in range(0, len(data), 65536):
            w.write(data[s: s + 65536])
        with zs.Reader(w.close(), 0) as r:
            assert r.read_all(len(data), 0) == data, cycle
        for cap in (1, 2, 3):
            ours = zs.Reader(img, cap)
            theirs = ref.open(img, cap)
            for off in SEQ:
                a = ours.pread(100, off)
                rb, b = theirs.pread(100, off)
                assert a == b, (cycle, cap, off)
            assert ours.stats()["cached_frames"] == theirs.stats()[1]["cached_frames"]
            ours.close()
            theirs.close()


def test_lz4_reader_churn(gpu, zs):
    """LZ4 readers (split and wave decoders) opened and closed in a loop, two
    alive at a time."""
    data = zs.synth_buffer(2 << 20)
    img = bytes(zs.lz4_seekable(data, 65536))
    keep = None
    for cycle in range(40):
        r = zs.Reader(img, cycle % 3)
        assert r.pread(4096, 65536 * (cycle % 30) + 17) == bytes(data[65536 * (cycle % 30) + 17:][:4096])
        if cycle % 4 == 0:
            assert r.read_all(len(data), 0) == bytes(data)
        if keep is not None:
            keep.close()
        keep = r
    keep.close()
