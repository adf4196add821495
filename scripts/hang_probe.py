"""Host-hang probe (GPU box, one process): test_gpu_zstd's writer round trip
and cache-LRU sequence (ours beside the compiled reference) in a loop, one
line per iteration; a C-level watchdog dumps every thread's Python stack
every 20 s (it needs no GIL).  mode: both | ours | ref | cache | readall
(cache: our cached single-frame reads only; readall: writer + full reads)."""
import faulthandler
import sys
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
faulthandler.dump_traceback_later(20, repeat=True)
from conftest import golden_file  # noqa: E402
from libzseek_amd import zseek as zs  # noqa: E402
from oracle.oracle import RefZseek  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "both"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
zs.lib()
zs.tools().zsk_tool_install_backtrace()
ref = RefZseek() if mode in ("both", "ref") else None
img = golden_file("zstd_64k_direct")
data = bytes(zs.synth_buffer(1 << 20))
seq = [0, 65536, 0, 131072, 200000, 0, 70000, 300000, 5, 400000]
for it in range(iters):
    if mode in ("both", "ours", "readall"):
        w = zs.Writer(zs.ZSEEK_ZSTD, 65536, nb_workers=1)
        for s in range(0, len(data), 65536):
            w.write(data[s: s + 65536])
        wimg = w.close()
        with zs.Reader(wimg, 0) as r:
            assert r.read_all(len(data), 0) == data
    for cap in (1, 2, 3):
        if mode == "readall":
            break
        ours = zs.Reader(img, cap) if mode in ("both", "ours", "cache") else None
        theirs = ref.open(img, cap) if ref else None
        for off in seq:
            a = ours.pread(100, off) if ours else None
            if theirs:
                rb, b = theirs.pread(100, off)
                if ours:
                    assert a == b
        if ours:
            ours.close()
        if theirs:
            theirs.close()
    print("iter", it, flush=True)
print("done", mode, iters, flush=True)
