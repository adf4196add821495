"""End-to-end read probe: zseek_pread of a whole synthetic image into host
memory (the bench line's end_to_end, smaller), at io_threads 1 and 8, best of
three.  Argument: GiB (default 1), frame bytes (default 64 KiB).  A/B runs
set the library's env switches around it."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libzseek_amd as z  # noqa: E402

size = int(float(sys.argv[1]) * (1 << 30)) if len(sys.argv) > 1 else 1 << 30
frame = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
data = z.synth_buffer(size)
img = z.lz4_seekable(data, frame)
T, L = z.tools(), z.lib()
buf = np.empty(size, np.uint8)
out = {}
for io in (1, 8):
    err = C.create_string_buffer(80)
    r = T.zsk_tool_open_mem(C.cast(L.zseek_reader_open_full, C.c_void_p), img.ctypes.data, img.size, 0, err)
    L.zsk_reader_set_io_threads(r, io)
    got = C.c_size_t(0)
    best = 0.0
    for _ in range(3):
        secs = T.zsk_tool_read_all(C.cast(L.zseek_pread, C.c_void_p), r, buf.ctypes.data, size, C.byref(got))
        best = max(best, got.value / secs / 1e9)
    T.zsk_tool_close_mem(C.cast(L.zseek_reader_close, C.c_void_p), r)
    out[f"io{io}"] = round(best, 2)
assert np.array_equal(buf[:1 << 20], data[:1 << 20])
print("e2e GB/s", out, os.environ.get("ZSEEK_DONE_FLAG", ""))
