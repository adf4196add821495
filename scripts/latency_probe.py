"""Single-frame read latency probe: 4 KiB zseek_pread requests at random
offsets of a 64 KiB-frame (third argument: frame bytes) LZ4 (or, with a second argument `zstd`, zstd)
image (cache off), timed per request in C
(tools zsk_tool_latency).  Run under `rocprofv3 --kernel-trace --stats` to
see where a request's time goes."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libzseek_amd as z  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
codec = sys.argv[2] if len(sys.argv) > 2 else "lz4"
frame = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
data = z.synth_buffer(256 << 20)
img = z.zstd_seekable(data, frame) if codec == "zstd" else z.lz4_seekable(data, frame)
T, L = z.tools(), z.lib()
fn = [C.cast(f, C.c_void_p) for f in (L.zseek_reader_open_full, L.zseek_pread, L.zseek_reader_close)]
err = C.create_string_buffer(80)
r = T.zsk_tool_open_mem(fn[0], img.ctypes.data, img.size, 0, err)
rng = np.random.default_rng(1)
offs = rng.integers(0, data.size - 4096, n).astype(np.uint64)
ns = np.zeros(n, np.uint64)
buf = np.empty(4096, np.uint8)
failed = C.c_size_t(0)
assert T.zsk_tool_latency(fn[1], r, offs.ctypes.data, n, 4096, buf.ctypes.data, ns.ctypes.data,
                          C.byref(failed)) == 0
us = ns[20:].astype(np.float64) / 1e3
print(f"{codec} 4 KiB reads: p50 {np.percentile(us, 50):.1f} us  p99 {np.percentile(us, 99):.1f} us  "
      f"mean {us.mean():.1f} us over {len(us)}")
T.zsk_tool_close_mem(fn[2], r)
