"""PCIe probe: D2H / H2D bandwidth into pinned, registered and pageable host
memory, and the cost of hipHostRegister -- the bounds of the drop-in
zseek_pread into host memory (bench.py end_to_end)."""
import ctypes as C
import json
import time

import numpy as np
import torch

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
hip.hipDeviceSynchronize.argtypes = []
D2H, H2D = 2, 1
N = 1 << 30
dev = torch.empty(N, dtype=torch.uint8, device="cuda")
dev.fill_(7)
torch.cuda.synchronize()
res = {}


def rate(dst, src, kind, reps=3):
    best = 0.0
    for _ in range(reps):
        t = time.perf_counter()
        assert hip.hipMemcpy(dst, src, N, kind) == 0
        best = max(best, N / (time.perf_counter() - t) / 1e9)
    return round(best, 2)


pin = torch.empty(N, dtype=torch.uint8, pin_memory=True)
res["d2h_pinned_GBps"] = rate(pin.data_ptr(), dev.data_ptr(), D2H)
res["h2d_pinned_GBps"] = rate(dev.data_ptr(), pin.data_ptr(), H2D)
page = np.empty(N, np.uint8)
page[:] = 1
res["d2h_pageable_GBps"] = rate(page.ctypes.data, dev.data_ptr(), D2H)
buf = np.empty(N, np.uint8)
buf[::4096] = 1   # touched
t = time.perf_counter()
assert hip.hipHostRegister(buf.ctypes.data, N, 0) == 0
res["host_register_GBps"] = round(N / (time.perf_counter() - t) / 1e9, 2)
res["d2h_registered_GBps"] = rate(buf.ctypes.data, dev.data_ptr(), D2H)
t = time.perf_counter()
hip.hipHostUnregister(buf.ctypes.data)
res["host_unregister_GBps"] = round(N / (time.perf_counter() - t) / 1e9, 2)
t = time.perf_counter()
np.copyto(page, pin.numpy())
res["host_memcpy_1thread_GBps"] = round(N / (time.perf_counter() - t) / 1e9, 2)
print(json.dumps(res))
