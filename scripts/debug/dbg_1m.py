import json, os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import torch
import libzseek_amd.zseek as zs
from conftest import golden_file
g = json.load(open("tests/golden/golden.json"))
rec = g["corrupt"]["1m_block4_offset0"]
base = bytearray(golden_file("lz4_1m_direct"))
for at, v in rec["mutations"]:
    base[at] = v
img = bytes(base)
for cache in (1, 0):
    with zs.Reader(img, cache) as r:
        out = np.empty(4096, np.uint8)
        ret = r.pread_raw(out.ctypes.data, 4096, 1 << 20)
        print("cache", cache, "ret", ret, "err", r.error, r.gpu_stats())
good = golden_file("lz4_1m_direct")
for cache in (1, 0):
    with zs.Reader(good, cache) as r:
        out = np.empty(4096, np.uint8)
        ret = r.pread_raw(out.ctypes.data, 4096, 1 << 20)
        print("good cache", cache, "ret", ret, "err", r.error)
arr = np.frombuffer(img, np.uint8)
c_off, d_off = zs.seek_table_of(arr)
for f in range(len(c_off) - 1):
    b = zs.frame_batch(c_off, d_off, f, f + 1)
    for eng in [None, "wave", "lean", "scan", "chunk"]:
        dev = torch.device("cuda", 0)
        desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
        comp = torch.zeros(b.comp_end - b.comp_begin + 256, dtype=torch.uint8, device=dev)
        comp[: b.comp_end - b.comp_begin].copy_(torch.from_numpy(arr[b.comp_begin: b.comp_end].copy()))
        out = torch.zeros(b.out_bytes, dtype=torch.uint8, device=dev)
        st = torch.full((1,), -1, dtype=torch.int32, device=dev)
        zs.decode_frames(desc, comp, out, st, engine=eng)
        torch.cuda.synchronize()
        print("frame", f, eng, zs.status_string(int(st[0])), hex(int(st[0])))
