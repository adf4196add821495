"""Where does a decoder variant's output differ from the input?  Per frame:
first differing offset, how many bytes differ, and the bytes around it.

    python scripts/vdiff.py --variant 75 --size 8388608
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", type=int, required=True)
    p.add_argument("--size", type=int, default=8 << 20)
    p.add_argument("--frame", type=int, default=64 << 10)
    p.add_argument("--show", type=int, default=6)
    args = p.parse_args()
    import torch

    import libzseek_amd as z
    L = z.lib()
    L.zsk_dev_lz4_decode_variant.restype = C.c_int
    L.zsk_dev_lz4_decode_variant.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda", 0)
    data = z.synth_buffer(args.size)
    img = z.lz4_seekable(data, args.frame)
    c_off, d_off = z.seek_table_of(img)
    n = len(c_off) - 1
    b = z.frame_batch(c_off, d_off, 0, n)
    comp = torch.empty(b.comp_end + 256, dtype=torch.uint8, device=dev)
    comp[: b.comp_end].copy_(torch.from_numpy(img[: b.comp_end]))
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    out = torch.zeros(b.out_bytes, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    rc = L.zsk_dev_lz4_decode_variant(args.variant, desc.data_ptr(), n, comp.data_ptr(),
                                      out.data_ptr(), status.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert rc == 0
    got = out.cpu().numpy()
    st = status.cpu().numpy()
    print(f"frames {n}, status != 0: {int((st != 0).sum())}")
    bad = 0
    for f in range(n):
        a, e = int(d_off[f]), int(d_off[f + 1])
        diff = np.nonzero(got[a:e] != data[a:e])[0]
        if len(diff) == 0:
            continue
        bad += 1
        if bad <= args.show:
            i = int(diff[0])
            print(f"frame {f}: {len(diff)} bytes differ, first at {i} (status {st[f]})")
            print("  want", data[a + max(0, i - 8): a + i + 24].tobytes().hex())
            print("  got ", got[a + max(0, i - 8): a + i + 24].tobytes().hex())
    print(f"{bad} of {n} frames differ")


if __name__ == "__main__":
    main()
