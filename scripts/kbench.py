"""Kernel A/B harness: time launch variants of the LZ4 decoder on one input,
interleaved in one process (rule: perf deltas from interleaved rounds).

Uses the tuning build libzseek_amd/lib/libzseek_tune.so (`make -C
libzseek_amd/csrc tune`; variants listed in csrc/tuning.hip), never the
product library.

    python scripts/kbench.py --size 4294967296 --variants 0,1,2 --rounds 5
"""
from __future__ import annotations

import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--size", type=int, default=4 << 30)
    p.add_argument("--frame", type=int, default=64 << 10)
    p.add_argument("--variants", default="0")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--input", default="synth", choices=["synth", "text", "zeros"])
    args = p.parse_args()
    import torch

    import libzseek_amd as z
    L = C.CDLL(os.path.join(ROOT, "libzseek_amd", "lib", "libzseek_tune.so"))
    L.zsk_dev_lz4_decode_variant.restype = C.c_int
    L.zsk_dev_lz4_decode_variant.argtypes = [C.c_int, C.c_void_p, C.c_uint32, C.c_void_p,
                                             C.c_void_p, C.c_void_p, C.c_void_p]
    dev = torch.device("cuda", 0)
    t0 = time.time()
    if args.input == "synth":
        data = z.synth_buffer(args.size)
    elif args.input == "zeros":
        data = np.zeros(args.size, np.uint8)
    else:
        rng = np.random.default_rng(5)
        words = [bytes(rng.integers(97, 123, int(rng.integers(2, 10)), dtype=np.uint8))
                 for _ in range(2000)]
        blob = b" ".join(words[i] for i in rng.integers(0, 2000, 200000))
        data = np.frombuffer((blob * (args.size // len(blob) + 1))[: args.size], np.uint8).copy()
    img = z.lz4_seekable(data, args.frame)
    c_off, d_off = z.seek_table_of(img)
    n = len(c_off) - 1
    b = z.frame_batch(c_off, d_off, 0, n)
    comp = torch.empty(b.comp_end + 256, dtype=torch.uint8, device=dev)
    comp[: b.comp_end].copy_(torch.from_numpy(img[: b.comp_end]))
    desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    out = torch.empty(b.out_bytes, dtype=torch.uint8, device=dev)
    status = torch.empty(n, dtype=torch.int32, device=dev)
    ref = torch.from_numpy(data).to(dev)
    alg = b.comp_end + b.out_bytes
    print(f"input {args.input} {args.size >> 20} MiB, {n} frames, comp {b.comp_end / 1e9:.3f} GB "
          f"({time.time() - t0:.1f}s)", flush=True)
    stream = torch.cuda.current_stream()
    variants = [int(v, 0) for v in args.variants.split(",")]
    res = {v: [] for v in variants}

    def launch(v):
        rc = L.zsk_dev_lz4_decode_variant(v, desc.data_ptr(), n, comp.data_ptr(),
                                          out.data_ptr(), status.data_ptr(), stream.cuda_stream)
        assert rc == 0, f"variant {v} launch failed"

    # stage subsets and diagnostic builds: timing only, output not complete
    diag = set(range(10, 16)) | {20} | set(range(0x100, 0x400)) | set(range(0x800, 0x900))

    for v in variants:   # correctness once per variant
        out.zero_()
        launch(v)
        torch.cuda.synchronize()
        ok = int((status != 0).sum()) == 0 and torch.equal(out, ref)
        print(f"variant {v}: {'bit-exact' if ok else 'MISMATCH' + (' (diagnostic build)' if v in diag else '')}",
              flush=True)
        if not ok and v not in diag:
            raise SystemExit(f"variant {v} is not bit-exact")
    for _ in range(args.rounds):
        for v in variants:
            launch(v)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                launch(v)
            e1.record(stream)
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / args.reps)
    for v in variants:
        ms = sorted(res[v])
        med = ms[len(ms) // 2]
        print(f"variant {v}: median {med:.3f} ms  min {ms[0]:.3f}  decoded {args.size / med / 1e6:.1f} GB/s"
              f"  alg {alg / med / 1e6:.1f} GB/s ({alg / med / 1e6 / 8000 * 100:.2f}% of 8 TB/s)",
              flush=True)


if __name__ == "__main__":
    main()
