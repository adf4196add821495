"""Single-frame read cases for tests/test_gpu_env_switches.py: run in a fresh
process (the library reads its environment switches once, at first use), it
prints one JSON object -- per case the SHA-256 of the bytes a caller's read
loop gets and the error text it ends with.  Test infrastructure only."""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def cases():
    g = os.path.join(ROOT, "tests", "golden")
    out = {}
    for name in ("lz4_64k_direct", "zstd_64k_direct", "lz4_1m_direct"):
        img = np.frombuffer(open(os.path.join(g, name + ".zs"), "rb").read(), np.uint8).copy()
        out[name] = img
        bad = img.copy()
        bad[len(img) // 3] ^= 0x5A   # inside a middle frame's compressed bytes
        out[name + "_corrupt"] = bad
    return out


def run():
    import libzseek_amd.zseek as zs
    res = {}
    for name, img in cases().items():
        for cache in (0, 1):
            with zs.Reader(img, cache) as r:
                total = int(r.frames()[1][-1])
                rng = np.random.default_rng(7)
                offs = [0, total // 3, total // 2 + 123, max(total - 4096, 0)] + \
                    [int(x) for x in rng.integers(0, max(total - 4096, 1), 12)]
                for off in offs:
                    got, err = b"", None
                    while len(got) < 4096:
                        try:
                            b = r.pread(4096 - len(got), off + len(got))
                        except zs.ZseekError as e:
                            err = str(e)
                            break
                        if not b:
                            break
                        got += b
                    res[f"{name}/c{cache}/{off}"] = [hashlib.sha256(got).hexdigest(), len(got), err]
    return res


if __name__ == "__main__":
    print(json.dumps(run()))
