"""FETCH_SIZE / WRITE_SIZE calibration on the LZ4 execute's own access
pattern (verdict r04 item 3): hand-built LZ4 frames whose sequences make the
execute (seq_exec_kernel) read a KNOWN number of bytes from memory, decoded
through the production device API, so a rocprofv3 --pmc pass relates the
counters to algorithmic bytes for exactly this kernel's loads and stores.

  literal : every sequence = a literal run of 17..63 bytes + an 8-byte match at
            offset 16 (its source is in the batch's stage, never memory):
            memory reads = the literal bytes + the 8-byte items
  match   : every sequence = 5 literal bytes + a 32..64-byte match 8..60 KiB
            back (its source is output written earlier: far enough that the
            frame's recent output in the stage never serves it): memory
            reads = match bytes + items + the literal bytes

(The literal kind's frames take the chunk parse -- 60 KB compressed -- and
the match kind's the scan parse; both execute on seq_exec_kernel, whose
counters are the ones read.)

One distinct frame per kind (64 KiB decoded), replicated 65,536 times (4 GiB
decoded, config 2's geometry), so frames never share cache lines.  Run under
`rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes); then
`python scripts/fetch_calib.py --summarize DIR` prints, per kind, the
counter per launch against the known bytes (round 5; `scripts/gpu.sh pmc` runs such a pass).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FRAME = 65536
NFRAMES = 65536


def block(seqs, last_lits):
    """raw LZ4 block: seqs = [(literal bytes, offset, match length)], then the
    final literals"""
    out = bytearray()

    def length(n):
        while n >= 255:
            out.append(255)
            n -= 255
        out.append(n)

    for lit, off, ml in seqs:
        L, M = len(lit), ml - 4
        out.append((min(L, 15) << 4) | min(M, 15))
        if L >= 15:
            length(L - 15)
        out += lit
        out += off.to_bytes(2, "little")
        if M >= 15:
            length(M - 15)
    L = len(last_lits)
    out.append(min(L, 15) << 4)
    if L >= 15:
        length(L - 15)
    out += last_lits
    return bytes(out)


def make_frame(kind: str, rng) -> tuple[bytes, bytes, dict]:
    """one LZ4F frame (64 KiB decoded, one block) -> (frame, decoded, counts)"""
    import xxhash
    dec = bytearray()
    seqs = []
    lit_bytes = match_bytes = 0
    while True:
        if kind == "literal":
            L, off, M = int(rng.integers(17, 64)), 16, 8
        else:
            # (5 literal bytes: >= 8 compressed bytes per sequence, the
            # parse's item-slot budget, else frames go to the wave kernel)
            L, M = 5, int(rng.integers(32, 65))
            off = int(rng.integers(8192, min(len(dec) + L, 61440) + 1)) if len(dec) > 8192 else 16
            if len(dec) < 16:
                L = 16
        if len(dec) + L + M + 12 + 5 > FRAME:
            break
        lit = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        dec += lit
        for _ in range(M):
            dec.append(dec[-off])
        seqs.append((lit, off, M))
        lit_bytes += L
        match_bytes += M
    last = rng.integers(0, 256, FRAME - len(dec), dtype=np.uint8).tobytes()
    dec += last
    lit_bytes += len(last)
    blk = block(seqs, last)
    flg, bd = 0x60, 0x40   # version 01, independent blocks; 64 KiB blocks
    hc = (xxhash.xxh32(bytes([flg, bd])).intdigest() >> 8) & 0xFF
    frame = (0x184D2204).to_bytes(4, "little") + bytes([flg, bd, hc]) + len(blk).to_bytes(4, "little") + blk + bytes(4)
    return frame, bytes(dec), {"sequences": len(seqs) + 1, "literal_bytes": lit_bytes, "match_bytes": match_bytes}


def run(kinds, launches):
    import torch

    import libzseek_amd as z
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    meta = {}
    for kind in kinds:
        frame, dec, cnt = make_frame(kind, rng)
        c = len(frame)
        comp = torch.zeros(c * NFRAMES + 256, dtype=torch.uint8, device=dev)
        one = torch.frombuffer(bytearray(frame), dtype=torch.uint8).to(dev)
        comp[: c * NFRAMES].view(NFRAMES, c).copy_(one.expand(NFRAMES, c))
        desc = np.zeros(NFRAMES, z.FRAME_DESC_DTYPE)
        desc["c_off"] = np.arange(NFRAMES, dtype=np.uint64) * c
        desc["d_off"] = np.arange(NFRAMES, dtype=np.uint64) * FRAME
        desc["c_size"] = c
        desc["d_size"] = FRAME
        d = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
        out = torch.empty(FRAME * NFRAMES, dtype=torch.uint8, device=dev)
        st = torch.empty(NFRAMES, dtype=torch.int32, device=dev)
        for _ in range(launches):
            z.decode_frames(d, comp, out, st)
        torch.cuda.synchronize()
        ref = torch.frombuffer(bytearray(dec), dtype=torch.uint8).to(dev)
        ok = int((st != 0).sum()) == 0 and bool(torch.equal(out.view(NFRAMES, FRAME)[::4099], ref.expand(16, FRAME)))
        meta[kind] = dict(cnt, frame_bytes=c, frames=NFRAMES, launches=launches, bit_exact=ok,
                          item_bytes=8 * cnt["sequences"])
        print(kind, json.dumps(meta[kind]), flush=True)
        del comp, out, d, st
        torch.cuda.empty_cache()
    return meta


def summarize(root):
    """per kind (dispatch order: literal launches first), seq_exec_kernel's
    FETCH_SIZE / WRITE_SIZE per launch (median) against the known bytes"""
    meta = json.load(open(os.path.join(root, "meta.json")))
    res = {}
    for counter, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        rows = []
        for f in glob.glob(os.path.join(root, sub, "**", "*_counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "seq_exec_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter:
                    rows.append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
        rows.sort()
        vals = [v for _, v in rows]
        at = 0
        for kind, m in meta.items():
            k = m["launches"]
            v = sorted(vals[at: at + k])[k // 2] if len(vals) >= at + k else None
            at += k
            res.setdefault(kind, dict(m))[counter + "_KiB"] = v
    for kind, m in res.items():
        n = m["frames"]
        reads = n * (m["literal_bytes"] + m["item_bytes"] + (m["match_bytes"] if kind == "match" else 0))
        writes = n * FRAME
        fk, wk = m.get("FETCH_SIZE_KiB"), m.get("WRITE_SIZE_KiB")
        m["known_read_bytes"] = reads
        m["known_write_bytes"] = writes
        if fk:
            m["fetch_bytes_raw"] = fk * 1024
            m["read_factor"] = round(reads / (fk * 1024), 3)   # multiply FETCH_SIZE bytes by this
        if wk:
            m["write_factor"] = round(writes / (wk * 1024), 3)
    print(json.dumps(res, indent=1))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=3)
    ap.add_argument("--kinds", default="literal,match")
    ap.add_argument("--meta", default=None, help="write the workload record here")
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    if a.summarize:
        summarize(a.summarize)
        return
    meta = run(a.kinds.split(","), a.launches)
    if a.meta:
        json.dump(meta, open(a.meta, "w"), indent=1)


if __name__ == "__main__":
    main()
