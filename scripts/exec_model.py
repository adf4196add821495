"""CPU model of the execute's batches on config 2's LZ4 stream (DESIGN.md §3,
round 6): compresses synthetic 64 KiB frames with liblz4 (the tools library),
walks their sequences and reports, per batch policy, the pending matches and
dependency rounds (exact rule of seq_exec's readiness search, and the
frontier rule), and for round 0 the descriptor-loop steps and entries per
batch at 16 / 32 / 64 / 128-byte entry granularity.

    python scripts/exec_model.py [frames]
"""
from __future__ import annotations

import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import libzseek_amd as z  # noqa: E402

N = 64 << 10


def sequences(img, c_off, fr):
    """(literal length, match length, offset) of every sequence of frame fr"""
    b = img[c_off[fr]:c_off[fr + 1]].tobytes()
    p = 7 + (8 if b[4] & 8 else 0)
    out = []
    while True:
        bs = int.from_bytes(b[p:p + 4], "little")
        p += 4
        if bs == 0:
            break
        if bs & 0x80000000:
            out.append((bs & 0x7FFFFFFF, 0, 0))
            p += bs & 0x7FFFFFFF
            continue
        e = p + bs
        while p < e:
            t = b[p]
            p += 1
            L = t >> 4
            if L == 15:
                while True:
                    x = b[p]
                    p += 1
                    L += x
                    if x != 255:
                        break
            p += L
            if p >= e:
                out.append((L, 0, 0))
                break
            off = b[p] | b[p + 1] << 8
            p += 2
            M = t & 15
            if M == 15:
                while True:
                    x = b[p]
                    p += 1
                    M += x
                    if x != 255:
                        break
            out.append((L, M + 4, off))
    return out


def batches(fr, outb, ns):
    """seq_exec's cut: up to ns sequences whose output fits outb bytes"""
    i = pos = 0
    while i < len(fr):
        j = i
        tot = 0
        while j < len(fr) and j - i < ns and tot + fr[j][0] + fr[j][1] <= outb:
            tot += fr[j][0] + fr[j][1]
            j += 1
        if j == i:
            j = i + 1
        yield i, j, pos
        pos += sum(a + b for a, b, _ in fr[i:j])
        i = j


def rounds(S, outb, ns):
    nb = seqs = pend = rx = rf = 0
    for fr in S:
        for i, j, bstart in batches(fr, outb, ns):
            ms, p = [], bstart
            for L, M, O in fr[i:j]:
                mb = p + L
                if M:
                    need = mb if O < M else mb - O + M
                    if need > bstart:
                        ms.append((mb, mb + M, mb - O, need))
                p = mb + M
            pend += len(ms)
            todo, r = list(range(len(ms))), 0
            while todo:
                ready = [a for a in todo if not any(b < a and ms[b][1] > ms[a][2] and ms[b][0] < ms[a][3]
                                                    for b in todo)]
                todo = [a for a in todo if a not in ready]
                r += 1
            rx += r
            todo, r = list(range(len(ms))), 0
            while todo:
                f = ms[todo[0]][0]
                todo = [a for k, a in enumerate(todo) if k and ms[a][3] > f]
                r += 1
            rf += r
            nb += 1
            seqs += j - i
    print(f"OUTB {outb} seqs<={ns}: batches/frame {nb / len(S):.1f}  seqs/batch {seqs / nb:.1f}  "
          f"pending/batch {pend / nb:.2f}  rounds exact {rx / nb:.2f}  frontier {rf / nb:.2f}")


def granularity(S, outb=3072, ns=64):
    def ceil(a, b):
        return -(-a // b)
    res = {g: [0, 0, 0] for g in (16, 32, 64, 128)}
    nb = 0
    for fr in S:
        for i, j, bstart in batches(fr, outb, ns):
            runs, p = [], bstart
            for L, M, O in fr[i:j]:
                mb = p + L
                early = M and mb - O + M <= bstart and O >= M
                runs.append((L, M if early else 0))
                p = mb + M
            for g, r in res.items():
                r[0] += max(max(ceil(L, g) if L >= 16 else 0, ceil(M, g) if M >= 16 else 0) for L, M in runs)
                tot = sum((ceil(L, g) if L >= 16 else 0) + (ceil(M, g) if M >= 16 else 0) for L, M in runs)
                r[1] += tot
                r[2] += ceil(tot * g // 16, 64)
            nb += 1
    for g, r in res.items():
        print(f"entries of {g} B: descriptor-loop steps/batch {r[0] / nb:.2f}  entries/batch {r[1] / nb:.1f}  "
              f"deal steps (64 lanes) {r[2] / nb:.2f}")


def main():
    nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    data = z.synth_buffer(nfr * N)
    img = z.lz4_seekable(data, N)
    c_off, _ = z.seek_table_of(img)
    S = [sequences(img, c_off, f) for f in range(1, nfr)]   # frame 0 has no history
    A = np.array([x for s in S for x in s])
    m = A[A[:, 1] > 0]
    print(f"{len(S)} frames: {np.mean([len(s) for s in S]):.0f} sequences/frame, literal run mean "
          f"{A[:, 0].mean():.1f} B, match mean {m[:, 1].mean():.1f} B, offset p50/p90/p95 "
          f"{np.percentile(m[:, 2], [50, 90, 95])}")
    for outb, ns in ((3072, 64), (4096, 64), (6144, 128), (2048, 64)):
        rounds(S, outb, ns)
    granularity(S)


if __name__ == "__main__":
    main()
