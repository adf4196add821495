"""Frame sharding across GPUs and the RCCL reassembly of decoded slabs
(BASELINE config 4).

Frames are independent, so a decoded range shards with no data-path
collective: rank r decodes its own frames.  When every rank needs the whole
contiguous range, the decoded slabs are reassembled with an all-gatherv —
RCCL has no variable-count all-gather, so it is a group of broadcasts, one per
source rank (`all_gatherv`).  Two partitions:

  contiguous   rank r takes frames [r*n/N, (r+1)*n/N): its slab IS a
               contiguous piece of the output, no permutation after the gather
  round_robin  frame i -> rank i % N (config 4's wording); the gathered
               rank-major slabs are permuted back to frame order
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Shard:
    rank: int
    frames: np.ndarray       # frame indices owned by this rank, ascending
    out_bytes: int           # decoded bytes of the shard


def plan(d_off: np.ndarray, world: int, mode: str = "contiguous") -> list[Shard]:
    """Split the frames of a seek table (d_off = n+1 prefix sums) over ranks."""
    n = len(d_off) - 1
    sizes = np.diff(d_off.astype(np.int64))
    shards = []
    for r in range(world):
        if mode == "contiguous":
            f0, f1 = r * n // world, (r + 1) * n // world
            idx = np.arange(f0, f1)
        elif mode == "round_robin":
            idx = np.arange(r, n, world)
        else:
            raise ValueError(mode)
        shards.append(Shard(r, idx, int(sizes[idx].sum())))
    return shards


def all_gatherv(dist, slab, counts: list[int], out=None, group=None):
    """Every rank receives every rank's slab, concatenated rank-major.

    `slab` is this rank's 1-D uint8 tensor (len == counts[rank]); `out` (len
    == sum(counts)) receives the result.  Equal slabs: the collective
    all-gather (RCCL's ring over xGMI); ragged slabs: one broadcast per source
    rank issued together (RCCL groups them), so each link carries each slab
    once.
    """
    import torch
    rank = dist.get_rank(group)
    total = sum(counts)
    if out is None:
        out = torch.empty(total, dtype=slab.dtype, device=slab.device)
    if len(set(counts)) == 1 and hasattr(dist, "all_gather_into_tensor"):
        try:
            dist.all_gather_into_tensor(out, slab[: counts[rank]], group=group)
            return out
        except (RuntimeError, NotImplementedError):
            pass   # a backend without it (older gloo): the broadcasts below
    starts = np.concatenate([[0], np.cumsum(counts)])
    out[starts[rank]: starts[rank + 1]].copy_(slab[: counts[rank]])
    reqs = []
    for src in range(len(counts)):
        if counts[src] == 0:
            continue
        view = out[starts[src]: starts[src + 1]]
        reqs.append(dist.broadcast(view, src=src, group=group, async_op=True))
    for q in reqs:
        q.wait()
    return out


def to_frame_order(gathered, shards: list[Shard], d_off: np.ndarray, chunk_bytes: int = 1 << 28):
    """Permute a rank-major gather back to frame order (round_robin plans).

    Uniform frames use one strided view (a device transpose).  Ragged frames
    are scattered in groups of consecutive gathered frames of at most
    ~chunk_bytes: each group's byte index (int64 per byte, built from
    per-frame (source, destination, length) triples with repeat_interleave)
    lives only for that group, so the index memory is bounded by
    ~16 x chunk_bytes whatever the gather's size.
    """
    import torch
    sizes = np.diff(d_off.astype(np.int64))
    n = len(sizes)
    world = len(shards)
    if n and (sizes[:-1] == sizes[0]).all() and n % world == 0 and sizes[-1] == sizes[0]:
        fs = int(sizes[0])
        return gathered.view(world, n // world, fs).transpose(0, 1).reshape(-1)
    order = np.concatenate([s.frames for s in shards]).astype(np.int64)   # gathered frame order
    lens = sizes[order]
    ends = np.cumsum(lens)
    src = np.concatenate([[0], ends[:-1]])                                # offset in gathered
    dst = d_off[:-1].astype(np.int64)[order]                               # offset in frame order
    dev = gathered.device
    out = torch.empty_like(gathered)
    i0 = 0
    while i0 < len(order):
        # frames [i0, i1): at least one, then as many as fit chunk_bytes
        i1 = max(i0 + 1, int(np.searchsorted(ends, src[i0] + chunk_bytes, side="right")))
        a, b = int(src[i0]), int(ends[i1 - 1])
        lens_t = torch.from_numpy(lens[i0:i1]).to(dev)
        base = torch.repeat_interleave(torch.from_numpy(dst[i0:i1] - src[i0:i1]).to(dev), lens_t)
        idx = torch.arange(a, b, device=dev) + base                        # destination of each byte
        out[idx] = gathered[a:b]
        del idx, base
        i0 = i1
    return out
