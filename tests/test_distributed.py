"""Multi-rank sharding + all-gatherv reassembly on CPU (gloo, world_size 2
and 4).  Each rank's "decoded slab" is the generator's bytes for its frames
(the GPU decode itself is covered by tests/test_gpu_parity.py); the test
checks that the shard plan and the grouped-broadcast all-gatherv rebuild the
exact contiguous range on every rank, for both partitions."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, mode, frame_sizes, result_q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from libzseek_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        d_off = np.concatenate([[0], np.cumsum(frame_sizes)]).astype(np.uint64)
        total = int(d_off[-1])
        full = (np.arange(total, dtype=np.uint64) * 2654435761 % 251).astype(np.uint8)
        shards = shard.plan(d_off, world, mode)
        mine = shards[rank]
        slab = np.concatenate([full[int(d_off[i]): int(d_off[i + 1])] for i in mine.frames]) \
            if len(mine.frames) else np.zeros(0, np.uint8)
        assert slab.size == mine.out_bytes
        counts = [s.out_bytes for s in shards]
        got = shard.all_gatherv(dist, torch.from_numpy(slab), counts)
        if mode == "round_robin":
            got = shard.to_frame_order(got, shards, d_off)
        result_q.put((rank, bool(np.array_equal(got.numpy(), full))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("mode", ["contiguous", "round_robin"])
@pytest.mark.parametrize("frames", ["uniform", "ragged"])
def test_shard_and_reassemble(world, mode, frames):
    if frames == "uniform":
        sizes = [4096] * 24
    else:
        rng = np.random.default_rng(world)
        sizes = list(rng.integers(1, 9000, 23))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, sizes, q))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def test_plan_covers_every_frame_once():
    from libzseek_amd import shard
    d_off = np.concatenate([[0], np.cumsum(np.full(1000, 65536))]).astype(np.uint64)
    for world in (1, 2, 3, 8):
        for mode in ("contiguous", "round_robin"):
            shards = shard.plan(d_off, world, mode)
            allf = np.sort(np.concatenate([s.frames for s in shards]))
            assert (allf == np.arange(1000)).all()
            assert sum(s.out_bytes for s in shards) == 1000 * 65536


@pytest.mark.parametrize("partition", ["contiguous", "round_robin"])
def test_bench_spawns_ranks_harness(partition):
    """`python bench.py --gpus 2` with no torchrun environment starts two rank
    processes itself (torch.distributed.run child; gloo rehearsal, no GPU),
    builds each rank's shard of a fixed total from replicated frames, gathers
    the full range on every rank and prints one JSON line with n_gpus 2 —
    the code path the driver's multi-GPU run takes (config 4), minus the
    decode."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2",
                        "--harness-check", "--total-size", "8M", "--size", "4M", "--steps", "2",
                        "--warmup", "1", "--partition", partition],
                       capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["decoded_bytes_total"] == 8 << 20
    assert d["config"]["frames_per_gpu"] == 64
    assert d["verified_bit_exact"] is True
    assert d["reassembly"]["full_range_matches_generator"] is True
    assert (d["reassembly"]["permute_s"] is not None) == (partition == "round_robin")


@pytest.mark.parametrize("chunk", [1, 5000, 1 << 28])
def test_to_frame_order_chunked(chunk):
    """Ragged round-robin permute in bounded groups (the byte index is built
    per group of ~chunk bytes): same result for every group size, including
    groups of one frame."""
    from libzseek_amd import shard
    rng = np.random.default_rng(5)
    sizes = rng.integers(1, 9000, 37)
    d_off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.uint64)
    full = (np.arange(int(d_off[-1]), dtype=np.uint64) * 2654435761 % 251).astype(np.uint8)
    for world in (2, 3):
        shards = shard.plan(d_off, world, "round_robin")
        gathered = np.concatenate([full[int(d_off[i]): int(d_off[i + 1])]
                                   for s in shards for i in s.frames])
        got = shard.to_frame_order(torch.from_numpy(gathered), shards, d_off, chunk_bytes=chunk)
        assert np.array_equal(got.numpy(), full)
