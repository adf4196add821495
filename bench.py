"""bench.py — decoded GB/s of the GPU LZ4 random-access decode path.

Workload (BASELINE.json configs[1] = config 2): the SURVEY §8d synthetic,
4 GiB, compressed into 64 KiB LZ4 frames exactly as the reference writer
does (65,536 frames, ~2.13 GB compressed), compressed image resident in HBM.
One step = one full-range decode of every frame (one grid, the product's
zsk_lz4_decode_frames C ABI) into a 4 GiB device buffer.

Multi-GPU (config 4, weak scaling): one process per GPU; rank r decodes its
own 4 GiB shard of a (4 GiB x N) buffer made of replicated compressed frames
(SURVEY §8d allows the replication); no collective on the timed path.  With
--reassemble (default for N > 1) the decoded shards are then gathered into
every rank with RCCL (all-gatherv as grouped broadcasts) and timed
separately.

Prints ONE JSON line (rank 0).  `value` = decoded bytes of all ranks / the
max-over-ranks time of the K timed steps.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "decompressed GB/s whole-node + achieved %HBM-read, LZ4 64KiB frames"
METRIC_ZSTD = "decompressed GB/s whole-node, zstd 64KiB frames (config 5)"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--size", type=int, default=4 << 30, help="decoded bytes per GPU")
    p.add_argument("--frame", type=int, default=64 << 10)
    p.add_argument("--threads", type=int, default=16, help="host threads (input gen, CPU baseline)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--reassemble", type=int, default=-1, help="1/0; default on when N>1")
    p.add_argument("--profile", action="store_true", help="few steps, no extras (rocprof runs)")
    p.add_argument("--codec", choices=["lz4", "zstd"], default="lz4",
                   help="lz4 = config 2 (the headline metric); zstd = config 5")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import libzseek_amd as z

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if args.profile:
        args.no_cpu_baseline = args.no_e2e = args.no_verify = True

    # ---- input: synthetic -> seekable LZ4 (the reference writer's bytes) ----
    t0 = time.time()
    data = z.synth_buffer(args.size, args.threads)
    zstd = args.codec == "zstd"
    img = (z.zstd_seekable(data, args.frame, 3, 1, args.threads) if zstd
           else z.lz4_seekable(data, args.frame, 0, args.threads))
    c_off, d_off = z.seek_table_of(img)
    nfr = len(c_off) - 1
    batch = z.frame_batch(c_off, d_off, 0, nfr)
    comp_bytes = int(batch.comp_end)
    log(f"[rank {rank}] input: {args.size / 2**30:.2f} GiB -> {comp_bytes / 1e9:.3f} GB "
        f"compressed, {nfr} frames, ratio {args.size / comp_bytes:.3f} ({time.time() - t0:.1f}s)")

    comp = torch.empty(comp_bytes + 256, dtype=torch.uint8, device=dev)
    comp[:comp_bytes].copy_(torch.from_numpy(img[:comp_bytes]))
    desc = torch.from_numpy(batch.desc.view(np.uint8).copy()).to(dev)
    out = torch.empty(batch.out_bytes, dtype=torch.uint8, device=dev)
    status = torch.empty(nfr, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def step():
        if zstd:
            z.zstd_decode_frames(desc, comp, out, status)
        else:
            z.decode_frames(desc, comp, out, status)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if int((status != 0).sum()) != 0:
        bad = int(torch.nonzero(status != 0)[0])
        raise SystemExit(f"frame {bad} failed: {z.status_string(int(status[bad]))}")

    # ---- timed region --------------------------------------------------------
    # the production launches alone (no per-stage events: recording them
    # between the kernels cost ~0.3 ms per launch at config 2)
    stream = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    w0 = time.perf_counter()
    ev[0].record(stream)
    for i in range(args.steps):
        step()
        ev[i + 1].record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - w0
    if world > 1:
        dist.barrier()
    kernel_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    # per-stage HIP events inside the library (plan / parse / execute /
    # hand-off kernels of each launch) from the same number of launches
    # right after, untimed
    z.kernel_timing(True)
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    n_timed, stage_ms = z.kernel_times()
    z.kernel_timing(False)
    t_local = sum(kernel_ms) / 1e3
    t = torch.tensor([t_local, wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t[0])
    ok_frames = int((status != 0).sum()) == 0

    # ---- correctness: decoded == generator (size-independent check) --------
    verified = None
    if not args.no_verify:
        ref_dev = torch.from_numpy(data).to(dev)
        verified = bool(ok_frames and torch.equal(out, ref_dev))
        del ref_dev
        if not verified:
            raise SystemExit("decoded output differs from the generator")

    # ---- optional RCCL reassembly (all-gatherv of decoded shards) ----------
    reassembly = None
    do_gather = (args.reassemble == 1) or (args.reassemble == -1 and world > 1)
    if world > 1 and do_gather:
        reassembly = reassemble(dist, torch, out, world, rank, dev)

    # ---- end-to-end zseek_pread (host buffers, PCIe-inclusive) --------------
    e2e = None
    if not args.no_e2e and rank == 0:
        e2e = end_to_end(z, img, args.size)

    # ---- CPU baseline: the reference library on the host cores -------------
    cpu = None
    if not args.no_cpu_baseline and rank == 0 and world == 1:
        cpu = cpu_baseline(img, args.size, args.frame, args.threads)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    dsum = args.size
    alg_bytes = comp_bytes + dsum           # sum(cSize + dSize)
    # one launch = the decode call: its kernels run back to back on the stream
    avg_kernel_s = sum(kernel_ms) / len(kernel_ms) / 1e3
    achieved = alg_bytes / avg_kernel_s / 1e9
    kname = "zstd_seq_kernel" if zstd else z.lib().zsk_lz4_kernel_name(nfr).decode()
    stages = None
    if n_timed:
        # the parse kernel the library picks for these frames (zsk_internal.h
        # chunk_parse_min: the chunk parse for big frames and small batches)
        avg_c = comp_bytes / nfr
        chunk = avg_c >= (49152 if nfr >= 32768 else 8192)
        lane_parse = "lz4_lean_kernel" if avg_c >= 12288 else "lz4_scan_kernel"   # zsk_internal.h kLeanMinCsize
        names = ({"plan": "zstd_plan_kernel + zstd_scan_kernel", "parse": "zstd_frame_kernel + zstd_huf_kernel + zstd_seq_kernel",
                  "execute": "seq_exec_kernel", "hand-off": "zstd_check_kernel"} if zstd else
                 {"plan": "lz4_plan_direct_kernel",
                  "parse": "lz4_chunk_kernel" if chunk else lane_parse,
                  "execute": "seq_exec_kernel", "hand-off": "lz4_wave_kernel<4096, 4, true>"})
        stages = {k: {"kernel": names[k], "avg_ms": round(v, 4)} for k, v in stage_ms.items()}
        if not zstd:   # the dominant kernel of the launch
            kname = max(("parse", "execute"), key=lambda k: stage_ms[k])
            kname = names[kname]
    value = dsum * world * args.steps / t_max / 1e9
    workload = ("config5: zstd 64KiB frames, 4 GiB synthetic per GPU, full-range decode, "
                "compressed image resident in HBM" if zstd else
                "config2: LZ4 64KiB frames, 4 GiB synthetic per GPU, full-range decode, "
                "compressed image resident in HBM" if args.frame == 64 << 10 else
                f"config3 (frame-size sweep): LZ4 {args.frame >> 10}KiB frames, "
                f"{args.size / 2**30:g} GiB synthetic per GPU, full-range decode, "
                "compressed image resident in HBM")
    line = {
        "metric": METRIC_ZSTD if zstd else METRIC,
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("synthetic (SURVEY §8d generator, compressed with libzstd 1.4.9 level 3 / strategy 1 "
                 "as the reference writer does)" if zstd else
                 "synthetic (SURVEY §8d generator, compressed with liblz4 1.9.3 as the reference writer does)"),
        "config": {"workload": workload,
                   "frame_bytes": args.frame, "frames_per_gpu": nfr,
                   "decoded_bytes_per_gpu": dsum, "compressed_bytes_per_gpu": comp_bytes,
                   "parallelism": f"frames sharded x{world}"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic_from_profile(kname, workload),
                     "kernel": kname, "launch": "zsk_lz4_decode_frames (stages below, back to back)",
                     "avg_launch_ms": round(avg_kernel_s * 1e3, 4),
                     "stages": stages,
                     "algorithmic_bytes_per_launch": alg_bytes},
        "cpu_baseline": cpu,
        "decoded_gbs_per_gpu": round(dsum / avg_kernel_s / 1e9, 2),
        "read_frac_of_hbm": round(comp_bytes / avg_kernel_s / 1e9 / HBM_PEAK_GBS, 4),
        "verified_bit_exact": verified,
        "end_to_end": e2e,
        "reassembly": reassembly,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def reassemble(dist, torch, out, world, rank, dev):
    """all-gatherv of the decoded shards (libzseek_amd.shard: one RCCL
    broadcast per source rank, grouped): every rank ends with all N slabs.
    Timed apart from the decode, on a 512 MiB slice per rank to bound memory."""
    from libzseek_amd import shard
    n = min(out.numel(), 512 << 20)
    counts = [n] * world
    full = torch.empty(n * world, dtype=torch.uint8, device=dev)
    shard.all_gatherv(dist, out[:n], counts, out=full)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    shard.all_gatherv(dist, out[:n], counts, out=full)
    torch.cuda.synchronize()
    t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = bool(torch.equal(full[rank * n:(rank + 1) * n], out[:n]))
    return {"bytes_per_rank": n, "seconds": round(float(t[0]), 6),
            "received_GBps_per_rank": round(n * (world - 1) / float(t[0]) / 1e9, 2),
            "method": "RCCL grouped broadcast (all-gatherv)", "own_slab_intact": ok}


def end_to_end(z, img, size):
    """zseek_pread of the whole range into host memory (pinned staging,
    PCIe both ways) — reported beside, never as `value`."""
    buf = np.empty(size, np.uint8)
    with z.Reader(img, 0) as r:
        r.pread_raw(buf.ctypes.data, 64 << 20, 0)      # warm the device context
        t0 = time.perf_counter()
        n = r.pread_raw(buf.ctypes.data, size, 0)
        dt = time.perf_counter() - t0
    return {"GBps": round(n / dt / 1e9, 2), "bytes": int(n), "api": "zseek_pread (host buffer)"}


def traffic_from_profile(kernel, workload):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic.json, written by scripts/round_profiles.py), used
    only when it was recorded for the kernel this build launches on this
    same workload (a config-3 sweep line gets none)."""
    for name in ("pmc_traffic.json", "pmc_traffic_zstd.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if kernel in rec.get("kernel", "") and rec.get("workload") == workload:
            return rec.get("hbm_bytes_per_launch")
    return None


def cpu_baseline(img, size, frame, threads):
    """The reference CPU path (oracle/_ref: /root/reference/src compiled
    against liblz4 1.9.3) timed on this host: T independent readers over
    disjoint frame-aligned slices of the same image, in-memory pread."""
    try:
        from oracle.oracle import RefBench
        rb = RefBench()
    except Exception as e:   # reference build absent
        return {"value": None, "unit": "GB/s", "cores": 0, "kind": "reference",
                "sample": f"unavailable: {e}"}
    sample = min(size, 2 << 30)
    best = 0.0
    for _ in range(3):
        secs, nbytes = rb.run(img, threads, 0, sample, frame, frame, 0)
        best = max(best, nbytes / secs / 1e9)
    one = min(size, 256 << 20)
    secs1, nb1 = rb.run(img, 1, 0, one, frame, frame, 0)
    return {"value": round(best, 2), "unit": "GB/s", "cores": threads, "kind": "reference",
            "sample": f"first {sample >> 20} MiB decoded by {threads} reference readers "
                      f"(cache_size=0, 64 KiB zseek_pread calls), best of 3; "
                      f"1 thread on {one >> 20} MiB: {nb1 / secs1 / 1e9:.2f} GB/s; "
                      f"host {os.cpu_count()} CPUs visible"}


if __name__ == "__main__":
    main()
