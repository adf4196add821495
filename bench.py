"""bench.py — decoded GB/s of the GPU LZ4 random-access decode path.

Workloads (BASELINE.json configs):
  N = 1 (default)   config 2: the SURVEY §8d synthetic, 4 GiB, compressed into
                    64 KiB LZ4 frames exactly as the reference writer does
                    (65,536 frames, ~2.13 GB compressed), image resident in HBM.
                    One step = one zsk_lz4_decode_frames launch over every frame.
  N > 1 (default)   config 4: a FIXED 64 GiB buffer (the 4 GiB synthetic's
                    compressed frames replicated x16, as SURVEY §8d allows;
                    1,048,576 frames) split over N ranks, one process per GPU
                    (strong scaling).  Frames shard contiguously (default) or
                    round-robin (--partition round_robin: frame i -> rank i %
                    N).  One step = each rank decodes all of its frames (launches
                    of <= 65,536 frames back to back on its stream); no
                    collective on the timed path.  The RCCL reassembly of the
                    full 64 GiB range on every rank (all-gather of the decoded
                    slabs, + the permute back to frame order for round-robin) is
                    timed separately (`reassembly`).
  --total-size B    any fixed total (strong scaling, e.g. config 4 at N = 1);
  --weak            N ranks x --size bytes each instead (weak scaling).

`python bench.py --gpus N` with no torchrun environment starts N rank
processes itself (torch.distributed.run as a child process; this parent never
touches the GPU) and exits with their status; under torchrun (WORLD_SIZE set)
it is one rank.  Rank 0 prints ONE JSON line: `value` = decoded bytes of all
ranks x steps / the max-over-ranks time of the timed steps.

Beside the line (rank 0, N = 1): `cpu_baseline` — the reference library
(oracle/_ref: /root/reference/src compiled against liblz4 1.9.3 / libzstd
1.4.9) on the host cores, 1 thread and every usable core; `end_to_end` — the
drop-in zseek_pread into host memory (PCIe-inclusive, never `value`);
`latency_4k_us` — 4 KiB random zseek_pread requests, ours and the reference's.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "decompressed GB/s whole-node + achieved %HBM-read, LZ4 64KiB frames"
METRIC_ZSTD = "decompressed GB/s whole-node, zstd 64KiB frames (config 5)"
METRIC_LZ4C = "LZ4 frame compression GB/s (input bytes) whole-node, 64KiB frames (SURVEY 8f row 4)"
GiB = 1 << 30
CHUNK_BYTES = 4 * GiB    # decoded bytes per decode launch (config 4's 64 GiB steps: several)


def chunk_frames(frame):
    """frames per decode launch: one launch for the 4 GiB configs (2, 3), 4 GiB
    launches for bigger per-rank workloads"""
    return max(65536, CHUNK_BYTES // frame)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def size_arg(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30, "T": 1 << 40}
    if s and s[-1] in mult:
        return int(float(s[:-1]) * mult[s[-1]])
    return int(s)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=10)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--size", type=size_arg, default=4 * GiB,
                   help="the generated synthetic (weak scaling: decoded bytes per GPU)")
    p.add_argument("--total-size", type=size_arg, default=None,
                   help="fixed decoded total split over the ranks (strong scaling); "
                        "default 64 GiB (config 4) when N > 1")
    p.add_argument("--weak", action="store_true", help="N > 1: --size per rank (weak scaling)")
    p.add_argument("--partition", choices=["contiguous", "round_robin"], default="round_robin",
                   help="N > 1: frame i -> rank i mod N (config 4), or contiguous slabs")
    p.add_argument("--frame", type=size_arg, default=64 << 10)
    p.add_argument("--threads", type=int, default=16, help="host threads for input generation")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-latency", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--reassemble", type=int, default=-1, help="1/0; default on when N > 1")
    p.add_argument("--profile", action="store_true", help="few steps, no extras (rocprof runs)")
    p.add_argument("--codec", choices=["lz4", "zstd", "lz4c"], default="lz4",
                   help="lz4 = configs 2-4 (the headline metric); zstd = config 5; lz4c = "
                        "GPU LZ4 frame compression (SURVEY §8f row 4, not a BASELINE config)")
    p.add_argument("--harness-check", action="store_true",
                   help="CPU rehearsal of the multi-rank harness (gloo, no GPU: a host "
                        "copy of the expected bytes stands in for the decode)")
    return p.parse_args(argv)


# ---------------------------------------------------------------------------
# launcher: N ranks from a plain `python bench.py --gpus N`
# ---------------------------------------------------------------------------
def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int) -> int:
    """torch.distributed.run as a child process, one rank per GPU.  The
    parent has not initialised HIP (it imports nothing GPU-related)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1",
           f"--master-port={free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "4")
    log(f"[bench] starting {n} ranks: {' '.join(cmd)}")
    return subprocess.call(cmd, env=env)


# ---------------------------------------------------------------------------
# host description for the CPU baseline
# ---------------------------------------------------------------------------
def host_cpus() -> dict:
    visible = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = visible
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = int(q) / int(per)
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    physical = None   # physical cores of the node (sockets x cores), for the reader's scale
    try:
        pairs, phys, core = set(), None, None
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("physical id"):
                phys = ln.split(":", 1)[1].strip()
            elif ln.startswith("core id"):
                core = ln.split(":", 1)[1].strip()
            elif not ln.strip() and phys is not None:
                pairs.add((phys, core))
                phys = core = None
        physical = len(pairs) or None
    except OSError:
        pass
    return {"visible": visible, "affinity": aff, "cgroup_quota": quota, "usable": usable,
            "physical_cores": physical, "model": model}


# ---------------------------------------------------------------------------
# one rank's shard of the (replicated) image
# ---------------------------------------------------------------------------
class Shard:
    """This rank's frames of a global range of F frames made of R replicas of
    a base image of B frames (global frame g = base frame g % B): their
    compressed bytes back to back (replica sub-images), descriptors, and
    where the decoded bytes come from (for verification)."""

    def __init__(self, z, img, c_off, d_off, total_frames, world, rank, partition):
        B = len(c_off) - 1
        self.base_frames = B
        self.F = total_frames
        if partition == "contiguous":
            g0, g1 = rank * total_frames // world, (rank + 1) * total_frames // world
            frames = np.arange(g0, g1, dtype=np.int64)
        else:
            frames = np.arange(rank, total_frames, world, dtype=np.int64)
        self.frames = frames
        base_idx = frames % B
        csz = np.diff(c_off.astype(np.int64))
        dsz = np.diff(d_off.astype(np.int64))
        self.cs = csz[base_idx]
        self.ds = dsz[base_idx]
        # replica pieces: (replica k, base frames of this rank in it)
        rep = frames // B
        self.pieces = []
        cache = {}
        starts = np.searchsorted(rep, np.arange(rep[0] if len(rep) else 0,
                                                (rep[-1] + 2) if len(rep) else 0))
        for i in range(len(starts) - 1):
            a, b = int(starts[i]), int(starts[i + 1])
            if a == b:
                continue
            sel = base_idx[a:b]
            contiguous = bool(len(sel) == sel[-1] - sel[0] + 1 and (np.diff(sel) == 1).all())
            key = (int(sel[0]), int(sel[-1]), len(sel), contiguous)
            if key not in cache:
                if contiguous:
                    sub = img[int(c_off[sel[0]]): int(c_off[sel[-1] + 1])]
                else:
                    sub = np.concatenate([img[int(c_off[j]): int(c_off[j + 1])] for j in sel])
                cache[key] = sub
            self.pieces.append((a, b, sel, cache[key], key))
        self.comp_bytes = int(self.cs.sum())
        self.out_bytes = int(self.ds.sum())
        desc = np.empty(len(frames), z.FRAME_DESC_DTYPE)
        desc["c_off"] = np.concatenate([[0], np.cumsum(self.cs)[:-1]]) if len(frames) else []
        desc["d_off"] = np.concatenate([[0], np.cumsum(self.ds)[:-1]]) if len(frames) else []
        desc["c_size"] = self.cs.astype(np.uint32)
        desc["d_size"] = self.ds.astype(np.uint32)
        self.desc = desc

    def upload(self, torch, dev):
        """Compressed shard into one device buffer (each distinct replica
        sub-image uploaded once, repeated by device copies)."""
        comp = torch.empty(self.comp_bytes + 256, dtype=torch.uint8, device=dev)
        at = 0
        uploaded = {}
        for a, b, sel, sub, key in self.pieces:
            n = sub.size
            if key in uploaded:
                src_at = uploaded[key]
                comp[at: at + n].copy_(comp[src_at: src_at + n])
            else:
                comp[at: at + n].copy_(torch.from_numpy(np.ascontiguousarray(sub)))
                uploaded[key] = at
            at += n
        assert at == self.comp_bytes
        return comp

    def expected_rows(self, torch, base_dev, frame):
        """(out row range, base frame indices) per replica piece, for uniform
        frames: decoded frame i of the shard == base frame sel."""
        for a, b, sel, sub, key in self.pieces:
            yield a, b, sel


def decode_launches(z, torch, desc_dev, n, comp, out, status, zstd, per):
    """One step: every frame of the rank, launches of <= per frames (LZ4)
    back to back on the current stream; zstd: one launch."""
    L = z.lib()
    stream = torch.cuda.current_stream().cuda_stream
    if zstd:
        if L.zsk_zstd_decode_frames(desc_dev.data_ptr(), n, comp.data_ptr(), out.data_ptr(),
                                    status.data_ptr(), stream) != 0:
            raise SystemExit("zsk_zstd_decode_frames launch failed")
        return
    for s in range(0, n, per):
        m = min(per, n - s)
        if L.zsk_lz4_decode_frames(desc_dev.data_ptr() + 24 * s, m, comp.data_ptr(), out.data_ptr(),
                                   status.data_ptr() + 4 * s, stream) != 0:
            raise SystemExit("zsk_lz4_decode_frames launch failed")


# ---------------------------------------------------------------------------
def main():
    args = parse()
    world_env = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not world_env:
        sys.exit(spawn_ranks(args.gpus))
    import torch
    import torch.distributed as dist

    import libzseek_amd as z

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    harness = args.harness_check
    if harness:
        dev = torch.device("cpu")
        if world > 1:
            dist.init_process_group("gloo")
    elif os.environ.get("ZSEEK_BENCH_SHARE_GPU") == "1":
        # rehearsal of the multi-rank GPU path on a one-GPU box: every rank
        # decodes on device 0, the collective runs over gloo (RCCL refuses
        # two ranks on one device); never the measured configuration
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(0)
        if world > 1:
            dist.init_process_group("gloo")
    else:
        dev = torch.device("cuda", local)
        if world > 1:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=dev)
    if args.profile:
        args.no_cpu_baseline = args.no_e2e = args.no_verify = args.no_latency = True
    if args.codec == "lz4c":
        return main_compress(args, torch, dist, z, dev, world, rank)
    zstd = args.codec == "zstd"

    # ---- workload -------------------------------------------------------------
    strong = args.total_size is not None or (world > 1 and not args.weak)
    total = args.total_size if args.total_size is not None else (
        64 * GiB if strong else args.size * world)
    base_size = min(args.size, total)
    if strong and (total % args.frame or base_size % args.frame or total % base_size):
        raise SystemExit("strong scaling needs --total-size a multiple of --size, both of --frame")

    t0 = time.time()
    data = z.synth_buffer(base_size, args.threads)
    img = (z.zstd_seekable(data, args.frame, 3, 1, args.threads) if zstd
           else z.lz4_seekable(data, args.frame, 0, args.threads))
    c_off, d_off = z.seek_table_of(img)
    base_frames = len(c_off) - 1
    if strong:
        sh = Shard(z, img, c_off, d_off, total // args.frame, world, rank, args.partition)
    else:   # weak: every rank decodes the whole base image
        sh = Shard(z, img, c_off, d_off, base_frames, 1, 0, "contiguous")
    nfr = len(sh.frames)
    log(f"[rank {rank}] input: base {base_size / GiB:.2f} GiB -> {int(c_off[-1]) / 1e9:.3f} GB "
        f"compressed ({base_frames} frames); shard {nfr} frames, {sh.out_bytes / GiB:.2f} GiB "
        f"decoded, {sh.comp_bytes / 1e9:.3f} GB compressed ({time.time() - t0:.1f}s)")

    comp = sh.upload(torch, dev)
    desc_dev = torch.from_numpy(sh.desc.view(np.uint8).copy()).to(dev)
    out = torch.empty(sh.out_bytes, dtype=torch.uint8, device=dev)
    status = torch.zeros(nfr, dtype=torch.int32, device=dev)
    base_dev = None
    if harness or not args.no_verify:
        base_dev = torch.from_numpy(data).to(dev)

    def step():
        if harness:   # rehearsal: the expected bytes stand in for the decode
            fill_expected(torch, out, sh, base_dev, args.frame)
        else:
            decode_launches(z, torch, desc_dev, nfr, comp, out, status, zstd, chunk_frames(args.frame))

    def sync():
        if not harness:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    sync()
    if int((status != 0).sum()) != 0:
        bad = int(torch.nonzero(status != 0)[0])
        raise SystemExit(f"frame {bad} failed: {z.status_string(int(status[bad]))}")

    # ---- timed region: K steps, barrier + synchronize on both sides ----------
    ev = None if harness else [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if world > 1:
        dist.barrier()
    sync()
    w0 = time.perf_counter()
    if ev:
        ev[0].record(torch.cuda.current_stream())
    for i in range(args.steps):
        step()
        if ev:
            ev[i + 1].record(torch.cuda.current_stream())
    sync()
    wall = time.perf_counter() - w0
    if world > 1:
        dist.barrier()
    step_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)] if ev else \
        [wall * 1e3 / args.steps] * args.steps
    t_local = sum(step_ms) / 1e3
    t = torch.tensor([t_local, wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t[0])

    # per-stage HIP events of the library's launches, from as many launches
    # right after the timed region (untimed: events between kernels cost time)
    stage_ms, n_timed = None, 0
    if not harness:
        z.kernel_timing(True)
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        n_timed, stage_ms = z.kernel_times(spans=zstd)
        z.kernel_timing(False)

    # ---- correctness: decoded == generator (size-independent check) --------
    verified = None
    if not args.no_verify:
        verified = bool(int((status != 0).sum()) == 0 and check_shard(torch, out, sh, base_dev, args.frame))
        if world > 1:
            v = torch.tensor([0 if verified else 1], dtype=torch.int32, device=dev)
            dist.all_reduce(v, op=dist.ReduceOp.MAX)
            verified = int(v) == 0
        if not verified:
            raise SystemExit("decoded output differs from the generator")

    # ---- RCCL reassembly of the full range on every rank ---------------------
    reassembly = None
    do_gather = (args.reassemble == 1) or (args.reassemble == -1 and world > 1)
    if world > 1 and do_gather and strong:
        reassembly = reassemble(dist, torch, out, sh, world, rank, dev, args, base_dev, harness)

    # ---- extras on rank 0, one GPU --------------------------------------------
    e2e = lat = cpu = None
    host = host_cpus()
    if rank == 0 and world == 1 and not harness:
        if not args.no_e2e:
            e2e = end_to_end(z, img, base_size)
        if not args.no_latency:
            lat = latency(z, img, base_size)
        if not args.no_cpu_baseline:
            cpu = cpu_baseline(img, base_size, args.frame, host, zstd, not args.no_latency)

    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    dsum = sh.out_bytes                      # decoded bytes per rank per step (rank 0)
    comp_bytes = sh.comp_bytes
    total_step = total if strong else dsum * world
    value = total_step * args.steps / t_max / 1e9
    alg_bytes = comp_bytes + dsum            # sum(cSize + dSize), per launch-set
    avg_step_s = t_local / args.steps
    achieved = alg_bytes / avg_step_s / 1e9
    stages, kname = None, None
    if stage_ms is not None and n_timed:
        avg_c = comp_bytes / max(nfr, 1)
        if zstd:
            # the decode runs in frame chunks over three streams: per-kernel
            # spans on the stream each kernel runs on, summed over the chunks
            # (they overlap one another; `stages` below are not additive)
            names = {"plan": "zstd_plan_kernel + zstd_scan_kernel + zstd_bounds_kernel",
                     "zstd_frame_kernel": "zstd_frame_kernel", "zstd_seq_kernel": "zstd_seq_kernel",
                     "zstd_huf_kernel": "zstd_huf_kernel", "seq_exec_kernel": "seq_exec_kernel"}
            launches = 1
            kernels = ("zstd_frame_kernel", "zstd_seq_kernel", "zstd_huf_kernel", "seq_exec_kernel")
        else:
            parse_k = z.parse_kernel_name(min(nfr, chunk_frames(args.frame)), int(avg_c))
            names = {"plan": "lz4_plan_direct_kernel", "parse": parse_k,
                     "execute": "seq_exec_kernel", "hand-off": "lz4_wave_kernel<4096, 4, true>"}
            launches = (nfr + chunk_frames(args.frame) - 1) // chunk_frames(args.frame)
            kernels = ("parse", "execute")
        # kernel_times gives per-launch medians; a step is `launches` launches
        stages = {k: {"kernel": names[k], "median_ms": round(stage_ms[k] * launches, 4)} for k in names}
        kname = names[max(kernels, key=lambda k: stage_ms[k])]
    dom = None
    if stages and kname:
        dk = [k for k, v in stages.items() if v["kernel"] == kname]
        if dk and stages[dk[0]]["median_ms"] > 0:   # (a library without per-stage timing reports 0)
            dms = stages[dk[0]]["median_ms"] / 1e3
            dom = {"kernel": kname, "median_ms": round(dms * 1e3, 4),
                   "achieved": round(alg_bytes / dms / 1e9, 1),
                   "frac": round(alg_bytes / dms / 1e9 / HBM_PEAK_GBS, 4)}
    if strong and world > 1:
        workload = (f"config4: LZ4 64KiB frames, fixed {total / GiB:g} GiB buffer ({total // args.frame} "
                    f"frames; the {base_size / GiB:g} GiB synthetic's frames x{total // base_size}) "
                    f"sharded {args.partition} over {world} GPUs, compressed shards resident in HBM")
    elif strong and total != base_size:
        workload = (f"config4 (N=1 point): LZ4 64KiB frames, fixed {total / GiB:g} GiB buffer "
                    f"(the {base_size / GiB:g} GiB synthetic's frames x{total // base_size}), one GPU")
    elif zstd:
        workload = ("config5: zstd 64KiB frames, 4 GiB synthetic per GPU, full-range decode, "
                    "compressed image resident in HBM")
    elif args.frame == 64 << 10:
        workload = ("config2: LZ4 64KiB frames, 4 GiB synthetic per GPU, full-range decode, "
                    "compressed image resident in HBM")
    else:
        workload = (f"config3 (frame-size sweep): LZ4 {args.frame >> 10}KiB frames, "
                    f"{base_size / GiB:g} GiB synthetic per GPU, full-range decode, "
                    "compressed image resident in HBM")
    line = {
        "metric": METRIC_ZSTD if zstd else METRIC,
        "value": None if harness else round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if (strong and world > 1) else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": ("harness rehearsal: gloo on CPU, a host copy of the expected bytes stands in "
                 "for the GPU decode (no measurement)" if harness else
                 (f"synthetic (SURVEY §8d generator, compressed with libzstd "
                  f"{z.zstd_tool_version()} level 3 / strategy 1 as the reference writer does)") if zstd else
                 "synthetic (SURVEY §8d generator, compressed with liblz4 1.9.3 as the reference "
                 "writer does)"),
        "config": {"workload": workload,
                   "frame_bytes": args.frame, "frames_per_gpu": nfr,
                   "decoded_bytes_total": total_step,
                   "decoded_bytes_per_gpu": dsum, "compressed_bytes_per_gpu": comp_bytes,
                   "parallelism": (f"frames sharded x{world} ({args.partition})" if world > 1
                                   else "one GPU")},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic_from_profile(kname, workload),
                     "kernel": kname,
                     "launch": "zsk_lz4_decode_frames (stages below, back to back)" if not zstd
                               else "zsk_zstd_decode_frames",
                     "avg_launch_ms": round(avg_step_s * 1e3, 4),
                     "dominant_kernel": dom,
                     "stages": stages,
                     "algorithmic_bytes_per_launch": alg_bytes},
        "cpu_baseline": cpu,
        "decoded_gbs_per_gpu": round(dsum / avg_step_s / 1e9, 2),
        "read_frac_of_hbm": round(comp_bytes / avg_step_s / 1e9 / HBM_PEAK_GBS, 4),
        "verified_bit_exact": verified,
        "end_to_end": e2e,
        "latency_4k_us": lat,
        "reassembly": reassembly,
        "host": host,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main_compress(args, torch, dist, z, dev, world, rank):
    """--codec lz4c: every rank compresses its own --size bytes of the §8d
    synthetic into --frame (<= 4 MiB; linked blocks above 64 KiB) LZ4 frames on its GPU, input resident
    in HBM (weak scaling).  One step = one zsk_lz4_compress_frames launch over
    every frame (memset of the position tables, lz4_compress_kernel,
    lz4_store_kernel).  Output: byte-identical to liblz4's frames (checked
    against the writer-identical seekable image after the timed region)."""
    if args.frame > 1 << 22:
        raise SystemExit("--codec lz4c: frames of at most 4 MiB (ZSK_LZ4_COMPRESS_MAX_FRAME)")
    t0 = time.time()
    size = args.size - args.size % args.frame
    data = z.synth_buffer(size, args.threads)
    nfr = size // args.frame
    desc, dst_bytes = z.lz4_compress_layout(np.full(nfr, args.frame, np.uint64))
    d_desc = torch.from_numpy(desc.view(np.uint8).copy()).to(dev)
    d_src = torch.from_numpy(data).to(dev)
    d_dst = torch.empty(dst_bytes, dtype=torch.uint8, device=dev)
    csize = torch.zeros(nfr, dtype=torch.int32, device=dev)
    scratch = torch.empty(z.lz4_compress_scratch_size(nfr), dtype=torch.uint8, device=dev)
    log(f"[rank {rank}] lz4c input: {size / GiB:.2f} GiB, {nfr} frames ({time.time() - t0:.1f}s)")
    stream = torch.cuda.current_stream()

    def step():
        z.lz4_compress_frames(d_desc, d_src, d_dst, csize, 0, scratch, stream.cuda_stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
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
    step_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    t_local = sum(step_ms) / 1e3
    t = torch.tensor([t_local, wall], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = float(t[0])

    cs = csize.cpu().numpy().astype(np.int64)
    comp_bytes = int(cs.sum())
    verified = None
    if not args.no_verify:
        img = np.asarray(z.lz4_seekable(data, args.frame, 0, args.threads))
        c_off, _ = z.seek_table_of(img)
        host = d_dst.cpu().numpy()
        ok = bool((cs == np.diff(c_off)).all())
        offs = desc["dst_off"]
        for f in range(nfr if ok else 0):
            if host[int(offs[f]):int(offs[f]) + int(cs[f])].tobytes() != \
                    img[int(c_off[f]):int(c_off[f + 1])].tobytes():
                ok = False
                break
        verified = ok
        if not ok:
            raise SystemExit("GPU frames differ from liblz4's")
    cpu = by_frames = writer = None
    host_info = host_cpus()
    if rank == 0 and world == 1 and not args.profile:
        # launch time against frames per launch (a lane compresses one frame
        # serially, so throughput grows with frames in flight)
        by_frames = {}
        for k in (1024, 4096, 16384):
            if k < nfr:
                ts = []
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    z.lz4_compress_frames(d_desc[: 24 * k], d_src, d_dst, csize[:k], 0, scratch,
                                          stream.cuda_stream)
                    e1.record(stream)
                    torch.cuda.synchronize()
                    ts.append(e0.elapsed_time(e1))
                by_frames[str(k)] = {"ms": round(min(ts), 3),
                                     "GBps": round(k * args.frame / min(ts) / 1e6, 2)}
        by_frames[str(nfr)] = {"ms": round(t_local / args.steps * 1e3, 3),
                               "GBps": round(size / (t_local / args.steps) / 1e9, 2)}
        writer = writer_end_to_end(z, data, args.frame)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_compress(z, data, args.frame, host_info, args.threads)
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    avg_s = t_local / args.steps
    alg = size + comp_bytes                  # input read once + frames written once
    workload_c = (f"lz4c: {size / GiB:g} GiB synthetic per GPU into {args.frame >> 10}KiB "
                  "LZ4 frames (level 0, as compress.c:203-207 / :750)")
    line = {
        "metric": METRIC_LZ4C, "value": round(size * world * args.steps / t_max / 1e9, 2),
        "unit": "GB/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(t_max / args.steps * 1e3, 4), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (SURVEY §8d generator), resident in HBM",
        "config": {"workload": workload_c,
                   "frame_bytes": args.frame, "frames_per_gpu": nfr, "input_bytes_per_gpu": size,
                   "compressed_bytes_per_gpu": comp_bytes,
                   "parallelism": f"x{world} independent ranks" if world > 1 else "one GPU"},
        "roofline": {"bound": "hbm", "achieved": round(alg / avg_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg / avg_s / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": traffic_from_profile("lz4_compress_kernel", workload_c),
                     "kernel": "lz4_compress_kernel",
                     "launch": "zsk_lz4_compress_frames (memset + lz4_compress_kernel + lz4_store_kernel)",
                     "avg_launch_ms": round(avg_s * 1e3, 4), "algorithmic_bytes_per_launch": alg},
        "cpu_baseline": cpu,
        "verified_bit_exact": verified,
        "launch_by_frames": by_frames,
        "writer_end_to_end": writer,
        "host": host_info,
    }
    print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def writer_end_to_end(z, data, frame, size=1 << 30):
    """The drop-in writer (zseek_write of frame-sized writes into an in-memory
    sink, then zseek_writer_close) over the first `size` bytes: host liblz4
    (the reference's path) against GPU mode with 1 GiB and 4 GiB batches
    (host staging, PCIe both ways and the write callbacks included).  Files
    compared byte for byte."""
    size = min(size, data.size)
    chunks = [data[o: o + frame] for o in range(0, size, frame)]
    res, files = {"input_bytes": size}, {}
    for name, batch in (("host", None), ("gpu_batch_1GiB", 1 << 30), ("gpu_batch_4GiB", 4 << 30)):
        w = z.Writer(z.ZSEEK_LZ4, frame)
        if batch is not None and not w.set_gpu_compress(batch):
            res[name] = None
            continue
        t0 = time.perf_counter()
        for c in chunks:
            w.write(c)
        files[name] = w.close()
        res[name + "_GBps"] = round(size / (time.perf_counter() - t0) / 1e9, 3)
    res["identical"] = len(set(files.values())) == 1
    return res


def cpu_baseline_compress(z, data, frame, host, threads):
    """liblz4 1.9.3's LZ4F_compressFrame, the compressor the reference writer
    calls, on the host: the reference writer itself (oracle/_ref, one thread)
    on the first 512 MiB, and frame-parallel liblz4 (libzseek_tools, T
    threads over independent frames, the writer's prefs) on the whole input."""
    res = {"unit": "GB/s", "kind": "reference"}
    one = min(data.size, 512 << 20)
    try:
        from oracle.oracle import RefZseek, ZSEEK_LZ4
        ref = RefZseek()
        t0 = time.perf_counter()
        ref.compress(data[:one].tobytes(), ZSEEK_LZ4, frame, frame)
        res["one_thread_GBps"] = round(one / (time.perf_counter() - t0) / 1e9, 3)
    except Exception as e:   # reference build absent
        res["one_thread_GBps"] = None
        res["one_thread_note"] = f"reference writer unavailable: {e}"
    best = 0.0
    cores = host["usable"]   # the CPUs this process may run on (affinity, cgroup quota)
    for _ in range(2):
        t0 = time.perf_counter()
        z.lz4_seekable(data, frame, 0, cores)
        best = max(best, data.size / (time.perf_counter() - t0) / 1e9)
    res.update({"value": round(best, 2), "cores": cores, "per_core_GBps": round(best / cores, 3),
                "node_physical_cores": host.get("physical_cores"),
                "sample": (f"reference writer (1 thread, {frame >> 10} KiB direct writes) on the first "
                           f"{one >> 20} MiB; liblz4 LZ4F_compressFrame with the writer's prefs over "
                           f"the whole {data.size >> 20} MiB, frames spread over {cores} threads "
                           f"(the usable CPUs); host {host['model']}")})
    return res


def fill_expected(torch, out, sh, base_dev, frame):
    """Harness rehearsal only: the bytes the decode would produce."""
    rows = out.view(-1, frame)
    base_rows = base_dev.view(-1, frame)
    for a, b, sel in sh.expected_rows(torch, base_dev, frame):
        rows[a:b].copy_(base_rows[torch.from_numpy(sel).to(base_dev.device)])


def check_shard(torch, out, sh, base_dev, frame):
    """Decoded shard == the generator's bytes for its frames (uniform frames:
    row views; the weak case is the base image itself)."""
    if sh.out_bytes == base_dev.numel() and len(sh.pieces) == 1 and sh.pieces[0][4][3]:
        return bool(torch.equal(out, base_dev))
    if sh.out_bytes % frame or base_dev.numel() % frame:
        raise SystemExit("verification of a replicated shard needs uniform frames")
    rows = out.view(-1, frame)
    base_rows = base_dev.view(-1, frame)
    for a, b, sel in sh.expected_rows(torch, base_dev, frame):
        s0, s1 = int(sel[0]), int(sel[-1]) + 1
        if s1 - s0 == b - a:
            ok = torch.equal(rows[a:b], base_rows[s0:s1])
        else:
            ok = torch.equal(rows[a:b], base_rows[torch.from_numpy(sel).to(base_dev.device)])
        if not ok:
            return False
    return True


def reassemble(dist, torch, out, sh, world, rank, dev, args, base_dev, harness):
    """The full decoded range on every rank: all-gather of the decoded slabs
    (RCCL over xGMI; equal slabs -> all_gather_into_tensor, ragged -> grouped
    broadcasts), then for round-robin the permute back to frame order.  Timed
    apart from the decode (once warm, then timed), max over ranks."""
    from libzseek_amd import shard as shmod
    counts = [0] * world
    cnt = torch.tensor([sh.out_bytes], dtype=torch.int64, device=dev)
    allc = [torch.zeros(1, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allc, cnt)
    counts = [int(c) for c in allc]
    full = torch.empty(sum(counts), dtype=torch.uint8, device=dev)

    def once():
        g0 = time.perf_counter()
        shmod.all_gatherv(dist, out, counts, out=full)
        if not harness:
            torch.cuda.synchronize()
        g1 = time.perf_counter()
        res = full
        if args.partition == "round_robin":
            res = full.view(world, -1, args.frame).transpose(0, 1).reshape(-1)
            if not harness:
                torch.cuda.synchronize()
        return res, g1 - g0, time.perf_counter() - g1

    once()
    dist.barrier()
    res, tg, tp = once()
    t = torch.tensor([tg, tp], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ok = None
    if base_dev is not None:
        b = base_dev.numel()
        ok = bool(res.numel() % b == 0 and all(torch.equal(res[i: i + b], base_dev)
                                               for i in range(0, res.numel(), b)))
        v = torch.tensor([0 if ok else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        ok = int(v) == 0
    recv = sum(counts) - counts[rank]
    return {"bytes_total": sum(counts), "gather_s": round(float(t[0]), 6),
            "permute_s": round(float(t[1]), 6) if args.partition == "round_robin" else None,
            "received_GBps_per_rank": round(recv / float(t[0]) / 1e9, 2),
            "method": ("all_gather_into_tensor" if len(set(counts)) == 1 else
                       "grouped broadcasts (all-gatherv)") +
                      (" over gloo (rehearsal)" if harness or dist.get_backend() == "gloo"
                       else " over RCCL/xGMI"),
            "full_range_matches_generator": ok}


def pcie_d2h_rate(nbytes=256 << 20, reps=5):
    """best device -> pinned host copy rate (GB/s) of one GPU"""
    import torch
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dev.fill_(1)
    pin = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    best = 0.0
    for _ in range(reps):
        torch.cuda.synchronize()
        t = time.perf_counter()
        pin.copy_(dev, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, nbytes / (time.perf_counter() - t) / 1e9)
    return round(best, 2)


def end_to_end(z, img, size):
    """zseek_pread of the whole range into host memory through the drop-in C
    API (a C in-memory pread callback; pinned staging, H2D, decode, D2H) —
    reported beside, never as `value`.  io_threads 1 is the reference's
    contract (one pread callback at a time); 8 is the opt-in
    zsk_reader_set_io_threads for a thread-safe callback."""
    T = z.tools()
    L = z.lib()
    import ctypes as C
    res = {"api": "zseek_pread (host buffer, one call, C in-memory pread callback)", "bytes": size}
    # the link a host destination crosses (verdict r05 item 8): one GPU's
    # device -> pinned-host copy rate, measured here (scripts/pcie_probe.py
    # has the full probe) -- the ceiling of any zseek_pread into host memory
    res["pcie_d2h_pinned_GBps"] = pcie_d2h_rate()
    res["bound"] = ("host destination: every decoded byte crosses PCIe, so one GPU delivers at most "
                    "pcie_d2h_pinned_GBps into host memory (the reference decodes in host memory: "
                    "cpu_baseline); zsk_pread_device keeps the bytes in HBM (the measured `value`)")
    buf = np.empty(size, np.uint8)
    gs = z.zseek.GpuStatsC()
    for io in (1, 8):
        err = C.create_string_buffer(80)
        r = T.zsk_tool_open_mem(C.cast(L.zseek_reader_open_full, C.c_void_p), img.ctypes.data,
                                img.size, 0, err)
        if not r:
            return {"error": err.value.decode()}
        L.zsk_reader_set_io_threads(r, io)
        got = C.c_size_t(0)
        T.zsk_tool_read_all(C.cast(L.zseek_pread, C.c_void_p), r, buf.ctypes.data, 64 << 20,
                            C.byref(got))
        best = 0.0
        for _ in range(2):
            secs = T.zsk_tool_read_all(C.cast(L.zseek_pread, C.c_void_p), r, buf.ctypes.data, size,
                                       C.byref(got))
            if got.value != size:
                return {"error": f"short read {got.value}"}
            best = max(best, got.value / secs / 1e9)
        L.zsk_reader_gpu_stats_ex(r, C.byref(gs), C.sizeof(gs))
        T.zsk_tool_close_mem(C.cast(L.zseek_reader_close, C.c_void_p), r)
        res["GBps" if io == 1 else f"GBps_io{io}"] = round(best, 2)
        # host threads the read ran on: the copy / pread pool (usable CPUs - 2)
        # and the concurrent pread callbacks per batch (io, capped at half the pool)
        res["threads" if io == 1 else f"threads_io{io}"] = {"copy_pool": gs.copy_threads, "pread_parts": gs.io_parts}
    return res


def latency_of(T, open_fn, pread_fn, close_fn, img, size, count, cache, n, seed):
    import ctypes as C
    err = C.create_string_buffer(80)
    r = T.zsk_tool_open_mem(open_fn, img.ctypes.data, img.size, cache, err)
    if not r:
        return {"error": err.value.decode()}
    rng = np.random.default_rng(seed)
    offs = rng.integers(0, size - count, n + 20).astype(np.uint64)
    ns = np.zeros(n + 20, np.uint64)
    buf = np.empty(count, np.uint8)
    failed = C.c_size_t(0)
    rc = T.zsk_tool_latency(pread_fn, r, offs.ctypes.data, n + 20, count, buf.ctypes.data,
                            ns.ctypes.data, C.byref(failed))
    T.zsk_tool_close_mem(close_fn, r)
    if rc != 0:
        return {"error": f"request {failed.value} failed"}
    us = ns[20:].astype(np.float64) / 1e3    # the first 20 warm the reader
    return {"p50": round(float(np.percentile(us, 50)), 1), "p99": round(float(np.percentile(us, 99)), 1),
            "mean": round(float(us.mean()), 1), "requests": n}


def latency(z, img, size):
    """4 KiB zseek_pread requests at uniformly random offsets of the image
    (each decodes its frame: 64 KiB, or two when it straddles), cache 0 and 1,
    through the drop-in API with a C in-memory pread callback."""
    import ctypes as C
    T, L = z.tools(), z.lib()
    fn = [C.cast(f, C.c_void_p) for f in (L.zseek_reader_open_full, L.zseek_pread, L.zseek_reader_close)]
    return {f"cache{c}": latency_of(T, *fn, img, size, 4096, c, 1000, 7) for c in (0, 1)}


def traffic_from_profile(kernel, workload):
    """HBM bytes per launch from the committed rocprofv3 PMC summary
    (profiles/pmc_traffic*.json, written by scripts/round_profiles.py), used
    only when it was recorded for the kernel this build launches on this same
    workload."""
    if not kernel:
        return None
    for name in ("pmc_traffic.json", "pmc_traffic_zstd.json", "pmc_traffic_lz4c.json", "pmc_traffic_f4096.json",
                 "pmc_traffic_f1048576.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                rec = json.load(f)
        except (OSError, ValueError):
            continue
        if kernel in rec.get("kernel", "") and rec.get("workload") == workload:
            return rec.get("hbm_bytes_per_launch")
    return None


def cpu_baseline(img, size, frame, host, zstd, with_latency):
    """The reference CPU path (oracle/_ref: /root/reference/src compiled
    against liblz4 1.9.3 / libzstd 1.4.9) timed on this host: T independent
    readers over disjoint frame-aligned slices of the same image, in-memory
    pread, cache off, frame-sized zseek_pread calls.  T = 1 and T = every
    usable CPU (affinity and cgroup CPU quota) — `value` and `cores`; when the
    quota is below the visible CPUs, T = all visible CPUs is recorded beside
    it as `oversubscribed` (quota-throttled, never the value)."""
    try:
        from oracle.oracle import REF_SO, RefBench
        rb = RefBench()
    except Exception as e:   # reference build absent
        return {"value": None, "unit": "GB/s", "cores": 0, "kind": "reference",
                "sample": f"unavailable: {e}"}
    usable = host["usable"]
    one = min(size, 1 << 30)
    s1, b1 = rb.run(img, 1, 0, one, frame, frame, 0)

    def best_of(threads, reps=3):
        best = 0.0
        for _ in range(reps):
            secs, nbytes = rb.run(img, threads, 0, size, frame, frame, 0)
            best = max(best, nbytes / secs / 1e9)
        return best

    # value = the CPUs this process may actually run on (affinity and the
    # cgroup quota); T = every visible CPU is recorded beside it only: under a
    # quota those threads share `usable` CPUs' time and measure the quota
    value = best_of(usable)
    res = {"value": round(value, 2), "unit": "GB/s", "cores": usable, "kind": "reference",
           "per_core_GBps": round(value / usable, 3),
           "one_thread_GBps": round(b1 / s1 / 1e9, 2),
           "node_physical_cores": host.get("physical_cores"),
           "sample": (f"{'zstd' if zstd else 'LZ4'}: the whole {size >> 20} MiB image decoded by "
                      f"{usable} reference readers (cache_size=0, {frame >> 10} KiB zseek_pread calls; "
                      f"liblz4 {rb.versions['lz4']} / libzstd {rb.versions['zstd']} in the reference's own "
                      f"link namespace), best of 3; 1 reader on the first {one >> 20} MiB; host "
                      f"{host['model']}: {usable} usable CPUs (affinity {host['affinity']}, cgroup quota "
                      f"{host['cgroup_quota']}) of {host['visible']} visible, "
                      f"{host.get('physical_cores')} physical cores in the node")}
    if host["visible"] > usable:   # informational: every visible CPU, quota-throttled
        res["oversubscribed"] = {"threads": host["visible"], "GBps": round(best_of(host["visible"], 2), 2),
                                 "note": "threads beyond the cgroup quota share the usable CPUs' time"}
    if with_latency:
        import ctypes as C
        import libzseek_amd as z
        T = z.tools()
        from oracle.oracle import ref_cdll
        RL = ref_cdll(REF_SO)
        fn = [C.cast(f, C.c_void_p) for f in (RL.zseek_reader_open_full, RL.zseek_pread,
                                              RL.zseek_reader_close)]
        res["latency_4k_us"] = {f"cache{c}": latency_of(T, *fn, img, size, 4096, c, 1000, 7)
                                for c in (0, 1)}
    return res


if __name__ == "__main__":
    main()
