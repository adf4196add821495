"""Config 4's multi-rank HIP path on the one-GPU test box.

`python bench.py --gpus 2` starts two rank processes itself, exactly as the
driver's multi-GPU run does; with ZSEEK_BENCH_SHARE_GPU=1 both ranks decode
their shard of a fixed total on device 0 with the real HIP kernels and
reassemble the full range over gloo (RCCL refuses two ranks on one device).
Each rank verifies its decoded shard against the generator and the full
range after the all-gatherv (and, round-robin, the permute back to frame
order).  The reference path this replaces is the serialised frame loop of
/root/reference/src/decompress.c:714-718."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("partition", ["contiguous", "round_robin"])
def test_bench_two_ranks_share_gpu(gpu, partition):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["ZSEEK_BENCH_SHARE_GPU"] = "1"
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--total-size", "512M", "--size", "256M", "--steps", "2", "--warmup", "1",
                        "--partition", partition, "--no-cpu-baseline", "--no-e2e", "--no-latency",
                        "--threads", "8"],
                       capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["decoded_bytes_total"] == 512 << 20
    assert d["config"]["frames_per_gpu"] == 4096
    assert d["verified_bit_exact"] is True
    rs = d["reassembly"]
    assert rs["full_range_matches_generator"] is True
    assert rs["bytes_total"] == 512 << 20
    assert "gloo" in rs["method"]
    assert (rs["permute_s"] is not None) == (partition == "round_robin")
