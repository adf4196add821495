"""The library's fallback switches: each one, set before the
first GPU call of a fresh process, must give the default path's bytes and
error strings on the single-frame read cases of tests/env_switch_probe.py.

  ZSEEK_HOST_DMA=1    uploads / downloads by DMA copies instead of the
                      small-batch I/O kernels (reader.cpp, host_io.hip)
  ZSEEK_ONE_FUSE=0    zstd one-frame route: the Huffman kernel on the side
                      stream instead of zstd_one_kernel
  ZSEEK_FRAME_HELP=0  zstd one-frame route: no helper wave in the frame kernel
  ZSEEK_ONE_WAVES=4   LZ4 one-frame parse over four waves (round 4's shape)
  ZSEEK_ONE_ROUTE=0   no one-frame route (the throughput kernels)
  ZSEEK_ONE_BIG=0     one-frame route, frames over 64 KiB: one sequential
                      parse and the wave execute (round 5) instead of the
                      job parse and the block-parallel execute
  ZSEEK_ONE_BLOCKS=0  ... the job parse, but the windowed execute
                      (seq_exec_big_kernel) instead of the block-parallel one
  ZSEEK_DONE_FLAG=0   a small batch's completion by the stream's event only
                      (no pinned completion word, no results posted by the
                      one-frame execute)
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))

SWITCHES = ["ZSEEK_HOST_DMA=1", "ZSEEK_ONE_FUSE=0", "ZSEEK_FRAME_HELP=0", "ZSEEK_ONE_WAVES=4",
            "ZSEEK_ONE_ROUTE=0", "ZSEEK_ONE_BIG=0", "ZSEEK_ONE_BLOCKS=0", "ZSEEK_DONE_FLAG=0"]


def _probe(env_kv=None):
    env = dict(os.environ)
    if env_kv:
        k, v = env_kv.split("=")
        env[k] = v
    p = subprocess.run([sys.executable, os.path.join(HERE, "env_switch_probe.py")], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.fixture(scope="module")
def default_answers(gpu):
    return _probe()


@pytest.mark.gpu
@pytest.mark.parametrize("switch", SWITCHES)
def test_switch_matches_default_path(gpu, default_answers, switch):
    got = _probe(switch)
    assert got.keys() == default_answers.keys()
    bad = [k for k in got if got[k] != default_answers[k]]
    assert not bad, (switch, bad[:5], [got[k] for k in bad[:3]], [default_answers[k] for k in bad[:3]])
