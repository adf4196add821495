"""Device-lane routing of a multi-frame zseek_pread, on the CPU:
libzseek_amd/csrc/lane_plan.h's pure functions -- the frame shards per lane
and, per batch, the copy route of its decoded bytes (host bounce, same-device
copy, peer copy) plus the pinned download window that also serves the cache.
reader.cpp's run / submit call exactly these (the reference's serialised path
they replace: decompress.c:714-718)."""
from __future__ import annotations

import ctypes as C
import pathlib
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
NONE, HOST, DEVICE, PEER = 0, 1, 2, 3


@pytest.fixture(scope="module")
def lp(tmp_path_factory):
    so = tmp_path_factory.mktemp("lane_plan") / "liblane_plan.so"
    subprocess.run(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Werror", "-o", str(so),
                    str(ROOT / "tests/native/lane_plan_shim.cpp")], check=True)
    L = C.CDLL(str(so))
    L.lp_plan_lanes.restype = C.c_size_t
    L.lp_plan_lanes.argtypes = [C.c_size_t, C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t, C.c_uint64,
                                C.c_void_p, C.c_void_p]
    L.lp_route_batch.restype = None
    L.lp_route_batch.argtypes = [C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_uint64, C.c_void_p, C.c_size_t,
                                 C.c_size_t, C.c_size_t, C.c_void_p]
    return L


def _plan(lp, lanes, offset, end, d_off, per_lane):
    d = np.ascontiguousarray(d_off, np.uint64)
    fa = np.zeros(max(lanes, 1), np.uint64)
    fb = np.zeros(max(lanes, 1), np.uint64)
    n = lp.lp_plan_lanes(lanes, offset, end, d.ctypes.data, len(d) - 1, per_lane, fa.ctypes.data,
                         fb.ctypes.data)
    return [(int(a), int(b)) for a, b in zip(fa[:n], fb[:n])]


def _route(lp, device_dst, dst_dev, lane_dev, offset, end, d_off, f0, f1, cache_cap):
    d = np.ascontiguousarray(d_off, np.uint64)
    out = np.zeros(6, np.uint64)
    lp.lp_route_batch(int(device_dst), dst_dev, lane_dev, offset, end, d.ctypes.data, f0, f1, cache_cap,
                      out.ctypes.data)
    return dict(zip(("route", "dst_off", "src_off", "len", "h_from", "h_len"), (int(x) for x in out)))


F = 65536
D_OFF = [i * F for i in range(4097)]   # 4,096 frames of 64 KiB (256 MiB)


@pytest.mark.parametrize("lanes,offset,end", [(1, 0, 4096 * F), (2, 0, 4096 * F), (8, 1000, 4096 * F - 7),
                                              (3, 5 * F + 17, 900 * F), (8, 0, 3 * F), (4, F - 1, F + 1)])
def test_lanes_cover_the_request_contiguously(lp, lanes, offset, end):
    per_lane = 1 << 20
    sh = _plan(lp, lanes, offset, end, D_OFF, per_lane)
    first, last = offset // F, (end - 1) // F
    assert sh[0][0] == first and sh[-1][1] == last + 1
    for (a, b), (c, _) in zip(sh, sh[1:]):
        assert b == c                                 # contiguous, no frame twice
    assert all(b > a for a, b in sh)                  # no empty lane
    assert len(sh) <= lanes
    assert len(sh) <= max(1, (end - offset) // per_lane)   # >= per_lane bytes each
    if len(sh) > 1:                                   # balanced by decoded bytes
        sizes = [b - a for a, b in sh]
        assert max(sizes) - min(sizes) <= 1 + (last + 1 - first) // len(sh) // 8


def test_lanes_never_empty_with_a_huge_last_frame(lp):
    """Cut points that all fall in the last (huge) frame still leave every
    lane a frame of its own."""
    d_off = [0, 100, 200, 300, 400, 400 + (64 << 20)]
    sh = _plan(lp, 4, 0, d_off[-1], d_off, 1 << 20)
    assert len(sh) == 4
    assert sh[-1][1] == 5 and all(b > a for a, b in sh)
    assert [a for a, _ in sh[1:]] == [b for _, b in sh[:-1]]


def test_route_host_destination(lp):
    r = _route(lp, False, -1, 0, 3 * F + 10, 9 * F - 5, D_OFF, 2, 6, 0)
    assert r["route"] == HOST
    assert (r["dst_off"], r["src_off"], r["len"]) == (0, F + 10, 3 * F - 10)
    assert (r["h_from"], r["h_len"]) == (F + 10, 3 * F - 10)        # only the request's bytes come down
    r = _route(lp, False, -1, 0, 3 * F + 10, 9 * F - 5, D_OFF, 6, 10, 0)
    assert (r["route"], r["dst_off"], r["src_off"], r["len"]) == (HOST, 3 * F - 10, 0, 3 * F - 5)


def test_route_same_device(lp):
    r = _route(lp, True, 1, 1, 0, 100 * F, D_OFF, 10, 20, 0)
    assert (r["route"], r["dst_off"], r["src_off"], r["len"]) == (DEVICE, 10 * F, 0, 10 * F)
    assert r["h_len"] == 0                                            # nothing downloaded


def test_route_peer_device(lp):
    r = _route(lp, True, 0, 3, 7, 100 * F, D_OFF, 0, 5, 0)
    assert (r["route"], r["dst_off"], r["src_off"], r["len"]) == (PEER, 0, 7, 5 * F - 7)
    assert r["h_len"] == 0


def test_route_cache_window(lp):
    """With a cache the batch's last cache_cap frames come down too (they may
    be kept), whatever the destination."""
    r = _route(lp, True, 0, 0, 0, 3 * F, D_OFF, 0, 8, 2)
    assert r["route"] == DEVICE and (r["h_from"], r["h_len"]) == (6 * F, 2 * F)
    r = _route(lp, False, -1, 0, F, 3 * F, D_OFF, 0, 8, 2)            # request part + cached frames
    assert r["route"] == HOST and (r["h_from"], r["h_len"]) == (F, 7 * F)
    r = _route(lp, False, -1, 0, F, 3 * F, D_OFF, 0, 3, 8)            # cache_cap > batch: all frames
    assert (r["h_from"], r["h_len"]) == (0, 3 * F)


def test_route_batch_outside_request(lp):
    r = _route(lp, False, -1, 0, 0, 2 * F, D_OFF, 4, 6, 0)
    assert r["route"] == NONE and r["len"] == 0 and r["h_len"] == 0
