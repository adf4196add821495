"""Shared fixtures.  `-m "not gpu"` runs everywhere; `-m gpu` needs an MI355X.

The oracle (oracle/) is used here only as the checker.
"""
from __future__ import annotations

import hashlib
import importlib.util
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


def sha(b) -> str:
    return hashlib.sha256(bytes(b)).hexdigest()


def _load_make_golden():
    spec = importlib.util.spec_from_file_location("make_golden",
                                                  os.path.join(GOLDEN, "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def make_golden():
    return _load_make_golden()


@pytest.fixture(scope="session")
def oracle():
    from oracle.oracle import Oracle
    return Oracle()


@pytest.fixture(scope="session")
def ref():
    """The reference library itself, when its out-of-tree build exists."""
    from oracle.oracle import REF_SO, RefZseek
    if not os.path.exists(REF_SO):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    return RefZseek()


@pytest.fixture(scope="session")
def zs():
    import libzseek_amd.zseek as z
    z.lib()
    return z


def golden_file(name: str) -> bytes:
    with open(os.path.join(GOLDEN, name + ".zs"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def payloads(golden, make_golden, oracle):
    """Decoded content of every golden file, regenerated from its recipe."""
    out = {}
    for name, entry in golden["files"].items():
        data = make_golden.payload(entry["payload"], oracle)
        assert sha(data) == entry["payload_sha256"], name
        out[name] = data
    return out


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(autouse=True)
def _hang_dump(request):
    """A GPU test still running after 120 s is taken to be hung: every
    thread's Python stack is printed, then the main thread gets SIGABRT, whose
    handler (the `gpu` fixture's) prints the native stack it is stuck in."""
    if request.node.get_closest_marker("gpu") is None:
        yield
        return
    import faulthandler
    import signal
    import threading
    main = threading.main_thread().ident

    def _fire():
        faulthandler.dump_traceback(all_threads=True)
        signal.pthread_kill(main, signal.SIGABRT)

    t = threading.Timer(120.0, _fire)
    t.daemon = True
    t.start()
    try:
        yield
    finally:
        t.cancel()


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    import torch
    # a crash in native code prints its native stack too (then pytest's own
    # Python traceback)
    from libzseek_amd import zseek
    zseek.tools().zsk_tool_install_backtrace()
    return torch.device("cuda", 0)
