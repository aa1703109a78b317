"""Runs the C++ API test program (tests/cpp/test_ws_api.cpp) on the GPU box:
WSClient / WSSession / WSServer scenarios of the reference tests/test_ws.cpp."""
import json
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "test_ws_api")


def test_cpp_ws_api():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


def test_concurrent_context_creation():
    """Eight threads released together each create a context and decode one
    host batch on it (tests/cpp/test_concurrent_create.cpp), in a fresh
    process: every context made, every batch exact."""
    exe = os.path.join(ROOT, "tests", "cpp", "_build", "test_concurrent_create")
    assert os.path.exists(exe), "build tests/cpp first"
    r = subprocess.run([exe, "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr[-2000:]


@pytest.mark.parametrize("mode,clients,threads", [("per_read", 1, 1), ("tick", 8, 1), ("per_read", 8, 2),
                                                  ("per_call", 1, 1)])
def test_echo_c1_modes(mode, clients, threads):
    """BASELINE config C1 through the drop-in API (tools/bench_echo): every
    echoed zero-byte message comes back as zero bytes after the client's GPU
    mask and the server's GPU unmask, in every batching mode."""
    exe = os.path.join(ROOT, "tools", "_build", "bench_echo")
    assert os.path.exists(exe), "build tools first: make -C tools"
    r = subprocess.run([exe, mode, str(clients), str(threads), "100", "32", "0.5"], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["payload_ok"] is True
    assert d["total_messages"] >= clients * 100
