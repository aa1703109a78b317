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


def test_per_call_path_on_the_lane_vs_oracle():
    """The per-call path (PrepareSendFrame / PrepareReceiveFrame outside a
    batch scope: what `Send*Async` from a non-IO thread and every sync `Send*`
    run, reference examples/ws_chat_client.cpp:131) through the C-ABI's
    per-connection codec: every masked payload is one task on the device's
    lane (the context's lane request count grows by one per masked payload),
    and every frame and every receive callback equals the oracle's.  Payloads
    of 0-80 bytes (inline in the task up to 40) and up to 70 KB (staged; over
    64 KiB the launch path)."""
    import numpy as np

    import cppserver_amd as ca
    import oracle

    rng = np.random.default_rng(77)
    codec = ca.Codec(0)
    try:
        prod, ref = ca.Session(codec), oracle.Session()
        rx_p, rx_r = ca.Session(codec), oracle.Session()
        r0, _, _ = codec.lane_stats()
        masked = 0
        for i in range(400):
            n = int(rng.integers(0, 81)) if i % 4 else int(rng.choice([300, 4000, 65536, 70000]))
            payload = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            key = int(rng.integers(1, 2**32))
            op = int(rng.choice([0x81, 0x82, 0x89, 0x8A, 0x88]))
            status = 1000 if op == 0x88 else 0
            prod.set_send_key(key)
            ref.set_send_key(key)
            frame = prod.prepare_send(op, True, payload, status)
            assert frame == ref.prepare_send(op, True, payload, status), i
            rx_p.prepare_receive(frame)
            rx_r.prepare_receive(frame)
            assert rx_p.events() == rx_r.events(), i
            _, h = ca.header_unpack(frame)
            body = len(frame) - int(h["hdr_len"])
            if 0 < body <= 65536:
                masked += 2   # the send's mask and the receive's unmask
        r1, _, _ = codec.lane_stats()
        assert r1 - r0 == masked, (r1 - r0, masked)
    finally:
        codec.close()
