"""WebSocket upgrade handshake (reference ws.cpp:26-210),
host-only: the Sec-WebSocket-Accept known answer of RFC 6455 §1.3 through the
C-ABI, and the C++ handshake program (tests/cpp/test_handshake.cpp) — HTTP
subset round trips, the reference's accept/reject rules and error texts, a
full client/session upgrade over an in-memory transport.  No GPU involved:
the upgrade carries no WebSocket frames."""
import ctypes
import os
import subprocess

import cppserver_amd as ca

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "_build", "test_handshake")


def _accept(key):
    L = ca.lib()
    f = L.wsg_ws_accept
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t]
    out = ctypes.create_string_buffer(29)
    assert f(key, len(key), out, 29) == 0
    return out.value


def test_rfc6455_accept_known_answer():
    assert _accept(b"dGhlIHNhbXBsZSBub25jZQ==") == b"s3pPLMBiTxaQ9kYGzzhZRbK+xOo="


def test_accept_matches_python_sha1():
    import base64
    import hashlib

    for key in [b"", b"x", b"AQIDBAUGBwgJCgsMDQ4PEA=="]:
        want = base64.b64encode(hashlib.sha1(key + b"258EAFA5-E914-47DA-95CA-C5AB0DC85B11").digest())
        assert _accept(key) == want


def test_cpp_handshake_program():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp")], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
