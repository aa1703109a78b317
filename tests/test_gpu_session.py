"""Per-connection codec (wsg_session_*, the reference WebSocket mix-in) vs the
oracle session: PrepareSendFrame bytes, PrepareReceiveFrame callbacks and
RequiredReceiveFrameSize, on known answers and on random split streams.
Bit-exact; the payload XOR runs on the GPU."""
import numpy as np
import pytest

import oracle
from tests import kat

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402

KAT = kat.load()
OPCODES = [0x81, 0x82, 0x01, 0x02, 0x00, 0x80, 0x88, 0x89, 0x8A, 0xC1, 0x83]


@pytest.fixture(scope="module")
def codec():
    c = ca.Codec(0)
    yield c
    c.close()


@pytest.mark.parametrize("v", KAT["encode"], ids=lambda v: v["name"])
def test_session_encode_kat(codec, v):
    s = ca.Session(codec, kat.key_of(v))
    out = s.prepare_send(v["opcode"], v["mask"], kat.payload_of(v), v["status"])
    if "expect" in v:
        assert out.hex() == v["expect"], v["source"]
    else:
        assert out[: len(v["expect_prefix"]) // 2].hex() == v["expect_prefix"]
        assert len(out) == v["expect_len"]


@pytest.mark.parametrize("v", KAT["decode"], ids=lambda v: v["name"])
def test_session_decode_kat(codec, v):
    s = ca.Session(codec)
    for c in v["chunks"]:
        s.prepare_receive(bytes.fromhex(c))
    assert s.events() == kat.events_of(v), v["source"]


@pytest.mark.parametrize("v", KAT["roundtrip"], ids=lambda v: v["name"])
def test_session_roundtrip_kat(codec, v):
    tx = ca.Session(codec, kat.key_of(v))
    rx = ca.Session(codec)
    rx.prepare_receive(tx.prepare_send(v["opcode"], v["mask"], kat.payload_of(v), v["status"]))
    assert rx.events() == kat.events_of(v), v["source"]


@pytest.mark.parametrize("v", KAT["split"], ids=lambda v: v["name"])
def test_session_split_quirk_kat(codec, v):
    payload = kat.payload_of(v)
    frame = ca.Session(codec, kat.key_of(v)).prepare_send(v["opcode"], True, payload)
    for k in v["wrong_at"] + v["correct_at"]:
        rx = ca.Session(codec)
        rx.prepare_receive(frame[:k])
        rx.prepare_receive(frame[k:])
        ok = [e[1] for e in rx.events()] == [payload]
        assert ok == (k in v["correct_at"]), k


def _random_frames(rng, n, max_len):
    frames = []
    for _ in range(n):
        op = int(rng.choice(OPCODES))
        mask = bool(rng.random() < 0.7)
        key = int(rng.integers(0, 2**32))
        status = int(rng.integers(-3, 70000)) if rng.random() < 0.3 else 0
        size = int(rng.choice([0, 1, 2, 3, 5, 125, 126, 127, 300, 65535, 65536, 70000]) if rng.random() < 0.3
                   else rng.integers(0, max_len))
        frames.append((op, mask, key, status, rng.integers(0, 256, size, dtype=np.uint8).tobytes()))
    return frames


def test_session_encode_random_vs_oracle(codec):
    rng = np.random.default_rng(100)
    prod, ref = ca.Session(codec), oracle.Session()
    for op, mask, key, status, payload in _random_frames(rng, 300, 5000):
        prod.set_send_key(key)
        ref.set_send_key(key)
        assert prod.prepare_send(op, mask, payload, status) == ref.prepare_send(op, mask, payload, status)


@pytest.mark.parametrize("seed,whole", [(1, True), (2, False), (3, False), (4, False)])
def test_session_stream_vs_oracle(codec, seed, whole):
    """A stream of frames delivered in random chunks: same callbacks, same
    final state.  Splits inside headers misparse identically."""
    rng = np.random.default_rng(seed)
    enc = oracle.Session()
    stream = b""
    for op, mask, key, status, payload in _random_frames(rng, 200, 3000):
        enc.set_send_key(key)
        stream += enc.prepare_send(op, mask, payload, status)
    prod, ref = ca.Session(codec), oracle.Session()
    at = 0
    while at < len(stream):
        n = len(stream) - at if whole else int(rng.integers(1, 700))
        chunk = stream[at: at + n]
        at += n
        prod.prepare_receive(chunk)
        ref.prepare_receive(chunk)
        assert prod.events() == ref.events()
        assert prod.required() == ref.required()


def test_session_required_framing_vs_oracle(codec):
    """The sync Receive* framing loop (ws_client.cpp:139-151) on both."""
    rng = np.random.default_rng(9)
    enc = oracle.Session()
    frames = []
    for op, mask, key, status, payload in _random_frames(rng, 100, 2000):
        enc.set_send_key(key)
        frames.append(enc.prepare_send(op, mask, payload, status))
    stream = b"".join(frames)
    prod, ref = ca.Session(codec), oracle.Session()
    at = 0
    while at < len(stream):
        r = prod.required()
        assert r == ref.required()
        if r == 0:
            prod.prepare_receive(b"")
            ref.prepare_receive(b"")
            continue
        prod.prepare_receive(stream[at: at + r])
        ref.prepare_receive(stream[at: at + r])
        at += r
        assert prod.events() == ref.events()


def test_session_clear(codec):
    s = ca.Session(codec, 0x11223344)
    s.prepare_receive(bytes([0x81, 0x85, 1, 2]))    # half a header
    s.clear()
    assert s.required() == 2
    assert s.prepare_send(0x82, True, b"ab") == bytes([0x82, 0x82, 0, 0, 0, 0, 0x61, 0x62])
