"""Batched send (wsg_tx_*) and the host-staged batch
encode under it (wsg_encode_batch_host) vs the oracle's per-call
PrepareSendFrame: every frame byte-identical, handed out in queue order.
Bit-exact; header pack + mask on the GPU."""
import os

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
from cppserver_amd.layout import SEND_DESC  # noqa: E402

OPCODES = [0x81, 0x82, 0x01, 0x02, 0x00, 0x80, 0x88, 0x89, 0x8A, 0xC1, 0x83]


@pytest.fixture(scope="module")
def codec():
    c = ca.Codec(0)
    yield c
    c.close()


def _oracle_frames(payload, desc):
    s = oracle.Session()
    out = []
    for d in desc:
        s.set_send_key(int(d["key"]))
        p = payload[int(d["src_off"]): int(d["src_off"]) + int(d["len"])].tobytes()
        out.append(s.prepare_send(int(d["opcode"]), bool(d["mask"]), p, int(d["status"])))
    return out


@pytest.mark.parametrize("stage_mb", [None, "1"])
def test_encode_batch_host_vs_oracle(codec, stage_mb):
    """Ragged frames, segmented (1 MiB segments cut the batch into many)."""
    rng = np.random.default_rng(31)
    lens = rng.integers(0, 70000, 300)
    lens[:8] = [0, 1, 125, 126, 65535, 65536, 2, 3]
    desc, total = wl.ragged_desc(rng, lens)
    desc["opcode"] = rng.choice(OPCODES, len(desc))
    desc["mask"] = rng.random(len(desc)) < 0.7
    desc["status"] = np.where(rng.random(len(desc)) < 0.3, rng.integers(-3, 70000, len(desc)), 0)
    payload = wl.random_bytes(rng, max(total, 1))
    old = os.environ.get("WSG_STAGE_MB")
    if stage_mb:
        os.environ["WSG_STAGE_MB"] = stage_mb
    try:
        rc, wire, off = codec.encode_batch_host(payload, desc)
    finally:
        if stage_mb:
            if old is None:
                del os.environ["WSG_STAGE_MB"]
            else:
                os.environ["WSG_STAGE_MB"] = old
    assert rc == 0
    ref = _oracle_frames(payload, desc)
    assert off[-1] == sum(len(f) for f in ref)
    assert wire.tobytes() == b"".join(ref)


def test_encode_batch_host_scattered_and_pinned(codec):
    """Descriptors out of order and reusing payload (gather path); pinned and
    pageable output buffers give the same bytes."""
    rng = np.random.default_rng(32)
    payload = wl.random_bytes(rng, 1 << 20)
    n = 500
    desc = np.zeros(n, dtype=SEND_DESC)
    desc["len"] = rng.integers(0, 4000, n)
    desc["src_off"] = [int(rng.integers(0, len(payload) - L + 1)) for L in desc["len"]]
    desc["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    desc["opcode"] = 0x82
    desc["mask"] = 1
    ref = b"".join(_oracle_frames(payload, desc))
    rc, wire, _ = codec.encode_batch_host(payload, desc)
    assert rc == 0 and wire.tobytes() == ref
    pinned = ca.pinned_empty(len(ref) + 16)
    rc, wire2, _ = codec.encode_batch_host(payload, desc, wire=pinned)
    assert rc == 0 and wire2.tobytes() == ref


def test_encode_batch_host_errors(codec):
    desc = np.zeros(1, dtype=SEND_DESC)
    desc["len"] = 10
    desc["src_off"] = 5
    rc, _, _ = codec.encode_batch_host(np.zeros(8, np.uint8), desc)      # payload range past the end
    assert rc == ca.WSG_EINVAL
    desc["src_off"] = 0
    rc, _, _ = codec.encode_batch_host(np.zeros(16, np.uint8), desc, wire=np.zeros(4, np.uint8))
    assert rc == ca.WSG_ENOMEM


@pytest.mark.parametrize("devices", [None, [0, 0, 0]])
def test_tx_batch_vs_oracle(codec, devices, monkeypatch):
    """Many sessions with their own keys queue random frames; one flush hands
    back every frame in queue order, each equal to the per-call encode (also
    with the flush spread over several contexts, wsg_tx_set_devices)."""
    monkeypatch.setenv("WSG_HOST_MULTI_SHARE", "1")
    rng = np.random.default_rng(33)
    S = 20
    sessions = [ca.Session(codec, int(rng.integers(0, 2**32))) for _ in range(S)]
    refs = [oracle.Session() for _ in range(S)]
    tx = ca.TxBatch(codec)
    if devices is not None:
        tx.set_devices(devices)
    expect = []
    for _ in range(400):
        i = int(rng.integers(0, S))
        op = int(rng.choice(OPCODES))
        mask = bool(rng.random() < 0.7)
        status = int(rng.integers(-3, 70000)) if rng.random() < 0.3 else 0
        size = int(rng.choice([0, 1, 125, 126, 65535, 65536]) if rng.random() < 0.2 else rng.integers(0, 5000))
        p = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        if rng.random() < 0.05:   # a key change between frames (Handshaked on reconnect)
            k = int(rng.integers(0, 2**32))
            sessions[i].set_send_key(k)
        refs[i].set_send_key(_key_of(sessions[i]))
        expect.append((i, refs[i].prepare_send(op, mask, p, status)))
        tx.queue(sessions[i], op, mask, p, status)
    assert tx.pending()[0] == 400
    got = tx.flush()
    index = {id(s): i for i, s in enumerate(sessions)}
    assert [(index[id(s)], f) for s, f in got] == expect
    assert tx.pending() == (0, 0) and tx.flush() == []


@pytest.mark.parametrize("seed", range(int(os.environ.get("WSG_FUZZ_SEEDS", 50))))
def test_tx_batch_fuzz_vs_oracle(codec, seed):
    """Random session counts, frame mixes and flush points (several flushes
    per run), key changes between frames: every flush hands back its frames
    in queue order, each the per-call encode's bytes.  $WSG_FUZZ_SEEDS
    widens the run."""
    rng = np.random.default_rng(9000 + seed)
    S = int(rng.integers(1, 40))
    sessions = [ca.Session(codec, int(rng.integers(0, 2**32))) for _ in range(S)]
    refs = [oracle.Session() for _ in range(S)]
    index = {id(s): i for i, s in enumerate(sessions)}
    tx = ca.TxBatch(codec)
    big = float(rng.choice([0.0, 0.02, 0.2]))
    expect = []
    for _ in range(int(rng.integers(1, 600))):
        i = int(rng.integers(0, S))
        op = int(rng.choice(OPCODES))
        mask = bool(rng.random() < 0.7)
        status = int(rng.integers(-3, 70000)) if rng.random() < 0.3 else 0
        size = int(rng.integers(65536, 200000)) if rng.random() < big else int(rng.integers(0, 3000))
        p = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        if rng.random() < 0.05:
            sessions[i].set_send_key(int(rng.integers(0, 2**32)))
        refs[i].set_send_key(_key_of(sessions[i]))
        expect.append((i, refs[i].prepare_send(op, mask, p, status)))
        tx.queue(sessions[i], op, mask, p, status)
        if rng.random() < 0.03:
            got = tx.flush()
            assert [(index[id(s)], f) for s, f in got] == expect
            expect = []
    got = tx.flush()
    assert [(index[id(s)], f) for s, f in got] == expect


def _key_of(session):
    """The session's current send key, read back through one encoded frame."""
    f = session.prepare_send(0x82, True, b"")
    return int.from_bytes(f[2:6], "little")


def test_tx_batch_forget(codec):
    a, b = ca.Session(codec, 1), ca.Session(codec, 2)
    tx = ca.TxBatch(codec)
    tx.queue(a, 0x81, True, b"one")
    tx.queue(b, 0x81, True, b"two")
    tx.queue(a, 0x81, True, b"three")
    tx.forget(a)
    got = tx.flush()
    assert len(got) == 1 and got[0][0] is b
    assert got[0][1] == oracle.Session(2).prepare_send(0x81, True, b"two")
