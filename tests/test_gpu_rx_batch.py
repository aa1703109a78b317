"""Batched receive over many sessions (wsg_rx_*) vs the
oracle's per-call PrepareReceiveFrame: every session's streams are fed in the
same interleaved order, and the batch must fire the same callbacks (kind,
payload bytes, status) in the same global order, only later — at each flush.
Splits inside headers included.  Bit-exact; unmask on the GPU."""
import os

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402

OPCODES = [0x81, 0x82, 0x01, 0x02, 0x00, 0x80, 0x88, 0x89, 0x8A, 0xC1, 0x83]


@pytest.fixture(scope="module")
def codec():
    c = ca.Codec(0)
    yield c
    c.close()


def _stream(rng, n, max_len, masked_p=0.7):
    enc = oracle.Session()
    out = []
    for _ in range(n):
        op = int(rng.choice(OPCODES))
        mask = bool(rng.random() < masked_p)
        status = int(rng.integers(-3, 70000)) if rng.random() < 0.3 else 0
        size = int(rng.choice([0, 1, 2, 125, 126, 127, 65535, 65536]) if rng.random() < 0.2
                   else rng.integers(0, max_len))
        enc.set_send_key(int(rng.integers(0, 2**32)))
        out.append(enc.prepare_send(op, mask, rng.integers(0, 256, size, dtype=np.uint8).tobytes(), status))
    return b"".join(out)


def _run(codec, rng, streams, chunk, flush_p, devices=None):
    """Feed `streams` interleaved in random chunks to the oracle (per call) and
    to one RxBatch; return (expected events, batch events)."""
    S = len(streams)
    ref = [oracle.Session() for _ in range(S)]
    prod = [ca.Session(codec) for _ in range(S)]
    index = {id(p): i for i, p in enumerate(prod)}
    rx = ca.RxBatch(codec)
    if devices is not None:
        rx.set_devices(devices)
    pos = [0] * S
    expect = []
    while True:
        live = [i for i in range(S) if pos[i] < len(streams[i])]
        if not live:
            break
        i = int(rng.choice(live))
        n = len(streams[i]) - pos[i] if chunk is None else int(rng.integers(1, chunk))
        part = streams[i][pos[i]: pos[i] + n]
        pos[i] += len(part)
        ref[i].prepare_receive(part)
        expect += [(i,) + e for e in ref[i].events()]
        rx.feed(prod[i], part)
        if rng.random() < flush_p:
            rx.flush()
    rx.flush()
    got = [(index[id(s)], kind, data, status) for s, kind, data, status in rx.events()]
    for i in range(S):
        assert prod[i].required() == ref[i].required()
    rx.close()
    return expect, got


@pytest.mark.parametrize("seed,chunk,flush_p", [(11, None, 0.05), (12, 700, 0.02), (13, 50, 0.3), (14, 4000, 0.0),
                                                (15, 3, 0.01)])
def test_rx_batch_interleaved_vs_oracle(codec, seed, chunk, flush_p):
    rng = np.random.default_rng(seed)
    streams = [_stream(rng, 40, 3000) for _ in range(16)]
    expect, got = _run(codec, rng, streams, chunk, flush_p)
    assert len(expect) > 0
    assert got == expect


@pytest.mark.parametrize("seed,chunk", [(31, None), (32, 700)])
def test_rx_batch_over_devices_vs_oracle(codec, seed, chunk, monkeypatch):
    """Flushes spread over several contexts (wsg_rx_set_devices; two of the
    one GPU, split as distinct GPUs would be): the same callbacks in the same
    order."""
    monkeypatch.setenv("WSG_HOST_MULTI_SHARE", "1")
    rng = np.random.default_rng(seed)
    streams = [_stream(rng, 40, 20000) for _ in range(16)]
    expect, got = _run(codec, rng, streams, chunk, 0.05, devices=[0, 0, 0])
    assert len(expect) > 0
    assert got == expect


@pytest.mark.parametrize("seed", range(int(os.environ.get("WSG_FUZZ_SEEDS", 10))))
def test_rx_batch_fuzz_vs_oracle(codec, seed):
    """Random session counts, frame mixes, read sizes (down to 1 byte, so
    headers split anywhere: SURVEY Q7) and flush points; $WSG_FUZZ_SEEDS
    widens the run."""
    rng = np.random.default_rng(5000 + seed)
    chunk = [None, 2, 9, 200, 3000][int(rng.integers(0, 5))]
    # every read is one Python call: the smaller the reads, the smaller the frames
    sizes = {None: [10, 300, 5000, 70000], 3000: [10, 300, 5000, 70000], 200: [10, 300, 5000]}.get(chunk, [10, 300])
    streams = [_stream(rng, int(rng.integers(1, 30)), int(rng.choice(sizes)))
               for _ in range(int(rng.integers(1, 24)))]
    expect, got = _run(codec, rng, streams, chunk, float(rng.choice([0.0, 0.01, 0.2])))
    assert got == expect


def test_rx_batch_large_frames_vs_oracle(codec):
    """Whole 64 KiB-class frames from many sessions: the copy-through fast path."""
    rng = np.random.default_rng(21)
    streams = []
    for _ in range(64):
        enc = oracle.Session(int(rng.integers(1, 2**32)))
        streams.append(b"".join(enc.prepare_send(0x82, True, rng.integers(0, 256, int(rng.integers(60000, 70000)),
                                                                          dtype=np.uint8).tobytes())
                                for _ in range(4)))
    expect, got = _run(codec, rng, streams, None, 0.0)
    assert len(expect) == 256 and got == expect


def test_rx_batch_fragments_across_flushes(codec):
    """A message split over three frames, each in a different flush; a
    continuation (opcode 0) after a completed message keeps the old opcode."""
    enc = oracle.Session(0x0A0B0C0D)
    frames = [enc.prepare_send(0x01, True, b"hel"), enc.prepare_send(0x00, True, b"lo "),
              enc.prepare_send(0x80, True, b"world"), enc.prepare_send(0x80, True, b"again")]
    ref, prod = oracle.Session(), ca.Session(codec)
    rx = ca.RxBatch(codec)
    for f in frames:
        ref.prepare_receive(f)
        rx.feed(prod, f)
        rx.flush()
    assert [e[1:] for e in rx.events()] == ref.events() == [(1, b"hello world", 0), (1, b"again", 0)]


def test_rx_batch_clear_in_order(codec):
    """ClearWSBuffers between queued frames: the pending fragment is dropped at
    that point of the delivery order, as the per-call path drops it."""
    enc = oracle.Session(0x01020304)
    a, b, c = (enc.prepare_send(0x02, True, b"frag"), enc.prepare_send(0x80, True, b"tail"),
               enc.prepare_send(0x81, True, b"next"))
    ref, prod = oracle.Session(), ca.Session(codec)
    rx = ca.RxBatch(codec)
    ref.prepare_receive(a)
    rx.feed(prod, a)
    ref.clear()
    rx.clear(prod)
    for f in (b, c):
        ref.prepare_receive(f)
        rx.feed(prod, f)
    assert rx.pending() == (3, len(a) + len(b) + len(c))
    assert rx.flush() == 3
    assert [e[1:] for e in rx.events()] == ref.events()


def test_rx_batch_forget_and_split_header(codec):
    """A forgotten session's queued frames are dropped; a header split inside
    its key field misparses exactly as the per-call path does."""
    enc = oracle.Session(0x11223344)
    f1 = enc.prepare_send(0x82, True, bytes(range(200)))
    f2 = enc.prepare_send(0x81, True, b"x" * 10)
    keep, gone = ca.Session(codec), ca.Session(codec)
    ref = oracle.Session()
    rx = ca.RxBatch(codec)
    for part in (f1[:5], f1[5:], f2):
        ref.prepare_receive(part)
        rx.feed(keep, part)
    rx.feed(gone, f2)
    rx.forget(gone)
    rx.flush()
    ev = rx.events()
    assert all(s is keep for s, *_ in ev)
    assert [e[1:] for e in ev] == ref.events()


def test_rx_batch_empty_flush(codec):
    rx = ca.RxBatch(codec)
    assert rx.pending() == (0, 0)
    assert rx.flush() == 0
    s = ca.Session(codec)
    rx.feed(s, bytes([0x81, 0x85, 1, 2]))   # half a header: nothing complete yet
    assert rx.pending() == (0, 0)
    assert rx.flush() == 0 and rx.events() == []
    assert s.required() == 2


def test_rx_batch_repeated_large_rounds(codec):
    """Several flush rounds of 256 sessions x 4 frames of ~64 KiB read in
    ~16 KiB pieces (multi-segment host decode every round; the batch's pinned
    buffers are reused and grown across rounds): every message byte-exact."""
    rng = np.random.default_rng(41)
    S = 256
    prod = [ca.Session(codec) for _ in range(S)]
    ref = [oracle.Session() for _ in range(S)]
    index = {id(p): i for i, p in enumerate(prod)}
    rx = ca.RxBatch(codec)
    for rnd in range(3):
        streams = []
        for _ in range(S):
            enc = oracle.Session(int(rng.integers(1, 2**32)))
            streams.append(b"".join(enc.prepare_send(0x82, True, rng.integers(0, 256, int(rng.integers(60000, 70000)),
                                                                              dtype=np.uint8).tobytes())
                                    for _ in range(4)))
        expect = []
        pos = [0] * S
        while True:
            live = [i for i in range(S) if pos[i] < len(streams[i])]
            if not live:
                break
            for i in live:
                part = streams[i][pos[i]: pos[i] + int(rng.integers(8000, 24000))]
                pos[i] += len(part)
                ref[i].prepare_receive(part)
                expect += [(i,) + e for e in ref[i].events()]
                rx.feed(prod[i], part)
        assert rx.flush() == 4 * S
        got = [(index[id(s)], kind, data, status) for s, kind, data, status in rx.events()]
        assert got == expect, "round %d" % rnd
    rx.close()
