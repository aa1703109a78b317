"""Differential fuzz of the HIP path against the oracle (the CPU restatement
of ws.cpp:212-498): 150 seeded random batches, each drawing its own frame
count, payload-length class mix (0, 1-125, 126-65535, 65536+ header
classes), opcodes (text/binary/continuation/close/ping/pong, RSV bits,
unknown), mask flags, close statuses and misaligned sources.  Every batch
goes through the device encode (piece or small-frame kernel, whichever the
batch selects) and decode, out of place and in place, and through the
host-staged pair (pageable buffers: the staged pipeline; page-locked
buffers: the direct path of small batches); bytes, offsets, per-frame fields and status must equal the
oracle's; every third batch is also decoded with a few wire bytes
overwritten or the wire cut short.  Bit-exact, no tolerance.
$WSG_FUZZ_SEEDS widens the run."""
import os

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
from tests.test_gpu_parity import INFO_FIELDS, gpu_decode, gpu_encode  # noqa: E402

OPCODES = [0x81, 0x82, 0x01, 0x02, 0x00, 0x80, 0x88, 0x89, 0x8A, 0xC2, 0x83, 0x8F, 0x08]
CLASSES = [(0, 0), (1, 125), (126, 65535), (65536, 200000)]


@pytest.fixture(scope="module")
def codec():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    c = ca.Codec(0)
    yield c
    c.close()


def _batch(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([1, 2, 7, 64, 300, 1500, 5000]))
    weights = rng.dirichlet(np.ones(len(CLASSES)))
    cls = rng.choice(len(CLASSES), n, p=weights)
    if n > 500:   # keep the large class rare in big batches (seconds of oracle time)
        cls[(cls == 3) & (rng.random(n) < 0.95)] = 2
    lens = np.array([rng.integers(CLASSES[c][0], CLASSES[c][1] + 1) for c in cls], dtype=np.int64)
    desc, total = wl.ragged_desc(rng, lens)
    desc["opcode"] = rng.choice(OPCODES, n)
    desc["mask"] = rng.random(n) < rng.random()
    desc["status"] = np.where(rng.random(n) < 0.25, rng.integers(-3, 70000, n), 0)
    desc["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    desc["src_off"] += rng.integers(0, 16, n).astype(np.uint64)
    payload = wl.random_bytes(rng, total + 16)
    return payload, desc


@pytest.mark.parametrize("seed", range(int(os.environ.get("WSG_FUZZ_SEEDS", 150))))
def test_fuzz_encode_decode_vs_oracle(codec, seed):
    payload, desc = _batch(1000 + seed)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    rc, wire, off = gpu_encode(codec, payload, desc)
    assert rc == 0
    assert np.array_equal(off, off_o)
    assert np.array_equal(wire, wire_o)
    fs = off_o[:-1].copy()
    rc_o, out_o, info_o = oracle.decode_batch(wire_o, fs)
    for inplace in (False, True):
        rc_g, out_g, info_g = gpu_decode(codec, wire_o, fs, inplace=inplace)
        assert rc_g == rc_o
        assert np.array_equal(out_g, out_o)
        for f in INFO_FIELDS:
            assert np.array_equal(info_g[f], info_o[f]), f
    # the host-staged pair on the same batch (pageable buffers)
    rc_h, wire_h, off_h = codec.encode_batch_host(payload, desc)
    assert rc_h == 0 and np.array_equal(wire_h, wire_o) and np.array_equal(off_h, off_o)
    rc_h, out_h, info_h = codec.decode_batch_host(wire_o, fs)
    assert rc_h == rc_o and np.array_equal(out_h, out_o)
    for f in INFO_FIELDS:
        assert np.array_equal(info_h[f], info_o[f]), f
    # and with page-locked buffers both ways: batches up to 4 MiB take the
    # direct path (the kernels read and write the host buffers in place)
    pin_p = ca.pinned_empty(len(payload))
    pin_p[:] = payload
    pin_w = ca.pinned_empty(max(len(wire_o), 1))
    rc_h, wire_h, off_h = codec.encode_batch_host(pin_p, desc, wire=pin_w)
    assert rc_h == 0 and np.array_equal(wire_h, wire_o) and np.array_equal(off_h, off_o)
    pin_in, pin_out = ca.pinned_empty(max(len(wire_o), 1)), ca.pinned_empty(max(len(wire_o), 1))
    pin_in[: len(wire_o)] = wire_o
    rc_h, out_h, info_h = codec.decode_batch_host(pin_in[: len(wire_o)], fs, out=pin_out)
    assert rc_h == rc_o and np.array_equal(out_h, out_o)
    for f in INFO_FIELDS:
        assert np.array_equal(info_h[f], info_o[f]), f
    # every third seed: a few wire bytes overwritten (headers broken, lengths
    # running into the next frame or past the wire) or the wire cut short,
    # the same frame table: status, bytes and records through the device
    # decode and both host paths (the lane, the launch path's latch, the
    # staged pipeline) against the oracle
    if seed % 3 == 0 and len(wire_o):
        rng = np.random.default_rng(7000 + seed)
        bad = wire_o.copy()
        for q in rng.integers(0, len(bad), int(rng.integers(1, 4))):
            bad[q] = rng.integers(0, 256)
        if rng.random() < 0.3:
            bad = bad[: int(rng.integers(0, len(bad)))]
        rc_b, out_b, info_b = oracle.decode_batch(bad, fs)
        got = [gpu_decode(codec, bad, fs, inplace=False), codec.decode_batch_host(bad, fs)]
        if len(bad):
            pin_in[: len(bad)] = bad
            got.append(codec.decode_batch_host(pin_in[: len(bad)], fs, out=pin_out))
        for rc_g, out_g, info_g in got:
            assert rc_g == rc_b
            assert np.array_equal(out_g[: len(bad)], out_b)
            for f in INFO_FIELDS:
                assert np.array_equal(info_g[f], info_b[f]), f


@pytest.mark.parametrize("seed", range(int(os.environ.get("WSG_FUZZ_SEEDS", 60))))
def test_fuzz_fanout_vs_oracle(codec, seed):
    """Fan-out (wsg_fanout_encode): random payload length (every length class,
    frame sizes on and off the period path), key count, opcode, mask flag and
    source alignment; every frame vs the oracle, nothing written past the
    last frame."""
    rng = np.random.default_rng(7000 + seed)
    length = int(rng.choice([int(rng.integers(0, 126)), int(rng.integers(126, 9000)),
                             int(rng.integers(60000, 70000))]))
    k = int(rng.integers(1, 3000 if length < 9000 else 60))
    opcode = int(rng.choice(OPCODES))
    mask = bool(rng.random() < 0.8)
    src_off = int(rng.integers(0, 16))
    payload, keys = wl.c4_fanout(length, k, seed=seed)
    ref = oracle.fanout_encode(payload, keys, opcode, mask)
    buf = np.zeros(length + src_off + 1, np.uint8)
    buf[src_off: src_off + length] = payload
    wire = torch.full((len(ref) + 48,), 0xA5, dtype=torch.uint8, device="cuda")
    codec.fanout(torch.from_numpy(buf).cuda()[src_off:], torch.from_numpy(keys.view(np.int32)).cuda(), opcode, mask,
                 wire=wire, length=length)
    codec.sync()
    got = wire.cpu().numpy()
    bad = np.nonzero(got[: len(ref)] != ref)[0]
    assert bad.size == 0, "first mismatch at byte %d of %d" % (bad[0], len(ref))
    assert (got[len(ref):] == 0xA5).all()


@pytest.mark.parametrize("seed", range(int(os.environ.get("WSG_FUZZ_SEEDS", 60)) // 2))
def test_fuzz_fanout_many_vs_oracle(codec, seed):
    """The ws_multicast tick (wsg_fanout_encode_many): 1-40 messages whose
    lengths and opcodes repeat (same-geometry messages share a launch of the
    period kernel, whose shape — waves per CU per message, no cap — was
    retuned in round 6) or differ, 1-3000 keys, mask flag, unaligned message
    starts; every message's frames vs oracle.fanout_encode, the gaps between
    messages and the bytes past the last frame untouched."""
    rng = np.random.default_rng(9000 + seed)
    m = int(rng.integers(1, 41))
    pool = [int(rng.choice([int(rng.integers(0, 126)), int(rng.integers(126, 9000)), 4096, 4092, 4088]))
            for _ in range(int(rng.integers(1, 4)))]
    lens = np.array([pool[int(rng.integers(0, len(pool)))] for _ in range(m)])
    ops = np.array([int(rng.choice([0x82, 0x81, 0x89])) for _ in range(m)])
    k = int(rng.integers(1, 3000))
    mask = bool(rng.random() < 0.8)
    keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
    src = np.zeros(m, np.uint64)
    src[1:] = np.cumsum(lens[:-1] + rng.integers(0, 17, m - 1))
    arena = wl.random_bytes(rng, int(src[-1] + lens[-1] + 16))
    total = 0
    for i in range(m):
        total = (total + 127) // 128 * 128 + k * int(ca.frame_size(int(ops[i]), mask, int(lens[i])))
    wire = torch.full((total + 256,), 0xA5, dtype=torch.uint8, device="cuda")
    wire_t, off = codec.fanout_many(torch.from_numpy(arena).cuda(), src, lens, ops,
                                    torch.from_numpy(keys.view(np.int32)).cuda(), mask=mask, wire=wire)
    codec.sync()
    got = wire.cpu().numpy()
    covered = np.zeros(len(got), bool)
    for i in range(m):
        msg = arena[int(src[i]): int(src[i]) + int(lens[i])]
        ref = oracle.fanout_encode(msg, keys, int(ops[i]), mask)
        a = int(off[i])
        bad = np.nonzero(got[a: a + len(ref)] != ref)[0]
        assert bad.size == 0, "message %d of %d: first mismatch at byte %d of %d" % (i, m, bad[0], len(ref))
        covered[a: a + len(ref)] = True
    assert (got[~covered] == 0xA5).all()


@pytest.mark.parametrize("seed", range(int(os.environ.get("WSG_FUZZ_SEEDS", 150)) // 3))
def test_fuzz_nothing_written_past_the_output(codec, seed):
    """Outputs of exactly the size the contract gives (encode: the frames'
    bytes as wire_cap; decode: wire_len bytes of output, out of place and in
    place), each inside a larger buffer filled with a sentinel: the frames
    equal the oracle's and not one byte past the output changes — through
    the device entry points and both host paths (page-locked buffers: the
    lane for small batches, the launch path for larger ones).  A whole
    16-byte store of a partial last chunk would write up to 15 bytes past
    a caller's buffer; the fan-out's period kernel did that (round 6)."""
    payload, desc = _batch(1000 + seed)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    n, total = len(desc), len(wire_o)
    S = 0xA5
    # device encode into wire_cap == total
    p = torch.from_numpy(payload if len(payload) else np.zeros(1, np.uint8)).cuda()
    d = ca.desc_to_tensor(desc, "cuda")
    buf = torch.full((total + 64,), S, dtype=torch.uint8, device="cuda")
    codec.encode_batch(p, d, wire=buf[: max(total, 1)], wire_cap=total)
    assert codec.sync_status() == 0
    got = buf.cpu().numpy()
    assert np.array_equal(got[:total], wire_o)
    assert (got[total:] == S).all(), np.nonzero(got[total:] != S)[0][:8]
    fs = off_o[:-1].copy()
    rc_o, out_o, _ = oracle.decode_batch(wire_o, fs)
    f = torch.from_numpy(fs.view(np.int64)).cuda()
    # device decode: out of place, then in place, wire_len == total
    src = torch.from_numpy(wire_o if total else np.zeros(1, np.uint8)).cuda()[:total]
    obuf = torch.full((total + 64,), S, dtype=torch.uint8, device="cuda")
    codec.decode_batch(src, f, out=obuf[:total])
    assert codec.sync_status() == rc_o
    got = obuf.cpu().numpy()
    assert np.array_equal(got[:total], out_o) and (got[total:] == S).all()
    ibuf = torch.full((total + 64,), S, dtype=torch.uint8, device="cuda")
    ibuf[:total] = src
    codec.decode_batch(ibuf[:total], f, out=ibuf[:total])
    assert codec.sync_status() == rc_o
    got = ibuf.cpu().numpy()
    assert np.array_equal(got[:total], out_o) and (got[total:] == S).all()
    # host paths, page-locked buffers with the sentinel behind the output
    pin_p = ca.pinned_empty(max(len(payload), 1))
    pin_p[: len(payload)] = payload
    pin_w = ca.pinned_empty(total + 64)
    pin_w[:] = S
    rc, wire_h, off_h = codec.encode_batch_host(pin_p[: len(payload)], desc, wire=pin_w[:total])
    assert rc == 0 and np.array_equal(pin_w[:total], wire_o) and (pin_w[total:] == S).all()
    pin_in = ca.pinned_empty(max(total, 1))
    pin_in[:total] = wire_o
    pin_out = ca.pinned_empty(total + 64)
    pin_out[:] = S
    rc, out_h, _ = codec.decode_batch_host(pin_in[:total], fs, out=pin_out[:total])
    assert rc == rc_o and np.array_equal(pin_out[:total], out_o) and (pin_out[total:] == S).all()
    assert n == len(fs)
