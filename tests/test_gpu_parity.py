"""Parity of the HIP path (through the C-ABI) with the pinned oracle.

Bit-exact for every byte: this is integer/byte work, no tolerance.
Runs on the MI355X box: `pytest -m gpu`.
"""
import numpy as np
import pytest

import oracle
from tests import kat

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
from cppserver_amd.layout import RECV_INFO, SEND_DESC, frame_size  # noqa: E402

KAT = kat.load()
INFO_FIELDS = ["payload_off", "len", "key", "opcode", "fin", "masked", "hdr_len", "b0", "error"]


@pytest.fixture(scope="module")
def codec():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    c = ca.Codec(0)
    yield c
    c.close()


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.cuda()


def gpu_decode(codec, wire, fs, inplace=False):
    n = len(fs)
    w = dev(wire if len(wire) else np.zeros(0, np.uint8))
    f = dev(np.asarray(fs, dtype=np.uint64).view(np.int64))
    out = w if inplace else None
    out, info = codec.decode_batch(w, f, out=out)
    rc = codec.sync_status()
    return rc, out.cpu().numpy(), ca.info_to_numpy(info, n)


def gpu_encode(codec, payload, desc, cap=None):
    n = len(desc)
    if cap is None:
        cap = int(sum(frame_size(int(d["opcode"]), bool(d["mask"]), int(d["len"]), int(d["status"]))
                      for d in desc)) if n else 16
    p = dev(payload if len(payload) else np.zeros(1, np.uint8))
    d = ca.desc_to_tensor(desc, "cuda")
    wire, off = codec.encode_batch(p, d, wire_cap=max(cap, 16))
    rc = codec.sync_status()
    off = off.cpu().numpy().view(np.uint64)
    return rc, wire.cpu().numpy()[: int(off[n])] if rc == 0 else None, off


def assert_decode_parity(codec, wire, fs, inplace=False):
    rc_o, out_o, info_o = oracle.decode_batch(wire, fs)
    rc_g, out_g, info_g = gpu_decode(codec, wire, fs, inplace=inplace)
    assert rc_g == rc_o
    assert np.array_equal(out_g, out_o)
    for f in INFO_FIELDS:
        assert np.array_equal(info_g[f], info_o[f]), f
    return out_g, info_g


# ---------------------------------------------------------------- golden KATs
@pytest.mark.parametrize("v", KAT["encode"], ids=lambda v: v["name"])
def test_encode_kat(codec, v):
    payload = np.frombuffer(kat.payload_of(v), dtype=np.uint8)
    desc = np.zeros(1, dtype=SEND_DESC)
    desc["len"] = len(payload)
    desc["key"] = kat.key_of(v)
    desc["status"] = v["status"]
    desc["opcode"] = v["opcode"]
    desc["mask"] = v["mask"]
    rc, wire, _ = gpu_encode(codec, payload, desc)
    assert rc == 0
    if "expect" in v:
        assert wire.tobytes().hex() == v["expect"], v["source"]
    else:
        assert wire[: len(v["expect_prefix"]) // 2].tobytes().hex() == v["expect_prefix"]
        assert len(wire) == v["expect_len"]
    if v.get("expect_payload_identity"):
        assert wire[len(wire) - len(payload):].tobytes() == payload.tobytes()


def test_decode_kat_frames(codec):
    """Every whole frame from the decode KATs, decoded as one batch."""
    frames = [bytes.fromhex(c) for v in KAT["decode"] for c in v["chunks"] if v["name"] != "rfc_fragmented_one_read"]
    wire = np.frombuffer(b"".join(frames), dtype=np.uint8)
    fs = np.cumsum([0] + [len(f) for f in frames[:-1]]).astype(np.uint64)
    out, info = assert_decode_parity(codec, wire, fs)
    hello = [i for i, f in enumerate(frames) if f.startswith(bytes.fromhex("8185"))][0]
    p = int(info["payload_off"][hello])
    assert out[p: p + 5].tobytes() == b"Hello"


@pytest.mark.parametrize("v", KAT["roundtrip"], ids=lambda v: v["name"])
def test_roundtrip_kat(codec, v):
    payload = np.frombuffer(kat.payload_of(v), dtype=np.uint8)
    desc = np.zeros(1, dtype=SEND_DESC)
    desc["len"], desc["key"], desc["status"] = len(payload), kat.key_of(v), v["status"]
    desc["opcode"], desc["mask"] = v["opcode"], v["mask"]
    rc, wire, off = gpu_encode(codec, payload, desc)
    assert rc == 0
    ref = oracle.Session(kat.key_of(v)).prepare_send(v["opcode"], v["mask"], payload.tobytes(), v["status"])
    assert wire.tobytes() == ref
    rc, out, info = gpu_decode(codec, wire, [0])
    assert rc == 0
    p, n = int(info["payload_off"][0]), int(info["len"][0])
    (kind, body, status), = kat.events_of(v)
    got = out[p: p + n].tobytes()
    if kind == 2:   # close: status is the first two payload bytes (ws.cpp:435-439)
        assert (got[0] << 8 | got[1], got[2:]) == (status, body)
    else:
        assert got == body


# ---------------------------------------------------------------- C2 (headline)
def test_c2_unmask_full_size_vs_oracle(codec):
    wire, fs, keys = wl.c2_wire(4096, 65536, seed=21)
    out, info = assert_decode_parity(codec, wire, fs)
    assert (info["len"] == 65536).all() and (info["hdr_len"] == 14).all()
    assert np.array_equal(info["key"], keys)


def test_c2_unmask_inplace(codec):
    wire, fs, _ = wl.c2_wire(512, 65536, seed=22)
    assert_decode_parity(codec, wire, fs, inplace=True)


@pytest.mark.parametrize("size", [0, 1, 2, 3, 15, 16, 17, 125, 126, 127, 4095, 65535, 65536, 65537, 200000])
def test_uniform_sizes_vs_oracle(codec, size):
    wire, fs, _ = wl.c2_wire(37, size, seed=size)
    assert_decode_parity(codec, wire, fs)


@pytest.mark.parametrize("size", [58, 57, 26, 25, 10, 0])
def test_decode_staged_round_sizes(codec, size):
    """Staged tiles hold 512 frames per round (two per lane): masked frames
    of 64 B (256 per 16 KiB tile), 63 B, 32 B (exactly 512: one round), 31 B
    (528: a second round), 16 B (1024) and 6 B (2730) per frame."""
    wire, fs, _ = wl.c2_wire(6000, size, seed=1000 + size)
    assert_decode_parity(codec, wire, fs)
    assert_decode_parity(codec, wire, fs, inplace=True)


# ---------------------------------------------------------------- ragged / C3
def _mixed_desc(rng, n, lo, hi):
    lens = rng.integers(lo, hi + 1, n)
    desc, total = wl.ragged_desc(rng, lens)
    desc["opcode"] = rng.choice([0x81, 0x82, 0x01, 0x02, 0x00, 0x80, 0x88, 0x89, 0x8A, 0xC2, 0x83], n)
    desc["mask"] = rng.random(n) < 0.6
    desc["status"] = np.where(rng.random(n) < 0.3, rng.integers(-5, 70000, n), 0)
    desc["src_off"] += rng.integers(0, 16, n).astype(np.uint64)   # misaligned sources
    payload = wl.random_bytes(rng, total + 16)
    return payload, desc


@pytest.mark.parametrize("lo,hi,n", [(0, 40, 3000), (0, 300, 2000), (100, 70000, 300), (128, 65536, 4096)])
def test_encode_mixed_vs_oracle(codec, lo, hi, n):
    rng = np.random.default_rng(lo * 7 + hi + n)
    payload, desc = _mixed_desc(rng, n, lo, hi)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    rc, wire_g, off_g = gpu_encode(codec, payload, desc)
    assert rc == 0
    assert np.array_equal(off_g, off_o)
    assert np.array_equal(wire_g, wire_o)
    # and the GPU decode of that wire matches the oracle decode
    assert_decode_parity(codec, wire_o, off_o[:-1])


SMALL_AVG = 4096   # wsg_internal.h: the small-frame kernel runs when wire_cap <= n * SMALL_AVG


@pytest.mark.parametrize("case", ["tiny", "one", "block-edge", "big-among-small", "close-status", "len-classes",
                                  "mid"])
def test_encode_small_and_piece_kernels(codec, case):
    """Both batch-encode kernels on the same frames: k_encode_small (exact
    capacity, average frame <= SMALL_AVG) and the piece kernel (capacity
    raised past n * SMALL_AVG), each byte-identical to the oracle."""
    rng = np.random.default_rng(sum(map(ord, case)) + 5)
    if case == "tiny":
        payload, desc = _mixed_desc(rng, 3000, 0, 40)
    elif case == "one":
        payload, desc = _mixed_desc(rng, 1, 5, 5)
    elif case == "block-edge":       # 256 frames per block at this size: the last block holds one
        payload, desc = _mixed_desc(rng, 257, 0, 20)
    elif case == "big-among-small":  # a block whose wire range spans many passes of its lanes
        payload, desc = _mixed_desc(rng, 2000, 0, 64)
        big = rng.choice(2000, 8, replace=False)
        desc["len"][big] = rng.integers(60000, 100000, 8)
        desc["src_off"] = rng.integers(0, 16, 2000).astype(np.uint64)
        payload = wl.random_bytes(rng, 100016)
    elif case == "mid":              # ~3 KiB average: 8 frames per block
        payload, desc = _mixed_desc(rng, 1500, 0, 6000)
    elif case == "close-status":
        payload, desc = _mixed_desc(rng, 1500, 0, 30)
        desc["opcode"] = 0x88
        desc["status"] = rng.integers(-3, 70000, 1500)
    else:                             # 7/16/64-bit length fields around their edges
        payload, desc = _mixed_desc(rng, 3000, 0, 3)
        desc["len"] = rng.choice([0, 1, 2, 15, 16, 17, 124, 125, 126, 127, 128], 3000)
        desc["len"][rng.choice(3000, 6, replace=False)] = [65535, 65536, 65537, 65535, 65536, 70000]
        desc["src_off"] = rng.integers(0, 16, 3000).astype(np.uint64)
        payload = wl.random_bytes(rng, 70016)
    _both_encode_kernels(codec, payload, desc)


def _both_encode_kernels(codec, payload, desc):
    n = len(desc)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    exact = int(off_o[n])
    assert exact <= n * SMALL_AVG
    for cap in (exact, n * SMALL_AVG + 4096):
        rc, wire_g, off_g = gpu_encode(codec, payload, desc, cap=cap)
        assert rc == 0
        assert np.array_equal(off_g, off_o), cap
        assert np.array_equal(wire_g, wire_o), cap


def test_encode_small_many_blocks(codec):
    """k_encode_small finalizes the scan's block-local frame offsets itself:
    batches of thousands of blocks and scan blocks, back to back with
    different sizes on one context."""
    rng = np.random.default_rng(77)
    for n, lo, hi in [(300000, 0, 40), (1000, 0, 10), (100000, 0, 2000), (300000, 30, 34), (7, 0, 3)]:
        payload, desc = _mixed_desc(rng, n, lo, hi)
        wire_o, off_o = oracle.encode_batch(payload, desc)
        rc, wire_g, off_g = gpu_encode(codec, payload, desc)
        assert rc == 0
        assert np.array_equal(off_g, off_o), n
        assert np.array_equal(wire_g, wire_o), n


# ------------------------------------------- k_decode tile paths (one launch)
def _frames_wire(rng, lens, gaps=None, lead=0):
    """Masked/unmasked frames of the given payload lengths back to back, with
    optional junk gaps before each frame (gap bytes are copied by decode)."""
    payload, desc = _mixed_desc(rng, len(lens), 0, 0)
    desc["len"] = lens
    desc["src_off"] = 0
    desc["status"] = 0
    payload = wl.random_bytes(rng, int(max(lens.max(), 1)) + 16)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    parts, fs, at = [], [], 0
    junk = lambda k: wl.random_bytes(rng, k)
    if lead:
        parts.append(junk(lead))
        at += lead
    for i in range(len(lens)):
        g = int(gaps[i]) if gaps is not None else 0
        if g:
            parts.append(junk(g))
            at += g
        f = wire_o[int(off_o[i]): int(off_o[i + 1])]
        fs.append(at)
        parts.append(f)
        at += len(f)
    return np.concatenate(parts), np.array(fs, dtype=np.uint64)


@pytest.mark.parametrize("case", ["tiny-then-huge", "huge-then-tiny", "empty-mix", "gaps", "lead-gap",
                                  "tile-edges"])
def test_decode_tile_paths_vs_oracle(codec, case):
    rng = np.random.default_rng(sum(map(ord, case)))
    gaps, lead = None, 0
    if case == "tiny-then-huge":      # the interpolation guess misses: searched tiles
        lens = np.concatenate([rng.integers(0, 20, 3000), rng.integers(60000, 200000, 40)])
    elif case == "huge-then-tiny":
        lens = np.concatenate([rng.integers(60000, 200000, 40), rng.integers(0, 20, 3000)])
    elif case == "empty-mix":         # empty payloads between large and small frames (staged tiles)
        lens = rng.choice([0, 0, 0, 1, 5, 300, 20000], 4000)
    elif case == "gaps":
        lens = rng.integers(0, 5000, 800)
        gaps = rng.integers(0, 40, 800) * (rng.random(800) < 0.5)
    elif case == "lead-gap":          # the first tiles have no frame start at or before them
        lens = rng.integers(100, 3000, 200)
        lead = 40000
    else:                             # frame starts on and next to 16 KiB tile edges
        lens = np.array([16384 - 14, 16384 - 6, 16384 - 2, 16384 - 15, 1, 16384 * 3 - 14, 0, 16384 - 8] * 8)
    wire, fs = _frames_wire(rng, lens.astype(np.uint64), gaps, lead)
    assert_decode_parity(codec, wire, fs)
    assert_decode_parity(codec, wire, fs, inplace=True)


def test_c3_roundtrip_full_size(codec):
    """C3 at BASELINE size (65536 frames, payload 128 B-64 KiB, 2.15 GB):
    every frame of the GPU encode byte for byte against the oracle's encode
    of the whole batch, every frame of the GPU decode of that wire (payloads,
    headers and wsg_recv_info) against the oracle's decode, and the decoded
    payloads are the input payloads (round trip)."""
    payload, desc = wl.c3_batch(65536, 128, 65536, seed=31)
    n = len(desc)
    p = dev(payload)
    d = ca.desc_to_tensor(desc, "cuda")
    cap = int(sum(frame_size(0x82, True, int(x)) for x in desc["len"]))
    wire, off = codec.encode_batch(p, d, wire_cap=cap)
    out, info = codec.decode_batch(wire[:cap], off[:-1])
    codec.sync()
    offs = off.cpu().numpy().view(np.uint64)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    assert np.array_equal(offs, off_o)
    wire_g = wire[:cap].cpu().numpy()
    assert np.array_equal(wire_g, wire_o)
    del wire_g
    rc_o, out_o, info_o = oracle.decode_batch(wire_o, off_o[:-1])
    assert rc_o == 0
    assert np.array_equal(out.cpu().numpy(), out_o)
    info_g = ca.info_to_numpy(info, n)
    for f in INFO_FIELDS:
        assert np.array_equal(info_g[f], info_o[f]), f
    # round trip: every decoded payload is its input payload
    po = info_g["payload_off"].astype(np.int64)
    ln = info_g["len"].astype(np.int64)
    so = desc["src_off"].astype(np.int64)
    bad = [i for i in range(n) if not np.array_equal(out_o[po[i]: po[i] + ln[i]], payload[so[i]: so[i] + ln[i]])]
    assert not bad, bad[:5]


# ---------------------------------------------------------------- C4 fan-out
def test_c4_fanout_vs_oracle(codec):
    payload, keys = wl.c4_fanout(4096, 10000, seed=41)
    ref = oracle.fanout_encode(payload, keys, 0x82, True)
    wire = codec.fanout(dev(payload), dev(keys.view(np.int32)), 0x82, True)
    codec.sync()
    assert np.array_equal(wire.cpu().numpy()[: len(ref)], ref)


@pytest.mark.parametrize("length,k,opcode,mask", [(0, 5, 0x88, True), (1, 33, 0x89, False), (125, 100, 0x81, True),
                                                 (126, 100, 0x82, False), (5000, 77, 0x8A, True),
                                                 (65536, 9, 0x82, True)])
def test_fanout_shapes(codec, length, k, opcode, mask):
    payload, keys = wl.c4_fanout(length, k, seed=length + k)
    ref = oracle.fanout_encode(payload, keys, opcode, mask)
    wire = codec.fanout(dev(payload if length else np.zeros(1, np.uint8)), dev(keys.view(np.int32)), opcode, mask,
                        length=length)
    codec.sync()
    assert np.array_equal(wire.cpu().numpy()[: len(ref)], ref)


@pytest.mark.parametrize("length,k,opcode,mask,src_off", [(2, 50, 0x82, True, 0), (3, 41, 0x89, True, 1),
                                                         (7, 64, 0x82, False, 5), (9, 17, 0x88, True, 0),
                                                         (10, 300, 0x81, True, 3), (4096, 257, 0x82, True, 7),
                                                         (65535, 5, 0x82, True, 9)])
def test_fanout_tiny_unaligned_tail(codec, length, k, opcode, mask, src_off):
    """Frames shorter than a 16-B chunk, payloads at any alignment, and no byte
    written past the k frames (sentinel-filled wire)."""
    payload, keys = wl.c4_fanout(length, k, seed=7 * length + k)
    ref = oracle.fanout_encode(payload, keys, opcode, mask)
    buf = np.zeros(length + src_off + 1, np.uint8)
    buf[src_off: src_off + length] = payload
    pbuf = dev(buf)
    wire = torch.full((len(ref) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    codec.fanout(pbuf[src_off:], dev(keys.view(np.int32)), opcode, mask, wire=wire, length=length)
    codec.sync()
    got = wire.cpu().numpy()
    assert np.array_equal(got[: len(ref)], ref)
    assert (got[len(ref):] == 0xA5).all()


@pytest.mark.parametrize("length,k,opcode,mask,src_off", [(1010, 700, 0x82, True, 0), (1018, 333, 0x89, False, 3),
                                                         (2047, 64, 0x8A, True, 1), (4096, 4097, 0x82, False, 0),
                                                         (4100, 999, 0x81, True, 11), (8190, 130, 0x89, True, 8),
                                                         (12268, 33, 0x82, True, 2), (12290, 7, 0x82, True, 0)])
def test_fanout_mid_sizes(codec, length, k, opcode, mask, src_off):
    """Frames of 1-12 KiB: frame starts at every phase of the 16-B chunks,
    status-prefixed opcodes, unmasked frames still XORed (Q1),
    unaligned payload sources, nothing written past the last frame."""
    payload, keys = wl.c4_fanout(length, k, seed=3 * length + k)
    ref = oracle.fanout_encode(payload, keys, opcode, mask)
    buf = np.zeros(length + src_off + 1, np.uint8)
    buf[src_off: src_off + length] = payload
    wire = torch.full((len(ref) + 48,), 0xA5, dtype=torch.uint8, device="cuda")
    codec.fanout(dev(buf)[src_off:], dev(keys.view(np.int32)), opcode, mask, wire=wire, length=length)
    codec.sync()
    got = wire.cpu().numpy()
    assert np.array_equal(got[: len(ref)], ref)
    assert (got[len(ref):] == 0xA5).all()


@pytest.mark.parametrize("length,k,opcode,mask,src_off", [
    (4096, 10000, 0x82, True, 0),   # C4: F = 4104, groups of 2 frames (513 chunks)
    (4096, 257, 0x82, True, 5),     # odd k: the last group is half a group
    (4088, 3000, 0x82, True, 0),    # F = 4096: one frame per group
    (1016, 5000, 0x81, True, 3),    # F = 1024: G = 64, every row is exactly one group
    (1006, 777, 0x88, True, 0),     # close with status prefix (Q2): F = 1016, G = 127
    (2040, 1001, 0x82, False, 1),   # unmasked, still XORed (Q1): F = 2044, groups of 4 frames
    (4096, 4097, 0x82, False, 0),   # F = 4100: 4-frame groups, wire ends inside a chunk
    (8190, 130, 0x89, True, 8),     # ping with status prefix: F = 8200
    (65538, 40, 0x82, True, 0),     # 8-byte length form: F = 65552, 4097-chunk groups
])
def test_fanout_period_path(codec, length, k, opcode, mask, src_off):
    """Fan-outs whose frame size is a multiple of 4 take k_fanout_period (one
    chunk template per lane, keys picked per pass): parity with the oracle,
    nothing written past the k frames."""
    payload, keys = wl.c4_fanout(length, k, seed=11 * length + k)
    ref = oracle.fanout_encode(payload, keys, opcode, mask)
    assert len(ref) % (4 * k) == 0
    buf = np.zeros(length + src_off + 1, np.uint8)
    buf[src_off: src_off + length] = payload
    wire = torch.full((len(ref) + 48,), 0xA5, dtype=torch.uint8, device="cuda")
    codec.fanout(dev(buf)[src_off:], dev(keys.view(np.int32)), opcode, mask, wire=wire, length=length)
    codec.sync()
    got = wire.cpu().numpy()
    bad = np.nonzero(got[: len(ref)] != ref)[0]
    assert bad.size == 0, "first mismatch at byte %d of %d" % (bad[0], len(ref))
    assert (got[len(ref):] == 0xA5).all()


@pytest.mark.parametrize("case", ["c4x16", "mixed", "many-groups", "flat-sizes"])
def test_fanout_many_vs_oracle(codec, case):
    """wsg_fanout_encode_many: m messages x k keys in one call (one launch per
    group of up to 32 same-geometry messages), each message's frames equal to
    oracle.fanout_encode of that message; nothing written outside them."""
    rng = np.random.default_rng(sum(map(ord, case)))
    if case == "c4x16":        # the multicast tick at C4's shape
        m, k = 16, 10000
        lens = np.full(m, 4096)
        ops = np.full(m, 0x82)
    elif case == "mixed":      # lengths / opcodes differ: several launches, status-prefixed ping (Q2)
        m, k = 9, 300
        lens = np.array([4096, 4096, 100, 4096, 1016, 65538, 4096, 0, 2040])
        ops = np.array([0x82, 0x81, 0x82, 0x82, 0x89, 0x82, 0x82, 0x88, 0x8A])
    elif case == "many-groups":  # more than 32 messages of one geometry: two launches
        m, k = 70, 257
        lens = np.full(m, 4088)
        ops = np.full(m, 0x82)
    else:                      # frame sizes the period path does not take (flat kernel per message)
        m, k = 5, 123
        lens = np.array([4097, 1, 30, 12290, 4097])
        ops = np.array([0x82, 0x81, 0x82, 0x82, 0x82])
    keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
    src = np.zeros(m, np.uint64)
    src[1:] = np.cumsum(lens[:-1] + 3)           # unaligned message starts
    arena = wl.random_bytes(rng, int(src[-1] + lens[-1] + 16))
    for mask in (True, False):
        wire_t, off = codec.fanout_many(dev(arena), src, lens, ops, dev(keys.view(np.int32)), mask=mask)
        codec.sync()
        got = wire_t.cpu().numpy()
        for i in range(m):
            msg = arena[int(src[i]): int(src[i]) + int(lens[i])]
            ref = oracle.fanout_encode(msg, keys, int(ops[i]), mask)
            a = int(off[i])
            assert a % 128 == 0
            assert np.array_equal(got[a: a + len(ref)], ref), (i, mask)
        assert int(off[m]) == int(off[m - 1]) + k * frame_size(int(ops[-1]), mask, int(lens[-1]))


@pytest.mark.parametrize("length,k,opcode", [
    (4092, 7, 0x82),     # F = 4100: P = 4, G = 1025, the last chunk partial (total % 16 = 12)
    (4096, 3, 0x82),     # F = 4104: P = 2 (C4's geometry), total % 16 = 8
    (4088, 5, 0x81),     # F = 4096: P = 1
    (122, 1000, 0x82),   # F = 128: G = 8 (below the period kernel's 64)
    (58, 33, 0x82),      # F = 64: G = 4
    (8190, 130, 0x89),   # ping with the status prefix: F = 8200, P = 2
    (65538, 40, 0x82),   # 8-byte length form: F = 65552
])
def test_fanout_many_geometries(length, k, opcode):
    """Several messages of one geometry in one call (wsg_fanout_encode_many)
    for every group period of the period kernel (P = 1, 2, 4, partial last
    chunk) and frame sizes it leaves to the flat kernel: every message's frames
    equal oracle.fanout_encode's, masked and unmasked."""
    rng = np.random.default_rng(length * 31 + k)
    m = 3
    keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
    lens = np.full(m, length)
    ops = np.full(m, opcode)
    src = np.zeros(m, np.uint64)
    src[1:] = np.cumsum(lens[:-1] + 5)            # unaligned message starts
    arena = wl.random_bytes(rng, int(src[-1] + lens[-1] + 16))
    c = ca.Codec(0)
    try:
        for mask in (True, False):
            wire_t, off = c.fanout_many(dev(arena), src, lens, ops, dev(keys.view(np.int32)), mask=mask)
            c.sync()
            got = wire_t.cpu().numpy()
            for i in range(m):
                ref = oracle.fanout_encode(arena[int(src[i]): int(src[i]) + length], keys, opcode, mask)
                a = int(off[i])
                assert np.array_equal(got[a: a + len(ref)], ref), (i, mask)
    finally:
        c.close()


@pytest.mark.parametrize("length,k,opcode,m", [
    (4096, 127, 0x82, 1),    # C4's geometry (F = 4104, P = 2): 32576 chunks = 509 whole rows, the last chunk 8 bytes
    (4096, 127, 0x82, 3),
    (4092, 2558, 0x81, 2),   # F = 4100, P = 4: 655488 chunks (10242 rows), the last chunk 8 bytes
    (4092, 1343, 0x82, 1),   # F = 4100: 344,138 chunks (not a whole row count), the last chunk 12 bytes
])
def test_fanout_last_chunk_partial_ends_a_row(length, k, opcode, m):
    """The period kernel's last row when the job's last 16-byte chunk is
    partial and the chunk count is a multiple of 64 (the row is otherwise
    whole): nothing may be written past the last frame — the whole-row store
    of round 5 wrote the next frame's first bytes there (up to 15), past the
    caller's capacity when wire_cap is the exact size.  Found by
    test_fuzz_fanout_many_vs_oracle (seed 123).  The output buffer is exactly
    the frames' size with a sentinel allocation behind it, and the messages of
    a many-message call must leave their alignment gaps untouched."""
    rng = np.random.default_rng(k)
    keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
    c = ca.Codec(0)
    try:
        for mask in (True, False):
            fsz = frame_size(opcode, mask, length)
            if m == 1:
                payload = wl.random_bytes(rng, length)
                ref = oracle.fanout_encode(payload, keys, opcode, mask)
                assert len(ref) == fsz * k
                buf = torch.full((len(ref) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
                c.fanout(dev(payload), dev(keys.view(np.int32)), opcode, mask, wire=buf[: len(ref)], length=length)
                c.sync()
                got = buf.cpu().numpy()
                assert np.array_equal(got[: len(ref)], ref), mask
                assert (got[len(ref):] == 0xA5).all(), np.nonzero(got[len(ref):] != 0xA5)[0][:16]
            else:
                lens = np.full(m, length)
                ops = np.full(m, opcode)
                src = np.zeros(m, np.uint64)
                src[1:] = np.cumsum(lens[:-1] + 5)
                arena = wl.random_bytes(rng, int(src[-1] + lens[-1] + 16))
                need = 0
                for _ in range(m):
                    need = (need + 127) // 128 * 128 + fsz * k
                buf = torch.full((need + 64,), 0xA5, dtype=torch.uint8, device="cuda")
                _, off = c.fanout_many(dev(arena), src, lens, ops, dev(keys.view(np.int32)), mask=mask,
                                       wire=buf[:need])
                c.sync()
                got = buf.cpu().numpy()
                covered = np.zeros(len(got), bool)
                for i in range(m):
                    ref = oracle.fanout_encode(arena[int(src[i]): int(src[i]) + length], keys, opcode, mask)
                    a = int(off[i])
                    assert np.array_equal(got[a: a + len(ref)], ref), (i, mask)
                    covered[a: a + len(ref)] = True
                assert (got[~covered] == 0xA5).all(), np.nonzero((got != 0xA5) & ~covered)[0][:16]
    finally:
        c.close()


def test_fanout_many_capacity(codec):
    keys = torch.zeros(4, dtype=torch.int32, device="cuda")
    with pytest.raises(ca.WSGError) as e:
        codec.fanout_many(torch.zeros(64, dtype=torch.uint8, device="cuda"), [0, 0], [10, 10], [0x82, 0x82], keys,
                          wire=torch.zeros(64, dtype=torch.uint8, device="cuda"))
    assert e.value.code == ca.WSG_ENOMEM


# ---------------------------------------------------------------- edge cases
def test_empty_batches(codec):
    rc, out, info = gpu_decode(codec, np.zeros(32, np.uint8), [])
    assert rc == 0 and np.array_equal(out, np.zeros(32, np.uint8))
    rc, wire, off = gpu_encode(codec, np.zeros(1, np.uint8), np.zeros(0, dtype=SEND_DESC))
    assert rc == 0 and off[0] == 0


def test_decode_errors_match_oracle(codec):
    frame = bytes([0x82, 0x05, 1, 2, 3, 4, 5])
    masked = oracle.Session(0x01020304).prepare_send(0x82, True, bytes(range(40)))
    wire = np.frombuffer(masked + frame + frame, dtype=np.uint8)
    n1 = len(masked)
    for fs, cut in [([0, n1, n1 + 7], 1), ([0, n1, n1 + 3], 0), ([0, 5], 0), ([0, n1, n1 + 7], 10)]:
        w = wire[: len(wire) - cut]
        rc_o, out_o, info_o = oracle.decode_batch(w, fs)
        rc_g, out_g, info_g = gpu_decode(codec, w, fs)
        assert rc_o != 0 and rc_g == rc_o
        assert np.array_equal(info_g["error"], info_o["error"])
        ok = info_o["error"] == 0
        for f in INFO_FIELDS:
            assert np.array_equal(info_g[f][ok], info_o[f][ok]), f
        assert np.array_equal(out_g, out_o)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_decode_garbage_starts_match_oracle(codec, seed):
    """Frame-start tables that break the contract (unsorted, repeated, past
    the wire's end, pointing into payloads): the launch ends, the status and
    every frame's error code are the oracle's (output bytes are unspecified
    for such a batch)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, 300).astype(np.uint64)
    wire, fs = _frames_wire(rng, lens)
    bad = fs.copy()
    pick = rng.random(len(bad))
    bad[pick < 0.2] = rng.integers(0, len(wire) + 100, int((pick < 0.2).sum()))
    bad[(pick >= 0.2) & (pick < 0.25)] = 0
    rng.shuffle(bad[: len(bad) // 3])
    rc_o, _, info_o = oracle.decode_batch(wire, bad)
    rc_g, _, info_g = gpu_decode(codec, wire, bad)
    assert rc_o != 0 and rc_g == rc_o
    assert np.array_equal(info_g["error"], info_o["error"])
    ok = info_o["error"] == 0
    for f in INFO_FIELDS:
        assert np.array_equal(info_g[f][ok], info_o[f][ok]), f


def test_misaligned_buffers_rejected(codec):
    w = torch.zeros(64, dtype=torch.uint8, device="cuda")
    f = torch.zeros(1, dtype=torch.int64, device="cuda")
    with pytest.raises(ca.WSGError) as e:
        codec.decode_batch(w[1:], f)
    assert e.value.code == ca.WSG_EINVAL


def test_encode_capacity_error(codec):
    payload = np.zeros(1000, np.uint8)
    desc = np.zeros(4, dtype=SEND_DESC)
    desc["len"] = 250
    desc["opcode"] = 0x82
    rc, _, _ = gpu_encode(codec, payload, desc, cap=500)
    assert rc == ca.WSG_ENOMEM


# ---------------------------------------------------------------- host-staged
@pytest.mark.parametrize("n,key,phase", [(1, 0xDEADBEEF, 0), (15, 1, 3), (4097, 0xA1B2C3D4, 2), (1 << 20, 7, 1)])
def test_xor_host(codec, n, key, phase):
    data = wl.random_bytes(np.random.default_rng(n), n)
    kb = np.frombuffer(int(key).to_bytes(4, "little"), np.uint8)
    exp = data ^ kb[(np.arange(n) + phase) % 4]
    assert codec.xor_host(data.tobytes(), key, phase) == exp.tobytes()


def test_decode_batch_host(codec):
    wire, fs, _ = wl.c2_wire(64, 5000, seed=9)
    rc, out, info = codec.decode_batch_host(wire, fs)
    rc_o, out_o, info_o = oracle.decode_batch(wire, fs)
    assert rc == rc_o == 0
    assert np.array_equal(out, out_o)
    for f in INFO_FIELDS:
        assert np.array_equal(info[f], info_o[f])


@pytest.mark.parametrize("stage_mb", ["1", "32"])
def test_decode_batch_host_segmented(codec, stage_mb, monkeypatch):
    """The pipelined host path cuts the batch into segments; results must not
    depend on where the cuts fall (ragged frames, misaligned segment starts,
    a truncated last frame, an overlap at a segment edge)."""
    monkeypatch.setenv("WSG_STAGE_MB", stage_mb)
    rng = np.random.default_rng(int(stage_mb))
    payload, desc = _mixed_desc(rng, 600, 0, 70000)
    wire, off = oracle.encode_batch(payload, desc)
    fs = off[:-1].copy()
    for variant in ("ok", "trunc", "overlap"):
        w, f = wire, fs
        if variant == "trunc":
            w = wire[:-5]
        if variant == "overlap":
            f = fs.copy()
            f[300] = f[300] + 1     # frame 299 now overlaps frame 300
        rc_o, out_o, info_o = oracle.decode_batch(w, f)
        for pinned in (False, True):
            src = w
            if pinned:
                src = ca.pinned_empty(len(w))
                src[:] = w
            rc, out, info = codec.decode_batch_host(src, f)
            assert rc == rc_o, (variant, pinned)
            assert np.array_equal(out, out_o), (variant, pinned)
            for fld in INFO_FIELDS:
                assert np.array_equal(info[fld], info_o[fld]), (variant, pinned, fld)


@pytest.mark.parametrize("direct_max", ["4194304", "0"])
def test_host_batches_pinned_errors(codec, direct_max, monkeypatch):
    """Small host batches in page-locked buffers: the direct path (kernels on
    the host buffers) and, with it off, the staged pipeline give the oracle's
    bytes, fields and status, also for a truncated last frame and an overlap."""
    monkeypatch.setenv("WSG_HOST_DIRECT_MAX", direct_max)
    c = ca.Codec(0)   # the knob is read when the context is made
    try:
        rng = np.random.default_rng(77)
        payload, desc = _mixed_desc(rng, 300, 0, 3000)
        wire, off = oracle.encode_batch(payload, desc)
        pin_p = ca.pinned_empty(len(payload))
        pin_p[:] = payload
        pin_w = ca.pinned_empty(len(wire) + 16)
        rc, w2, off2 = c.encode_batch_host(pin_p, desc, wire=pin_w)
        assert rc == 0 and np.array_equal(w2, wire) and np.array_equal(off2, off)
        fs = off[:-1].copy()
        for variant in ("ok", "trunc", "overlap"):
            w, f = wire, fs
            if variant == "trunc":
                w = wire[:-5]
            if variant == "overlap":
                f = fs.copy()
                f[150] += 1
            rc_o, out_o, info_o = oracle.decode_batch(w, f)
            src, dst = ca.pinned_empty(len(w) + 16), ca.pinned_empty(len(w) + 16)
            src[: len(w)] = w
            rc, out, info = c.decode_batch_host(src[: len(w)], f, out=dst)
            assert rc == rc_o, variant
            assert np.array_equal(out, out_o), variant
            for fld in INFO_FIELDS:
                assert np.array_equal(info[fld], info_o[fld]), (variant, fld)
    finally:
        c.close()


def test_host_batches_registered_memory(codec):
    """Host batches in memory page-locked with hipHostRegister (a server's own
    socket buffers registered in place): such memory may have another device
    address, so the direct small-batch path must not hand the host pointer
    to a kernel; results are the oracle's either way, at buffer offsets too."""
    import ctypes

    hip = ctypes.CDLL("libamdhip64.so")
    rng = np.random.default_rng(78)
    payload, desc = _mixed_desc(rng, 200, 0, 3000)
    wire, off = oracle.encode_batch(payload, desc)
    fs = off[:-1].copy()
    rc_o, out_o, info_o = oracle.decode_batch(wire, fs)
    need = 3 * (len(wire) + len(payload)) + (1 << 16)
    raw = np.zeros(need + 8192, dtype=np.uint8)
    base = raw.ctypes.data + (-raw.ctypes.data) % 4096
    region = raw[base - raw.ctypes.data: base - raw.ctypes.data + need]
    assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(need), 0) == 0
    try:
        for shift in (0, 4096 + 16):
            a = shift
            src = region[a: a + len(wire)]
            a += (len(wire) + 15) // 16 * 16
            dst = region[a: a + len(wire)]
            a += (len(wire) + 15) // 16 * 16
            pl = region[a: a + len(payload)]
            a += (len(payload) + 15) // 16 * 16
            wout = region[a: a + len(wire)]
            src[:] = wire
            rc, out, info = codec.decode_batch_host(src, fs, out=dst)
            assert rc == rc_o and np.array_equal(out, out_o), shift
            for fld in INFO_FIELDS:
                assert np.array_equal(info[fld], info_o[fld]), (shift, fld)
            pl[:] = payload
            rc, w2, off2 = codec.encode_batch_host(pl, desc, wire=wout)
            assert rc == 0 and np.array_equal(w2, wire) and np.array_equal(off2, off), shift
    finally:
        hip.hipHostUnregister(ctypes.c_void_p(base))


def test_host_pipeline_keeps_caller_latch(codec):
    """A host-staged call between an async batch call and its wsg_sync must
    not clear (or add to) the error that async call latched."""
    frame = bytes([0x82, 0x05, 1, 2, 3, 4, 5])
    bad = np.frombuffer(frame + frame[:4], dtype=np.uint8)   # the second frame runs past the wire
    w = dev(bad)
    f = dev(np.array([0, 7], dtype=np.int64))
    codec.decode_batch(w, f)                                  # async: latches ETRUNC
    wire, fs, _ = wl.c2_wire(8, 1000, seed=3)
    rc, _, _ = codec.decode_batch_host(wire, fs)              # a clean host-staged batch
    assert rc == 0
    rc2, _, _ = codec.decode_batch_host(bad, np.array([0, 7], np.uint64))   # its own error, its own status
    assert rc2 == ca.WSG_ETRUNC
    assert codec.sync_status() == ca.WSG_ETRUNC               # the async call's error is still there
    assert codec.sync_status() == 0


def test_encode_wire_cap_checked(codec):
    wire = torch.empty(64, dtype=torch.uint8, device="cuda")
    with pytest.raises(ca.WSGError):
        codec.encode_batch(dev(np.zeros(16, np.uint8)), ca.desc_to_tensor(np.zeros(1, dtype=SEND_DESC), "cuda"),
                           wire=wire, wire_cap=128)


def test_timing_hook_counts_launches(codec):
    wire, fs, _ = wl.c2_wire(64, 65536, seed=10)
    w, f = dev(wire), dev(fs.view(np.int64))
    codec.timing(True)
    for _ in range(3):
        codec.decode_batch(w, f)
    ms, launches = codec.timing_read()
    codec.timing(False)
    codec.sync()
    assert launches == 3 and ms > 0


def _xor_key_chunks(x, key, at):
    """x ^ key bytes (byte j of the key = (key >> 8j) & 0xFF) for a chunk of
    payload that starts at payload offset `at` (a multiple of 4)."""
    kb = torch.tensor(list(int(key).to_bytes(4, "little")), dtype=torch.uint8, device=x.device)
    reps = (x.numel() + 3) // 4
    return x ^ kb.repeat(reps)[: x.numel()]


@pytest.mark.parametrize("length", [(5 << 30) + 3])
def test_single_frame_over_4gib(codec, length):
    """Maximum sizes: ONE frame whose payload passes 2^32 bytes (64-bit length
    header, ws.cpp:234-239 / :354-371; every 64-bit offset in the kernels
    past the u32 range).  Encode: the header equals wsg_header_pack's (the
    host code the KAT vectors pin) and the payload is x ^ key (ws.cpp:269-270,
    key byte i % 4), checked in 1 GiB chunks on the device; decode of the
    encoded wire, out of place and in place, gives the payload back with the
    frame's fields; the encoded first and last MiB also byte for byte
    against the oracle."""
    key = 0xA1B2C3D4
    gen = torch.Generator(device="cuda").manual_seed(4242)
    payload = torch.randint(0, 256, (length,), dtype=torch.uint8, device="cuda", generator=gen)
    desc = np.zeros(1, dtype=SEND_DESC)
    desc["len"], desc["key"], desc["opcode"], desc["mask"] = length, key, 0x82, 1
    hdr = ca.header_pack(0x82, True, length, 0, key)
    assert len(hdr) == 14
    wire, off = codec.encode_batch(payload, ca.desc_to_tensor(desc, "cuda"), wire_cap=length + 14)
    assert codec.sync_status() == 0
    assert int(off[1].item()) == length + 14
    assert bytes(wire[:14].cpu().numpy()) == hdr
    step = 1 << 30
    for a in range(0, length, step):
        b = min(a + step, length)
        assert torch.equal(wire[14 + a: 14 + b], _xor_key_chunks(payload[a:b], key, a)), "encode chunk %d" % a
    # the GPU's encoded bytes around the payload's first and last MiB against
    # the oracle's encode of a frame of the same header class (64-bit
    # length) over those bytes (key phase 0 at a multiple of 4)
    for a in (0, length - (1 << 20)):
        a -= a % 4
        part = payload[a: a + (1 << 20)].cpu().numpy()
        d = desc.copy()
        d["len"] = len(part)
        w_o, _ = oracle.encode_batch(part, d)
        assert np.array_equal(wire[14 + a: 14 + a + len(part)].cpu().numpy(), w_o[14:]), "oracle at %d" % a
    fs = torch.zeros(1, dtype=torch.int64, device="cuda")
    out, info = codec.decode_batch(wire, fs)
    assert codec.sync_status() == 0
    r = ca.info_to_numpy(info, 1)[0]
    assert (int(r["payload_off"]), int(r["len"]), int(r["key"]), int(r["opcode"]), int(r["fin"]), int(r["error"])) \
        == (14, length, key, 2, 1, 0)
    for a in range(0, length, step):
        b = min(a + step, length)
        assert torch.equal(out[14 + a: 14 + b], payload[a:b]), "decode chunk %d" % a
    del out
    codec.decode_batch(wire, fs, out=wire)   # in place
    assert codec.sync_status() == 0
    for a in range(0, length, step):
        b = min(a + step, length)
        assert torch.equal(wire[14 + a: 14 + b], payload[a:b]), "in-place chunk %d" % a
    del payload, wire


def test_ragged_wire_over_4gib(codec):
    """Maximum sizes, many frames: a 90,000-frame ragged batch (payload 0 to
    110,000 B, ~4.95 GB of wire) encoded and decoded on the GPU, so frame
    starts, tiles and payloads straddle the 2^32-byte mark.  Every frame's
    decode info vs its descriptor (vectorized); payloads of the frames around
    2^32 and 500 sampled ones vs their input; the wire around 2^32 decoded
    byte for byte by the oracle."""
    rng = np.random.default_rng(432)
    n = 90000
    lens = rng.integers(0, 110001, n).astype(np.uint64)
    desc = np.zeros(n, dtype=SEND_DESC)
    desc["len"] = lens
    desc["src_off"][1:] = np.cumsum(lens)[:-1]
    desc["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    desc["opcode"], desc["mask"] = 0x82, 1
    total = int(lens.sum())
    gen = torch.Generator(device="cuda").manual_seed(7)
    payload = torch.randint(0, 256, (total,), dtype=torch.uint8, device="cuda", generator=gen)
    sizes = ca.frame_sizes(desc).astype(np.uint64)
    cap = int(sizes.sum())
    assert cap > (1 << 32) + (1 << 28)
    wire, off = codec.encode_batch(payload, ca.desc_to_tensor(desc, "cuda"), wire_cap=cap)
    assert codec.sync_status() == 0
    offs = off.cpu().numpy().view(np.uint64)
    assert np.array_equal(offs[1:], np.cumsum(sizes))
    out, info = codec.decode_batch(wire, off[:-1])
    assert codec.sync_status() == 0
    r = ca.info_to_numpy(info, n)
    hdr = sizes - lens
    assert np.array_equal(r["payload_off"], offs[:-1] + hdr)
    assert np.array_equal(r["len"], lens)
    assert np.array_equal(r["key"], desc["key"])
    assert not r["error"].any()
    j = int(np.searchsorted(offs, 1 << 32, side="right")) - 1   # the frame holding byte 2^32
    pick = sorted(set(range(max(0, j - 20), min(n, j + 21))) | set(rng.integers(0, n, 500).tolist()))
    for i in pick:
        po, ln, so = int(r["payload_off"][i]), int(lens[i]), int(desc["src_off"][i])
        assert torch.equal(out[po: po + ln], payload[so: so + ln]), "frame %d" % i
    a, b = max(0, j - 5), min(n, j + 6)
    lo, hi = int(offs[a]), int(offs[b])
    rc_o, out_o, _ = oracle.decode_batch(wire[lo:hi].cpu().numpy(), (offs[a:b] - offs[a]).astype(np.uint64))
    assert rc_o == 0 and np.array_equal(out[lo:hi].cpu().numpy(), out_o)
    del payload, wire, out


def test_host_pipeline_frames_larger_than_segments(codec, monkeypatch):
    """The host-staged paths cut batches into ~$WSG_STAGE_MB segments of whole
    frames; frames several times a segment's size make segments of one frame
    each (decode and encode, pinned and pageable) and still match the oracle."""
    monkeypatch.setenv("WSG_STAGE_MB", "1")
    rng = np.random.default_rng(77)
    lens = np.array([5 << 20, 17, (3 << 20) + 5, 0, 2 << 20], dtype=np.uint64)
    payload = wl.random_bytes(rng, int(lens.sum()) + 16)
    desc = np.zeros(len(lens), dtype=SEND_DESC)
    desc["len"] = lens
    desc["src_off"][1:] = np.cumsum(lens)[:-1]
    desc["key"] = rng.integers(1, 2**32, len(lens), dtype=np.uint64).astype(np.uint32)
    desc["opcode"], desc["mask"] = 0x82, 1
    wire_o, off_o = oracle.encode_batch(payload, desc)
    rc_o, out_o, info_o = oracle.decode_batch(wire_o, off_o[:-1])
    assert rc_o == 0
    for pinned in (False, True):
        p = payload
        if pinned:
            p = ca.pinned_empty(len(payload))
            p[:] = payload
        rc, wire, off = codec.encode_batch_host(p, desc)
        assert rc == 0 and np.array_equal(wire, wire_o) and np.array_equal(off, off_o)
        rc, out, info = codec.decode_batch_host(wire_o, off_o[:-1])
        assert rc == 0 and np.array_equal(out, out_o)
        for f in INFO_FIELDS:
            assert np.array_equal(info[f], info_o[f]), f


def test_prepare_decode_matches_decode_batch(codec):
    """Codec.prepare_decode (the bench's pre-bound C-ABI launch) decodes the
    same bytes and fields as decode_batch, launch after launch."""
    wire, fs, _ = wl.c2_wire(64, 5000, seed=12)
    w = dev(wire)
    f = dev(fs.view(np.int64))
    out = torch.empty_like(w)
    info = torch.empty(64 * RECV_INFO.itemsize, dtype=torch.uint8, device="cuda")
    launch = codec.prepare_decode(w, f, out, info)
    for _ in range(3):
        launch()
    assert codec.sync_status() == 0
    rc, out_r, info_r = gpu_decode(codec, wire, fs)
    assert rc == 0 and np.array_equal(out.cpu().numpy(), out_r)
    got = ca.info_to_numpy(info, 64)
    for fld in INFO_FIELDS:
        assert np.array_equal(got[fld], info_r[fld]), fld


def test_checked_launches(monkeypatch):
    """$WSG_CHECK=1: operand ranges outside their device allocation are
    refused on the host (WSG_EINVAL) before any kernel runs; valid calls give
    the usual results.  The out-of-range operands are exact hipMalloc blocks
    (torch's allocator hands out views of larger segments)."""
    import ctypes

    monkeypatch.setenv("WSG_CHECK", "1")
    hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch and libwsg share
    blocks = []

    def hip_alloc(nbytes):
        p = ctypes.c_void_p()
        assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) == 0
        blocks.append(p)
        return p.value

    c = ca.Codec(0)
    try:
        wire, fs, _ = wl.c2_wire(64, 5000, seed=5)
        rc, out, info = gpu_decode(c, wire, fs)
        rc_o, out_o, _ = oracle.decode_batch(wire, fs)
        assert rc == rc_o == 0 and np.array_equal(out, out_o)
        L = c._L
        w = hip_alloc(2 << 20)
        o = hip_alloc(4 << 20)
        f = hip_alloc(64)
        inf = hip_alloc(64)
        vp = ctypes.c_void_p
        assert hip.hipMemset(vp(f), 0, ctypes.c_size_t(64)) == 0
        # decode: an output 1 MiB before the end of its 4 MiB block, 2 MiB wire
        assert L.wsg_decode_batch(c._ctx, vp(w), 2 << 20, vp(f), 1, vp(o + (3 << 20)), vp(inf), None) == ca.WSG_EINVAL
        # the same wire into the block's start is accepted
        assert L.wsg_decode_batch(c._ctx, vp(w), 2 << 20, vp(f), 1, vp(o), vp(inf), None) == 0
        # a wire length past the wire's block
        assert L.wsg_decode_batch(c._ctx, vp(w), 3 << 20, vp(f), 1, vp(o), vp(inf), None) == ca.WSG_EINVAL
        c.sync_status()
        # encode: a descriptor whose payload range runs past the payload block
        payload = hip_alloc(1 << 20)
        desc = np.zeros(2, dtype=SEND_DESC)
        desc["len"], desc["opcode"] = 1000, 0x82
        desc["src_off"][1] = (1 << 20) - 10
        d = ca.desc_to_tensor(desc, "cuda")
        wire_o = torch.empty(4096, dtype=torch.uint8, device="cuda")
        off = torch.empty(3, dtype=torch.int64, device="cuda")
        args = (c._ctx, vp(payload), vp(d.data_ptr()), 2, vp(wire_o.data_ptr()), 4096, vp(off.data_ptr()), None)
        assert L.wsg_encode_batch(*args) == ca.WSG_EINVAL
        desc["src_off"][1] = 0
        d.copy_(ca.desc_to_tensor(desc, "cuda"))
        assert L.wsg_encode_batch(*args) == 0
        assert c.sync_status() == 0 and int(off[2].item()) == 2 * 1004
        # fan-out: 100 frames of 1004 B into a 64 KiB block with a larger stated capacity
        keys = dev(np.arange(100, dtype=np.int32))
        small = hip_alloc(64 << 10)
        assert L.wsg_fanout_encode(c._ctx, vp(payload), 1000, vp(keys.data_ptr()), 100, 0x82, 1, vp(small),
                                   1 << 20, None) == ca.WSG_EINVAL
        torch.cuda.synchronize()
    finally:
        c.close()
        for p in blocks:
            hip.hipFree(p)


def test_prepare_fanout_matches_oracle(codec):
    """Codec.prepare_fanout (the bench's pre-bound C-ABI fan-out) writes the
    oracle's frames, launch after launch."""
    payload, keys = wl.c4_fanout(4096, 777, seed=31)
    ref = oracle.fanout_encode(payload, keys, 0x82, True)
    wire = torch.full((len(ref) + 32,), 0xA5, dtype=torch.uint8, device="cuda")
    launch = codec.prepare_fanout(dev(payload), dev(keys.view(np.int32)), 0x82, True, wire)
    for _ in range(3):
        launch()
    assert codec.sync_status() == 0
    got = wire.cpu().numpy()
    assert np.array_equal(got[: len(ref)], ref) and (got[len(ref):] == 0xA5).all()
