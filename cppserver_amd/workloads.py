"""Seeded synthetic batches for the BASELINE.json configurations (host numpy).

C2  unmask-only: n masked binary frames of `size` payload bytes, one random
    32-bit key per frame (client frames, ws.cpp:241-248).
C3  round trip: n frames, payload length uniform in [lo, hi] (ragged).
C4  fan-out: one payload, k client keys.
C5  round-robin shard of N x size frames for rank r of w ranks.
"""
import numpy as np

from .layout import SEND_DESC, WS_BINARY, WS_FIN


def random_bytes(rng, n):
    return np.frombuffer(rng.bytes(int(n)), dtype=np.uint8).copy()


def c2_wire(n=4096, size=65536, seed=2):
    """n masked 0x82 frames back to back.  Returns (wire, frame_start, keys).

    The wire's payload bytes are random (masking random bytes is still random
    bytes); each header is the exact header PrepareSendFrame emits for a
    masked binary frame of `size` bytes (ws.cpp:222-248)."""
    rng = np.random.default_rng(seed)
    keys = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    if size < 126:
        ext = b""
        b1 = 0x80 | size
    elif size < 65536:
        ext = size.to_bytes(2, "big")
        b1 = 0x80 | 126
    else:
        ext = size.to_bytes(8, "big")
        b1 = 0x80 | 127
    hdr_len = 2 + len(ext) + 4
    fsz = hdr_len + size
    wire = random_bytes(rng, n * fsz).reshape(n, fsz)
    wire[:, 0] = WS_FIN | WS_BINARY
    wire[:, 1] = b1
    if ext:
        wire[:, 2: 2 + len(ext)] = np.frombuffer(ext, dtype=np.uint8)
    wire[:, 2 + len(ext): hdr_len] = keys.view(np.uint8).reshape(n, 4)
    frame_start = (np.arange(n, dtype=np.uint64) * np.uint64(fsz))
    return wire.reshape(-1), frame_start, keys


def ragged_desc(rng, lens, opcode=WS_FIN | WS_BINARY, mask=True, align=1):
    """Descriptors for payloads packed back to back (offsets rounded to `align`)."""
    n = len(lens)
    lens = np.asarray(lens, dtype=np.uint64)
    padded = ((lens + np.uint64(align - 1)) // np.uint64(align)) * np.uint64(align)
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(padded[:-1])
    desc = np.zeros(n, dtype=SEND_DESC)
    desc["src_off"] = offs
    desc["len"] = lens
    desc["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    desc["opcode"] = opcode
    desc["mask"] = 1 if mask else 0
    total = int(offs[-1] + padded[-1]) if n else 0
    return desc, total


def c3_batch(n=65536, lo=128, hi=65536, seed=3):
    """Ragged round-trip batch: returns (payload, desc)."""
    rng = np.random.default_rng(seed)
    lens = rng.integers(lo, hi + 1, n)
    desc, total = ragged_desc(rng, lens)
    payload = random_bytes(rng, max(total, 1))
    return payload, desc


def c4_fanout(length=4096, k=10000, seed=4):
    rng = np.random.default_rng(seed)
    payload = random_bytes(rng, length)
    keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
    return payload, keys


def c5_rank_frames(rank, world, n_total=1 << 20, chunk=1024):
    """Frame indices owned by `rank` (chunks dealt round-robin, shard.py)."""
    from .shard import rank_frames

    return rank_frames(rank, world, n_total, chunk)


_M32 = 0xFFFFFFFF


def _mix32(x, xp):
    """32-bit integer hash (xorshift-multiply) on non-negative int64/uint64
    arrays holding 32-bit values; every product stays below 2**63, so numpy
    (uint64) and torch (int64, CPU or GPU) compute the same words."""
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x2C1B3C6D) & _M32
    return x ^ (x >> 12)


def c5_key_of(ids):
    """Key of global frame g (splitmix-like hash of g): the same job at any
    world size."""
    g = np.asarray(ids).astype(np.uint64)
    z = (g + np.uint64(0x9E3779B97F4A7C15)) * np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(31)
    return (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)


def c5_payload_np(ids, size=16384):
    """Payload bytes of global frames `ids` (a function of the frame index
    only, so any shard of the job regenerates its frames), host numpy."""
    assert size % 4 == 0
    w = size // 4
    g = np.asarray(ids, dtype=np.uint64)[:, None]
    x = (g * np.uint64(w) + np.arange(w, dtype=np.uint64)[None, :]) & np.uint64(_M32)
    return _mix32(x, np).astype(np.uint32).view(np.uint8).reshape(-1)


def c5_payload_torch(ids, size=16384, device="cuda", step=1 << 14):
    """c5_payload_np computed on the device (the 16 GiB job of C5 is made in
    HBM, not on the host): uint8 tensor of len(ids) * size bytes."""
    import torch

    assert size % 4 == 0
    w = size // 4
    ids = torch.as_tensor(np.asarray(ids, dtype=np.int64), device=device)
    out = torch.empty(len(ids) * size, dtype=torch.uint8, device=device)
    words = out.view(torch.int32).view(len(ids), w)
    j = torch.arange(w, dtype=torch.int64, device=device)[None, :]
    for a in range(0, len(ids), step):
        g = ids[a: a + step, None]
        x = (g * w + j) & _M32
        x = _mix32(x, torch)
        words[a: a + step] = (x - ((x >> 31) << 32)).to(torch.int32)   # wrap to signed 32-bit
    return out


def c5_desc(ids, size=16384):
    """Descriptors of a shard whose payloads lie back to back (local order)."""
    n = len(ids)
    desc = np.zeros(n, dtype=SEND_DESC)
    desc["src_off"] = np.arange(n, dtype=np.uint64) * np.uint64(size)
    desc["len"] = size
    desc["key"] = c5_key_of(ids)
    desc["opcode"] = WS_FIN | WS_BINARY
    desc["mask"] = 1
    return desc


def c5_shard(rank, world, n_total=1 << 20, size=16384, chunk=1024, seed=5, max_frames=None):
    """This rank's encode batch: (payload, desc, frame_ids).  Keys derive from
    the global frame index (shards are disjoint, the key set is the same job
    at any world size); payload bytes are seeded per shard."""
    ids = c5_rank_frames(rank, world, n_total, chunk)
    if max_frames is not None:
        ids = ids[:max_frames]
    n = len(ids)
    rng = np.random.default_rng([seed, rank, world])
    desc = np.zeros(n, dtype=SEND_DESC)
    desc["src_off"] = np.arange(n, dtype=np.uint64) * np.uint64(size)
    desc["len"] = size
    # key of frame g = splitmix-like hash of g: identical across world sizes
    g = ids.astype(np.uint64)
    z = (g + np.uint64(0x9E3779B97F4A7C15)) * np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(31)
    desc["key"] = (z & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    desc["opcode"] = WS_FIN | WS_BINARY
    desc["mask"] = 1
    payload = random_bytes(rng, n * size)
    return payload, desc, ids
