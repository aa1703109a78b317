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
