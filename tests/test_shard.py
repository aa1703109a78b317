"""Multi-process sharding and the C5 gather on CPU: world_size 2 and 3 over
gloo (127.0.0.1).  Each rank encodes its round-robin shard with the oracle
(the same per-rank work the GPU does through wsg_encode_batch), gathers to
rank 0 with cppserver_amd.shard.gather_frames, and rank 0 checks that the
reassembled job is byte-identical to encoding the whole job in one batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from cppserver_amd import shard
from cppserver_amd.layout import SEND_DESC


def _job(n_total, seed=5):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, n_total)
    keys = rng.integers(0, 2**32, n_total, dtype=np.uint64).astype(np.uint32)
    ops = rng.choice([0x81, 0x82, 0x88, 0x89], n_total)
    data = [rng.integers(0, 256, int(l), dtype=np.uint8) for l in lens]
    return lens, keys, ops, data


def _batch(ids, lens, keys, ops, data):
    desc = np.zeros(len(ids), dtype=SEND_DESC)
    offs = np.zeros(len(ids), dtype=np.uint64)
    if len(ids) > 1:
        offs[1:] = np.cumsum(lens[ids][:-1])
    desc["src_off"] = offs
    desc["len"] = lens[ids]
    desc["key"] = keys[ids]
    desc["opcode"] = ops[ids]
    desc["mask"] = 1
    payload = np.concatenate([data[i] for i in ids] + [np.zeros(1, np.uint8)])
    return payload, desc


def _worker(rank, world, port, n_total, chunk, results):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        job = _job(n_total)
        ids = shard.rank_frames(rank, world, n_total, chunk)
        payload, desc = _batch(ids, *job)
        wire, off = oracle.encode_batch(payload, desc)
        parts = shard.gather_frames(torch.from_numpy(wire.copy()), torch.from_numpy(off.view(np.int64).copy()))
        if rank == 0:
            got, got_off = shard.reassemble(parts, n_total, chunk)
            ref, ref_off = oracle.encode_batch(*_batch(np.arange(n_total), *job))
            results[0] = bool(np.array_equal(got.numpy(), ref) and
                              np.array_equal(got_off.numpy().view(np.uint64), ref_off))
        else:
            assert parts is None
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,n_total,chunk", [(2, 300, 16), (3, 257, 10), (2, 5, 8)])
def test_gather_reassembles_job(world, n_total, chunk):
    results = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _free_port(), n_total, chunk, results), nprocs=world, join=True)
    assert results.get(0) is True


def test_rank_frames_partition():
    n, chunk = 10000, 64
    for world in (1, 2, 3, 8):
        parts = [shard.rank_frames(r, world, n, chunk) for r in range(world)]
        allf = np.sort(np.concatenate(parts))
        assert np.array_equal(allf, np.arange(n))
        for r, p in enumerate(parts):
            assert ((p // chunk) % world == r).all()
