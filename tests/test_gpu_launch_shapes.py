"""Launch shapes of the batch kernels against the oracle (round 3).

The encode grid now covers every piece (one wave per piece, up to 2^31
threads); grid-stride returns beyond that, and the piece kernel can run as
several launches over piece ranges (`WSG_ENC_LAUNCH_PIECES`, an A/B knob).
Each shape must give the same bytes: the grid-stride path is forced here with
a 1-block-per-CU grid, the piece ranges with odd run lengths.  Also the
measurement hooks bench.py reads (per-launch extremes) and the prepared
launch's argument checks.
"""
import os

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def _codec(**env):
    keys = ("WSG_ENC_BLOCKS_PER_CU", "WSG_ENC_LAUNCH_PIECES")
    for k in keys:
        os.environ.pop(k, None)
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return ca.Codec(0)
    finally:
        for k in keys:
            os.environ.pop(k, None)


def _ragged(n, lo, hi, seed):
    rng = np.random.default_rng(seed)
    desc, total = wl.ragged_desc(rng, rng.integers(lo, hi + 1, n))
    desc["opcode"] = rng.choice([0x81, 0x82, 0x88, 0x89, 0x02], n)
    desc["status"] = np.where(desc["opcode"] == 0x88, 1001, 0)
    desc["mask"] = rng.integers(0, 2, n)
    return wl.random_bytes(rng, max(total, 1)), desc


@pytest.mark.parametrize("env", [dict(WSG_ENC_BLOCKS_PER_CU=1), dict(WSG_ENC_BLOCKS_PER_CU=3),
                                 dict(WSG_ENC_LAUNCH_PIECES=37), dict(WSG_ENC_LAUNCH_PIECES=1000),
                                 dict(WSG_ENC_BLOCKS_PER_CU=2, WSG_ENC_LAUNCH_PIECES=4097), {}],
                         ids=lambda e: ",".join("%s=%s" % kv for kv in e.items()) or "default")
def test_encode_launch_shapes_vs_oracle(env):
    payload, desc = _ragged(3000, 4000, 70000, seed=sum(map(int, env.values())) + 1)
    ref, ref_off = oracle.encode_batch(payload, desc)
    c = _codec(**env)
    try:
        w, off = c.encode_batch(torch.from_numpy(payload).cuda(), ca.desc_to_tensor(desc, "cuda"),
                                wire_cap=len(ref) + 64)
        c.sync()
        assert np.array_equal(off.cpu().numpy().view(np.uint64), ref_off)
        assert np.array_equal(w.cpu().numpy()[: len(ref)], ref)
    finally:
        c.close()


def test_c5_shape_grid_stride_vs_covering():
    """C5-shape frames (16 KiB payloads, 5 pieces each) with the old 1024
    blocks/CU cap (grid-stride once pieces outnumber waves) and the covering
    grid: same bytes, both against the oracle on sampled frames."""
    n = 1 << 16
    ids = np.arange(n)
    payload = wl.c5_payload_torch(ids, 16384, device="cuda")
    desc = ca.desc_to_tensor(wl.c5_desc(ids, 16384), "cuda")
    fsz = ca.frame_size(0x82, True, 16384)
    outs = []
    for env in (dict(WSG_ENC_BLOCKS_PER_CU=16), {}):   # 16 blocks/CU: ~20 pieces per wave
        c = _codec(**env)
        try:
            w, _ = c.encode_batch(payload, desc, wire_cap=n * fsz)
            c.sync()
            outs.append(w)
        finally:
            c.close()
    assert torch.equal(outs[0], outs[1])
    for g in (0, 1, 777, n - 1):
        ref, _ = oracle.encode_batch(wl.c5_payload_np(np.array([g]), 16384), wl.c5_desc(np.array([g]), 16384))
        assert np.array_equal(outs[1][g * fsz: (g + 1) * fsz].cpu().numpy(), ref)


def test_timing_minmax():
    c = ca.Codec(0)
    try:
        wire, fs, _ = wl.c2_wire(256, 65536, seed=9)
        w = torch.from_numpy(wire).cuda()
        f = torch.from_numpy(fs.view(np.int64)).cuda()
        out = torch.empty_like(w)
        c.timing(True, 1)
        c.timing_read(reset=True)
        for _ in range(5):
            c.decode_batch(w, f, out=out)
        lo, hi = c.timing_minmax()
        total, launches = c.timing_read(reset=True)
        assert launches == 5
        assert 0 < lo <= total / launches <= hi
        assert c.timing_minmax() == (0.0, 0.0)   # reset clears the extremes
        c.timing(False)
    finally:
        c.close()


def test_prepared_launch_checks():
    c = ca.Codec(0)
    try:
        w = torch.zeros(4096, dtype=torch.uint8, device="cuda")
        f = torch.zeros(4, dtype=torch.int64, device="cuda")
        with pytest.raises(ca.WSGError):
            c.prepare_decode(w, f, torch.empty(100, dtype=torch.uint8, device="cuda"),
                             torch.empty(4 * 32, dtype=torch.uint8, device="cuda"))
        keys = torch.zeros(10, dtype=torch.int32, device="cuda")
        with pytest.raises(ca.WSGError):
            c.prepare_fanout(w[:64], keys, 0x82, True, torch.empty(100, dtype=torch.uint8, device="cuda"))
        # stream=None: the launch uses torch's current stream at launch time
        wire, fs, _ = wl.c2_wire(8, 1000, seed=3)
        ww = torch.from_numpy(wire).cuda()
        ff = torch.from_numpy(fs.view(np.int64)).cuda()
        out = torch.empty_like(ww)
        info = torch.empty(8 * 32, dtype=torch.uint8, device="cuda")
        launch = c.prepare_decode(ww, ff, out, info)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            launch()
        s.synchronize()
        rc, ref, _ = oracle.decode_batch(wire, fs)
        assert rc == 0 and np.array_equal(out.cpu().numpy(), ref)
    finally:
        c.close()


def test_encode_refuses_piece_bound_past_u32():
    """a wire_cap whose piece bound passes 2^32 (the launch's u32
    piece indices) is refused with WSG_EINVAL instead of wrapping q_end
    below q_begin and skipping pieces silently."""
    import torch

    import cppserver_amd as ca
    from cppserver_amd import workloads as wl

    codec = ca.Codec(0)
    rng = np.random.default_rng(3)
    desc, total = wl.ragged_desc(rng, np.full(4, 70000))
    payload = torch.from_numpy(wl.random_bytes(rng, total)).cuda()
    d = ca.desc_to_tensor(desc, "cuda")
    wire = torch.empty(4 * 70016, dtype=torch.uint8, device="cuda")
    woff = torch.empty(5, dtype=torch.int64, device="cuda")
    lib = ca.lib()
    import ctypes

    rc = lib.wsg_encode_batch(codec._ctx, ctypes.c_void_p(payload.data_ptr()), ctypes.c_void_p(d.data_ptr()), 4,
                              ctypes.c_void_p(wire.data_ptr()), 1 << 45, ctypes.c_void_p(woff.data_ptr()),
                              codec._stream(None))
    assert rc == ca.WSG_EINVAL
    w, off = codec.encode_batch(payload, d, wire=wire, wire_off=woff)   # a real capacity still encodes
    codec.sync()
    assert int(off[-1].item()) == int(ca.frame_sizes(desc).sum())
    codec.close()
