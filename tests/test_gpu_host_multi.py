"""One host batch over several contexts (wsg_decode_batch_host_multi /
wsg_encode_batch_host_multi, and the wsg_mgpu forms): results and status
must be those of the one-context host call, i.e. the oracle's, wherever the
runs are cut.  On the one-GPU box the contexts share device 0, which
exercises the split, the per-run rebasing and the status merge exactly as
distinct GPUs would (only the PCIe links are shared).
"""
import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
from cppserver_amd.layout import SEND_DESC  # noqa: E402
from tests.test_gpu_parity import INFO_FIELDS, _frames_wire, _mixed_desc  # noqa: E402


@pytest.fixture(scope="module")
def codecs():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    cs = [ca.Codec(0) for _ in range(4)]
    yield cs
    for c in cs:
        c.close()


@pytest.fixture(autouse=True)
def share_device(monkeypatch):
    # the library splits over one context per device; the one-GPU box needs
    # every context of device 0 to take a run for the split to be exercised
    monkeypatch.setenv("WSG_HOST_MULTI_SHARE", "1")


def _pin(a):
    p = ca.pinned_empty(len(a))
    p[:] = a
    return p


def _check_decode(codecs, k, wire, fs, pinned=False):
    rc_o, out_o, info_o = oracle.decode_batch(wire, fs)
    src = _pin(wire) if pinned else wire
    rc, out, info = ca.decode_batch_host_multi(codecs[:k], src, fs)
    assert rc == rc_o, (k, rc, rc_o)
    assert np.array_equal(out, out_o)
    for f in INFO_FIELDS:
        assert np.array_equal(info[f], info_o[f]), f
    return rc


@pytest.mark.parametrize("k", [2, 3, 4])
@pytest.mark.parametrize("case", ["ragged", "gaps", "lead-gap", "tiny"])
def test_decode_multi_vs_oracle(codecs, k, case):
    rng = np.random.default_rng(k * 100 + len(case))
    gaps, lead = None, 0
    if case == "ragged":
        lens = rng.integers(0, 70000, 300)
    elif case == "gaps":
        lens = rng.integers(0, 5000, 500)
        gaps = rng.integers(0, 40, 500) * (rng.random(500) < 0.5)
    elif case == "lead-gap":
        lens = rng.integers(100, 3000, 200)
        lead = 40000
    else:
        lens = rng.integers(0, 40, 3000)
    wire, fs = _frames_wire(rng, lens.astype(np.uint64), gaps, lead)
    assert _check_decode(codecs, k, wire, fs) == 0
    assert _check_decode(codecs, k, wire, fs, pinned=True) == 0


@pytest.mark.parametrize("k", [2, 4])
def test_decode_multi_errors_vs_oracle(codecs, k):
    """Truncated last frame, a frame that overlaps the next one at every
    position around the run cuts, frames starting past the wire's end: the
    status and every frame's fields are the oracle's (and so the one-context
    call's)."""
    rng = np.random.default_rng(7 + k)
    payload, desc = _mixed_desc(rng, 400, 0, 20000)
    wire, off = oracle.encode_batch(payload, desc)
    fs = off[:-1].copy()
    variants = [("trunc", wire[:-5], fs)]
    for at in sorted({1, 50, 100, 133, 199, 200, 201, 266, 300, 399}):
        f = fs.copy()
        f[at] += 1   # frame at - 1 overlaps frame at
        variants.append(("overlap%d" % at, wire, f))
    past = np.concatenate([fs, np.array([len(wire) + 3, len(wire) + 40], np.uint64)])
    variants.append(("past-end", wire, past))
    errs = 0
    for name, w, f in variants:
        rc_o, _, _ = oracle.decode_batch(w, f)
        assert _check_decode(codecs, k, w, f) == rc_o, name
        errs += rc_o != 0
    assert errs >= 2   # the truncated and past-the-end batches at least


def test_decode_multi_unsorted_falls_back(codecs):
    rng = np.random.default_rng(3)
    lens = rng.integers(0, 3000, 300).astype(np.uint64)
    wire, fs = _frames_wire(rng, lens)
    bad = fs.copy()
    bad[10], bad[11] = bad[11], bad[10]
    rc_o, _, info_o = oracle.decode_batch(wire, bad)
    rc, _, info = ca.decode_batch_host_multi(codecs, wire, bad)
    assert rc == rc_o
    assert np.array_equal(info["error"], info_o["error"])


def test_decode_multi_small_batches(codecs):
    """Fewer frames than contexts, one frame, none."""
    rng = np.random.default_rng(11)
    for lens in ([5], [70000, 3], [0, 1, 2]):
        wire, fs = _frames_wire(rng, np.array(lens, np.uint64))
        assert _check_decode(codecs, 4, wire, fs) == 0
    junk = wl.random_bytes(rng, 100)
    rc, out, info = ca.decode_batch_host_multi(codecs, junk, np.zeros(0, np.uint64))
    assert rc == 0 and np.array_equal(out, junk) and len(info) == 0


def test_decode_multi_c2_size(codecs):
    """BASELINE C2 (4096 x 64 KiB) from pinned host memory over 4 contexts."""
    wire, fs, _ = wl.c2_wire(4096, 65536, seed=21)
    assert _check_decode(codecs, 4, wire, fs, pinned=True) == 0


@pytest.mark.parametrize("k", [2, 3, 4])
@pytest.mark.parametrize("lo,hi,n", [(0, 300, 3000), (100, 70000, 300), (0, 40, 5)])
def test_encode_multi_vs_oracle(codecs, k, lo, hi, n):
    rng = np.random.default_rng(k * 1000 + n)
    payload, desc = _mixed_desc(rng, n, lo, hi)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    for pinned in (False, True):
        p = _pin(payload) if pinned else payload
        out = ca.pinned_empty(max(len(wire_o), 1)) if pinned else None
        rc, wire, off = ca.encode_batch_host_multi(codecs[:k], p, desc, wire=out)
        assert rc == 0
        assert np.array_equal(off, off_o)
        assert np.array_equal(wire, wire_o)


def test_encode_multi_errors(codecs):
    payload = np.zeros(1000, np.uint8)
    desc = np.zeros(8, dtype=SEND_DESC)
    desc["len"] = 100
    desc["opcode"] = 0x82
    rc, _, _ = ca.encode_batch_host_multi(codecs, payload, desc, wire=np.empty(300, np.uint8))
    assert rc == ca.WSG_ENOMEM
    desc["src_off"][5] = 950   # runs past the payload
    rc, _, _ = ca.encode_batch_host_multi(codecs, payload, desc)
    assert rc == ca.WSG_EINVAL
    rc, wire, off = ca.encode_batch_host_multi(codecs, payload, desc[:0])
    assert rc == 0 and off[0] == 0


def test_one_context_per_device_by_default(codecs, monkeypatch):
    """Without the knob, four contexts of one GPU take the one-context path
    (same results)."""
    monkeypatch.delenv("WSG_HOST_MULTI_SHARE")
    rng = np.random.default_rng(9)
    wire, fs = _frames_wire(rng, rng.integers(0, 9000, 200).astype(np.uint64))
    assert _check_decode(codecs, 4, wire, fs) == 0


def test_mgpu_host_paths_world1():
    """The wsg_mgpu forms over the group's local GPUs (RCCL group of one on
    the one-GPU box)."""
    g = ca.MultiGPU([0])
    try:
        rng = np.random.default_rng(5)
        payload, desc = _mixed_desc(rng, 500, 0, 20000)
        wire_o, off_o = oracle.encode_batch(payload, desc)
        rc, wire, off = g.encode_batch_host(payload, desc)
        assert rc == 0 and np.array_equal(wire, wire_o) and np.array_equal(off, off_o)
        rc_o, out_o, info_o = oracle.decode_batch(wire_o, off_o[:-1])
        rc, out, info = g.decode_batch_host(wire_o, off_o[:-1])
        assert rc == rc_o == 0 and np.array_equal(out, out_o)
        for f in INFO_FIELDS:
            assert np.array_equal(info[f], info_o[f]), f
    finally:
        g.close()
