"""BASELINE config C5 (1 Mi x 16 KiB frames sharded round-robin over the GPUs
of a node, framed output gathered to one rank) on the GPU.

* the full-size job on one GPU: every one of the 1 Mi frames checked against
  an independent torch restatement of PrepareSendFrame's bytes
  (ws.cpp:222-270: header 82 fe 40 00 + key, payload XOR key), and the first
  64 Ki frames byte for byte against the oracle;
* the multi-process flow at world size 2 (gloo, both ranks on cuda:0): each
  rank encodes its shard with the HIP kernels, the shards are gathered and
  reassembled, and the job equals the oracle's encode of the whole job;
* the C-ABI multi-GPU entry (wsg_mgpu_encode_gather): the one-process form
  at world sizes 1, 2, 3 and 8 with every rank on the one GPU (device
  copies to the root), chunk sizes 1, 300, 700 and 1024, ragged jobs, other
  roots, ranks holding nothing, an encode error on a non-root rank; the
  RCCL rank-per-process form at world size 1 over the real RCCL, and at
  world sizes 2, 3 and 8 with ranks as threads over a loopback RCCL test
  double (tests/cpp/loopback_rccl.cpp); all against the oracle.
"""
import os
import socket

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import shard  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
from cppserver_amd.layout import SEND_DESC, frame_size  # noqa: E402

SIZE = 16384
FSZ = frame_size(0x82, True, SIZE)   # 16392: 8-byte header (126 form + key)


@pytest.fixture(scope="module")
def codec():
    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    c = ca.Codec(0)
    yield c
    c.close()


def test_c5_payload_generators_agree():
    ids = np.array([0, 1, 2, 1023, 1024, 77777, (1 << 20) - 1])
    host = wl.c5_payload_np(ids, SIZE)
    dev = wl.c5_payload_torch(ids, SIZE, device="cuda").cpu().numpy()
    assert np.array_equal(host, dev)


def _expected_words(ids_dev, keys_dev):
    """Frame words (int32, little-endian) PrepareSendFrame emits for masked
    0x82 frames of SIZE bytes: 82 fe 40 00 | key | payload ^ key."""
    n = ids_dev.numel()
    pay = wl.c5_payload_torch(ids_dev.cpu().numpy(), SIZE, device="cuda").view(torch.int32).view(n, SIZE // 4)
    k = keys_dev.view(n, 1)
    hdr = torch.full((n, 1), 0x0040FE82, dtype=torch.int32, device="cuda")
    return torch.cat([hdr, k, pay ^ k], dim=1)


def test_c5_full_size_one_gpu(codec):
    n = 1 << 20
    ids = np.arange(n, dtype=np.int64)
    payload = wl.c5_payload_torch(ids, SIZE, device="cuda")          # 16 GiB in HBM
    desc = wl.c5_desc(ids, SIZE)
    cap = n * FSZ
    wire, off = codec.encode_batch(payload, ca.desc_to_tensor(desc, "cuda"), wire_cap=cap)
    codec.sync()
    offs = off.cpu().numpy()
    assert np.array_equal(offs, np.arange(n + 1, dtype=np.int64) * FSZ)
    # every frame against the torch restatement
    keys = torch.from_numpy(desc["key"].view(np.int32).copy()).cuda()
    words = wire[:cap].view(torch.int32).view(n, FSZ // 4)
    step = 1 << 16
    ids_dev = torch.from_numpy(ids).cuda()
    for a in range(0, n, step):
        exp = _expected_words(ids_dev[a: a + step], keys[a: a + step])
        assert torch.equal(words[a: a + step], exp), "frames %d.." % a
    # the first 64 Ki frames (1 GiB) byte for byte against the oracle
    sub = 1 << 16
    wire_o, off_o = oracle.encode_batch(payload[: sub * SIZE].cpu().numpy(), desc[:sub])
    assert np.array_equal(wire[: sub * FSZ].cpu().numpy(), wire_o)
    assert np.array_equal(off_o, offs[: sub + 1].astype(np.uint64))
    del payload, wire, words


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gloo_worker(rank, world, port, n_total, chunk, results):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c = ca.Codec(0)
        ids = shard.rank_frames(rank, world, n_total, chunk)
        payload = wl.c5_payload_torch(ids, SIZE, device="cuda")
        desc = wl.c5_desc(ids, SIZE)
        wire, off = c.encode_batch(payload, ca.desc_to_tensor(desc, "cuda"), wire_cap=len(ids) * FSZ)
        c.sync()
        parts = shard.gather_frames(wire.cpu(), off.cpu())
        if rank == 0:
            got, got_off = shard.reassemble(parts, n_total, chunk)
            allids = np.arange(n_total)
            ref, ref_off = oracle.encode_batch(wl.c5_payload_np(allids, SIZE), wl.c5_desc(allids, SIZE))
            results[0] = bool(np.array_equal(got.numpy(), ref) and
                              np.array_equal(got_off.numpy().view(np.uint64), ref_off))
        c.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_total,chunk", [(16384, 1024), (5000, 700)])
def test_c5_world2_gloo_hip_encode(n_total, chunk):
    import torch.multiprocessing as mp

    results = mp.Manager().dict()
    mp.spawn(_gloo_worker, args=(2, _free_port(), n_total, chunk, results), nprocs=2, join=True)
    assert results.get(0) is True


def _ragged_job(n, seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 3000, n)
    big = rng.random(n) < 0.05
    lens[big] = rng.integers(60000, 70000, int(big.sum()))
    desc, total = wl.ragged_desc(rng, lens)
    desc["opcode"] = rng.choice([0x81, 0x82, 0x88, 0x89], n)
    desc["status"] = np.where(desc["opcode"] == 0x88, 1000, 0)
    return wl.random_bytes(rng, max(total, 1)), desc


def _mgpu_check(g, payload, desc, chunk):
    n = len(desc)
    ref, ref_off = oracle.encode_batch(payload, desc)
    # world 1: the shard is the whole job, in order
    assert ca.MultiGPU.shard_count(n, chunk, 1, 0) == n
    cap = int(ref_off[-1]) + 16
    p = torch.from_numpy(payload).cuda()
    d = ca.desc_to_tensor(desc, "cuda")
    wire = torch.empty(cap, dtype=torch.uint8, device="cuda")
    woff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    out = torch.full((cap + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    enc_ms, gat_ms = g.encode_gather(n, chunk, [p], [d], [wire], [woff], root=0, out=out, out_off=out_off)
    got = out.cpu().numpy()
    assert np.array_equal(got[: len(ref)], ref)
    assert (got[len(ref):] == 0xA5).all()
    assert np.array_equal(out_off.cpu().numpy().view(np.uint64), ref_off)
    assert enc_ms >= 0 and gat_ms >= 0


@pytest.mark.parametrize("n,chunk", [(3000, 1024), (1000, 1), (4096, 1024)])
def test_mgpu_single_process_world1(n, chunk):
    g = ca.MultiGPU([0])
    assert (g.world, g.nlocal, g.first_rank) == (1, 1, 0)
    try:
        _mgpu_check(g, *_ragged_job(n, seed=n + chunk), chunk)
    finally:
        g.close()


def test_mgpu_rank_world1_c5_shape():
    g = ca.MultiGPU.rank(0, ca.MultiGPU.unique_id(), 0, 1)
    try:
        ids = np.arange(4096)
        _mgpu_check(g, wl.c5_payload_np(ids, SIZE), wl.c5_desc(ids, SIZE), 1024)
    finally:
        g.close()


def test_mgpu_rejects_wrong_shard():
    g = ca.MultiGPU([0])
    try:
        payload, desc = _ragged_job(100, seed=3)
        p = torch.from_numpy(payload).cuda()
        d = ca.desc_to_tensor(desc[:50], "cuda")   # half the job is not world 1's shard
        w = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
        o = torch.empty(51, dtype=torch.int64, device="cuda")
        with pytest.raises(ca.WSGError) as e:
            g.encode_gather(100, 10, [p], [d], [w], [o], out=w.clone())
        assert e.value.code == ca.WSG_EINVAL
    finally:
        g.close()


def _world_job(world, n, chunk, seed, root=0, bad_rank=None):
    """The one-process group at `world` ranks, all on device 0: the job's
    round-robin shards encoded per rank, gathered to `root` by device
    copies; the root's wire and offsets against the oracle's encode of the
    whole job.  bad_rank: that rank's wire buffer is too short (its encode
    latches WSG_ENOMEM), which must stop the call on every rank."""
    payload, desc = _ragged_job(n, seed)
    ref, ref_off = oracle.encode_batch(payload, desc)
    g = ca.MultiGPU([0] * world)
    assert (g.world, g.nlocal, g.first_rank) == (world, world, 0)
    try:
        p = torch.from_numpy(payload).cuda()   # every rank's descriptors point into the one arena
        descs, wires, woffs = [], [], []
        for r in range(world):
            ids = shard.rank_frames(r, world, n, chunk)
            assert len(ids) == ca.MultiGPU.shard_count(n, chunk, world, r)
            d = desc[ids]
            cap = int(ca.frame_sizes(d).sum()) if len(ids) else 0
            if r == bad_rank:
                cap //= 2
            descs.append(ca.desc_to_tensor(d, "cuda") if len(ids) else torch.empty(0, dtype=torch.uint8,
                                                                                   device="cuda"))
            wires.append(torch.empty(max(cap, 16), dtype=torch.uint8, device="cuda"))
            woffs.append(torch.empty(len(ids) + 1, dtype=torch.int64, device="cuda"))
        out = torch.full((len(ref) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
        out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        if bad_rank is not None:
            with pytest.raises(ca.WSGError) as e:
                g.encode_gather(n, chunk, [p] * world, descs, wires, woffs, root=root, out=out, out_off=out_off)
            assert e.value.code == ca.WSG_ENOMEM
            return
        enc_ms, gat_ms = g.encode_gather(n, chunk, [p] * world, descs, wires, woffs, root=root, out=out,
                                         out_off=out_off)
        got = out.cpu().numpy()
        assert np.array_equal(got[: len(ref)], ref)
        assert (got[len(ref):] == 0xA5).all()
        assert np.array_equal(out_off.cpu().numpy().view(np.uint64), ref_off)
        assert enc_ms >= 0 and gat_ms >= 0
    finally:
        g.close()


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("n,chunk", [(1000, 1), (5000, 700), (9000, 1024)])
def test_mgpu_world_n_one_device(world, n, chunk):
    """the world > 1 placement (chunk sizes, chunk offsets
    in job order, per-chunk transfers, rank-by-rank offset stage, rebase) run
    with every rank on the one GPU."""
    _world_job(world, n, chunk, seed=world * 7919 + n + chunk)


@pytest.mark.parametrize("world,root", [(3, 2), (8, 5)])
def test_mgpu_world_n_other_root(world, root):
    _world_job(world, 4000, 300, seed=11 + world, root=root)


def test_mgpu_world_fewer_chunks_than_ranks():
    """8 ranks, 3 chunks: five ranks hold nothing."""
    _world_job(8, 2500, 1024, seed=5)


@pytest.mark.parametrize("bad_rank", [1, 2])
def test_mgpu_error_on_non_root_rank(bad_rank):
    """An encode error on a non-root rank stops the whole call (status round)."""
    _world_job(3, 3000, 500, seed=17, root=0, bad_rank=bad_rank)


def test_mgpu_world8_c5_shape_one_device():
    """C5-shape frames (16 KiB payloads) at world 8 on one device, 64 Ki frames."""
    n, chunk = 1 << 16, 1024
    g = ca.MultiGPU([0] * 8)
    try:
        ids_all = np.arange(n)
        ref_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(FSZ)
        payloads, descs, wires, woffs = [], [], [], []
        for r in range(8):
            ids = shard.rank_frames(r, 8, n, chunk)
            payloads.append(wl.c5_payload_torch(ids, SIZE, device="cuda"))
            descs.append(ca.desc_to_tensor(wl.c5_desc(ids, SIZE), "cuda"))
            wires.append(torch.empty(len(ids) * FSZ, dtype=torch.uint8, device="cuda"))
            woffs.append(torch.empty(len(ids) + 1, dtype=torch.int64, device="cuda"))
        out = torch.empty(n * FSZ, dtype=torch.uint8, device="cuda")
        out_off = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        g.encode_gather(n, chunk, payloads, descs, wires, woffs, root=0, out=out, out_off=out_off)
        assert np.array_equal(out_off.cpu().numpy().view(np.uint64), ref_off)
        keys = torch.from_numpy(wl.c5_desc(ids_all, SIZE)["key"].view(np.int32).copy()).cuda()
        words = out.view(torch.int32).view(n, FSZ // 4)
        exp = _expected_words(torch.from_numpy(ids_all).cuda(), keys)
        assert torch.equal(words, exp)
    finally:
        g.close()


def test_mgpu_rank_form_world_n():
    """The RCCL rank-per-process form at world 2, 3 and 8 on one GPU: ranks
    are threads, RCCL is the loopback test double (tests/mgpu_rank_job.py);
    the status and size all-gathers and the per-chunk Send/Recv into the root
    against the oracle, other roots, empty ranks, an encode error on any
    rank stopping every rank."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "tests", "cpp", "_build", "libloopback_rccl.so")
    assert os.path.exists(lib), "build tests/cpp first (make -C tests/cpp)"
    env = dict(os.environ, WSG_RCCL_LIB=lib)
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "mgpu_rank_job.py")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(d["cases"]) == 16
    for c in d["cases"]:
        assert not c["hung"], c
        if c["bad_rank"] is None:
            assert c["rc"] == [0] * c["world"] and c["wire_ok"] and c["off_ok"], c
        else:
            assert c["rc"] == [ca.WSG_ENOMEM] * c["world"], c   # every rank learns of the failure
    assert d["loopback_errors"] == 0   # every Send met its Recv, sizes agreed


@pytest.mark.gpu
def test_mgpu_rank_form_real_rccl_processes():
    """The RCCL rank form over the REAL RCCL, one process per rank, at world 2
    and 3 on the one GPU (tests/mgpu_rank_procs.py: a host id per rank, so
    RCCL connects the ranks through its socket transport instead of refusing
    two ranks on one device): ncclCommInitRank, the status / size
    all-gathers and the grouped per-chunk Send/Recv, process against
    process; the root's wire and offsets vs the oracle, an encode error on
    rank 1 reaching every rank."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "mgpu_rank_procs.py")], capture_output=True,
                       text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(d["cases"]) == 9
    for c in d["cases"]:
        assert not c["hung"], c
        rcs = [x.get("rc") for x in c["ranks"]]
        if c["bad_rank"] is None:
            assert rcs == [0] * c["world"], c
            top = c["ranks"][c["root"]]
            assert top["wire_ok"] and top["off_ok"], c
        else:
            assert rcs == [ca.WSG_ENOMEM] * c["world"], c


@pytest.mark.gpu
def test_mgpu_rank_form_copy_ordering():
    """Every host->device and device->device copy of the rank-form gather is
    ordered on the stream its consumer runs on (commit 0b854e9; the round-3
    flake: rc 0 on every rank, stale root offsets).  $WSG_TEST_NULL_SPIN_US
    makes the library park the device's null stream for 50 ms before each
    host->device round and before the transfers, so a plain hipMemcpy /
    hipMemset (null stream, not ordered with the contexts' non-blocking
    streams) lands after its consumer every time.  World 2 and 3 over the
    loopback double (ranks as threads), world 2 over the real RCCL (ranks as
    processes): the root's wire and offsets vs the oracle."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = os.path.join(root, "tests", "cpp", "_build", "libloopback_rccl.so")
    assert os.path.exists(lib), "build tests/cpp first (make -C tests/cpp)"
    env = dict(os.environ, WSG_TEST_NULL_SPIN_US="50000")
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "mgpu_rank_job.py")], capture_output=True,
                       text=True, timeout=200, env=dict(env, WSG_RCCL_LIB=lib, WSG_RANK_JOB="ordering"))
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(d["cases"]) == 2
    for c in d["cases"]:
        assert not c["hung"] and c["rc"] == [0] * c["world"] and c["wire_ok"] and c["off_ok"], c
    assert d["loopback_errors"] == 0
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "mgpu_rank_procs.py"), "--ordering"],
                       capture_output=True, text=True, timeout=200, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    (c,) = d["cases"]
    assert not c["hung"] and [x.get("rc") for x in c["ranks"]] == [0, 0], c
    assert c["ranks"][0]["wire_ok"] and c["ranks"][0]["off_ok"], c


@pytest.mark.gpu
def test_mgpu_c5_tool_world1():
    """tools/mgpu_c5.py (the C-ABI leg bench.py runs at N > 1) at world 1 on
    a reduced job: encode + gather through wsg_mgpu_create, root check."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "mgpu_c5.py"), "1", "8192"],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-500:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["root_check"] is True
    assert d["host_decode"].get("check") is True, d["host_decode"]


@pytest.mark.gpu
def test_bench_n2_c5_rank_form():
    """bench.py at N = 2 (torchrun, ranks sharing the one GPU over RCCL's
    socket transport, as the driver's N > 1 runs but on one card): its c5_job
    leg is the product's RCCL rank form (wsg_mgpu_create_rank +
    wsg_mgpu_encode_gather) on a reduced job, with a per-rank roofline, root
    ingress and the root's oracle check; the run exits 0 only if every leg's
    check holds."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, WSG_BENCH_SHARE_DEVICES="1", WSG_C5_FRAMES="16384", WSG_BENCH_CAPI_RCCL="0",
               WSG_BENCH_HOST_LEGS="0", NCCL_DEBUG="VERSION")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29533", os.path.join(root, "bench.py"),
                        "--gpus", "2", "--steps", "5", "--warmup", "2", "--no-extras"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-3000:])
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["spot_check"] is True and line["failed_checks"] == []
    c5 = line["c5_job"]
    assert c5["root_check"] is True, c5
    assert c5["path"].startswith("C-ABI rank form")
    assert c5["roofline_per_rank"]["kernel"] == "k_encode_mask" and c5["roofline_per_rank"]["frac"] > 0
    assert c5["bytes_into_root"] == 16384 // 2 * (16384 + 8)
    # one RCCL stack per rank: the bench's own group is gloo, so the only RCCL
    # initialised is the one the product library loads (torch's bundled RCCL,
    # another version, would print its own banner)
    import re

    versions = set(re.findall(r"RCCL version\s*:\s*(\S+)", r.stdout + r.stderr))
    assert len(versions) == 1, versions
