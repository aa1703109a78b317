#!/usr/bin/env python
"""Benchmark: WS payload mask/unmask GiB/s (device-resident), batched frames.

Default (N=1) workload = BASELINE.json configs[1] ("C2"): unmask-only decode
of 4096 masked binary frames x 64 KiB payload, one random key per frame,
inputs resident in HBM.  One step = one wsg_decode_batch call over the whole
batch = one k_decode launch (header unpack + unmask).

N>1 (`torch.distributed.run --nproc-per-node N bench.py --gpus N`): one
process per GPU; every rank decodes its own independent batch of the same
shape (frames shard with no data-path collective: weak scaling); the timed
region is bracketed by barrier + synchronize and the max over ranks is used.

The default N=1 run also measures the other BASELINE configs, each as a
bounded leg with its own object in the line ("c3", "c4", "c5": value,
ms_per_step, roofline of its dominant kernels -- C3 both halves of the round
trip --, CPU baseline, spot check): C3 mask+unmask round trip of 65536 ragged
frames, C4 fan-out of one 4 KiB payload to 10000 keys, C5 the whole 1 Mi x
16 KiB job on this GPU.  --config c3|c4|c5 makes one of them the headline.
"""
import argparse
import gc
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "WS payload mask/unmask GiB/s (device-resident), batched 64KiB frames"
HBM_PEAK_GBPS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
GIB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4", "c5"])
    ap.add_argument("--frames", type=int, default=None)
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--messages", type=int, default=1,
                    help="c4: messages per fan-out call (wsg_fanout_encode_many; ws_multicast's per-tick batch)")
    ap.add_argument("--no-c5-job", action="store_true", help="N>1: skip the C5 encode+gather leg")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip copy-ceiling and PCIe-inclusive legs")
    ap.add_argument("--no-configs", action="store_true", help="c2 at N=1: skip the C3/C4/C5 legs")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--dry-run", action="store_true",
                    help="the rank launch and the line's shape only (gloo, no GPU work): tests of --gpus N")
    return ap.parse_args()


XGMI_LINK_GBPS = 153.0   # one xGMI link, per direction (MI355X_MICROARCH.md)


def root_ingress_expectation(world):
    """GB/s the gather root can take in: one xGMI link from each other rank
    (the node's GPUs are fully connected, 7 links each)."""
    return round((world - 1) * XGMI_LINK_GBPS, 1) if world > 1 else None


def launch_ranks(args):
    """`python bench.py --gpus N` (N > 1) outside a torch.distributed launch:
    start one rank per GPU with torch.distributed.run as a child process (no
    torch or GPU call in this one), pass its output through and exit with its
    status.  Rank 0 prints the line."""
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "1"))
    r = subprocess.run(cmd, env=env)
    sys.exit(r.returncode)


def check_world(args):
    """The ranks actually running must be the --gpus asked for: a mismatch
    exits non-zero instead of reporting another N."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        if args.gpus > 1:
            launch_ranks(args)   # (does not return)
        return
    if int(env_world) != args.gpus:
        print("bench.py: WORLD_SIZE=%s but --gpus %d: launch one rank per GPU asked for" % (env_world, args.gpus),
              file=sys.stderr, flush=True)
        sys.exit(2)


def dry_run(args):
    """The launch path alone (gloo ranks, barrier, max over ranks): the line
    with the fields the N-rank run fills, no GPU work."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
    t0 = time.perf_counter()
    barrier(world)
    elapsed = time.perf_counter() - t0
    if world > 1:
        import torch
        import torch.distributed as dist

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": 0.0, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "dry_run": True, "barrier_s": round(elapsed, 6),
                          "root_ingress_expectation_GBps": root_ingress_expectation(world)}), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


def dist_setup(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # $WSG_BENCH_SHARE_DEVICES=1 rehearses the N-rank path on fewer GPUs
        # (ranks share devices round-robin); the real run is one GPU per rank
        share = os.environ.get("WSG_BENCH_SHARE_DEVICES") == "1"
        if share:
            local = local % torch.cuda.device_count()
        elif local >= torch.cuda.device_count():
            print("bench.py: --gpus %d needs a GPU per rank, %d visible (WSG_BENCH_SHARE_DEVICES=1 lets ranks "
                  "share them for a rehearsal)" % (world, torch.cuda.device_count()), file=sys.stderr, flush=True)
            sys.exit(2)
        if share:
            # RCCL over ranks sharing a GPU (a rehearsal on a smaller box): a host
            # id per rank makes RCCL see one GPU per host and connect the ranks
            # through its socket transport (it refuses two ranks of one host on
            # one device); the real run leaves this unset
            os.environ.setdefault("NCCL_HOSTID", "wsg-bench-rank-%d" % rank)
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            os.environ.setdefault("NCCL_IB_DISABLE", "1")
        # one node (the driver's launch): RCCL's bootstrap over loopback, as
        # the rendezvous itself (127.0.0.1); the data path between the GPUs is
        # RCCL's P2P over xGMI either way
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        torch.cuda.set_device(local)
        # The bench's own group is gloo: barriers, max over ranks and the
        # product's RCCL id travel over host sockets, so the only RCCL in a
        # rank is the one the product library loads (wsg_mgpu_create_rank) —
        # not torch's bundled RCCL beside it.  torch's RCCL is set up only for
        # the cross-check asked for with $WSG_BENCH_TORCH_GATHER=1 (rccl_group).
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
    return rank, world, local


_RCCL_GROUP = None


def rccl_group():
    """torch.distributed's own RCCL group, made on first use (every rank
    calls it): only the labelled torch-gather cross-check uses it."""
    global _RCCL_GROUP
    if _RCCL_GROUP is None:
        import torch.distributed as dist

        _RCCL_GROUP = dist.new_group(backend="nccl")
    return _RCCL_GROUP


def barrier(world, group=None):
    if world > 1:
        import torch.distributed as dist

        dist.barrier(group=group)


def max_over_ranks(x, world, device=None):
    """The max of a host scalar over the ranks (over the gloo group: no
    device collective)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def pmc_traffic(path, config):
    """HBM bytes per launch of the dominant kernel, from the committed PMC
    summary (profiles/pmc_traffic.json, produced by tools/pmc_summary.py)."""
    try:
        with open(path) as f:
            doc = json.load(f)
        return doc[config]["hbm_bytes_per_launch"]
    except Exception:
        return None


def host_cpu():
    """The host the CPU baseline runs on: model, CPUs visible, and the
    threads used (the affinity set, capped by a cgroup CPU quota and by
    $OMP_NUM_THREADS where the box sets one: a GPU box's CPU share is smaller
    than the machine nproc reports)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    nproc = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    threads = nproc if quota is None else min(nproc, quota)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        threads = min(threads, int(omp))
    return {"cpu_model": model, "nproc": nproc, "cgroup_cpus": quota, "threads": max(1, threads)}


class Workload:
    """Holds device inputs/outputs and runs one step."""

    def __init__(self, args, codec, rank, device):
        import torch

        import cppserver_amd as ca
        from cppserver_amd import workloads as wl

        self.cfg = args.config
        self.codec = codec
        self.torch = torch
        if self.cfg == "c2":
            n = args.frames or 4096
            size = args.size or 65536
            wire, fs, keys = wl.c2_wire(n, size, seed=1000 + rank)
            self.host = (wire, fs, keys)
            self.wire = torch.from_numpy(wire).to(device)
            self.fs = torch.from_numpy(fs.view(np.int64)).to(device)
            self.out = torch.empty_like(self.wire)
            # steps alternate between two distinct batches (2 x 537 MB touched),
            # so no step reads its input from the 256 MiB Infinity Cache that
            # the previous step left warm: every step is fresh HBM traffic
            wire2 = wl.c2_wire(n, size, seed=2000 + rank)[0]
            self.batches = [(self.wire, self.out), (torch.from_numpy(wire2).to(device), torch.empty_like(self.wire))]
            self.turn = 0
            self.info = torch.empty(n * ca.RECV_INFO.itemsize, dtype=torch.uint8, device=device)
            # one wsg_decode_batch per step through pre-bound C-ABI arguments
            # (what a C++ server's loop over its batch arena does), so the
            # Python argument marshalling stays out of the short timed region
            self.launch = [codec.prepare_decode(wi, self.fs, o, self.info) for wi, o in self.batches]
            self.payload_bytes = n * size
            # k_decode: read wire + write out, plus per frame its start (8 B)
            # and wsg_recv_info (32 B)
            self.alg_bytes = 2 * len(wire) + n * 40
            self.kernel = "k_decode"
            self.workload = "C2 unmask-only: %d masked binary frames x %d B payload, one key per frame" % (n, size)
            self.extra = {"frames": n, "payload_bytes_per_frame": size, "wire_bytes": len(wire)}
        elif self.cfg == "c3":
            n = args.frames or 65536
            payload, desc = wl.c3_batch(n, 128, args.size or 65536, seed=3000 + rank)
            self.host = (payload, desc)
            self.payload = torch.from_numpy(payload).to(device)
            self.desc = ca.desc_to_tensor(desc, device)
            cap = int(sum(ca.frame_size(0x82, True, int(x)) for x in desc["len"]))
            self.wire = torch.empty(cap, dtype=torch.uint8, device=device)
            self.woff = torch.empty(n + 1, dtype=torch.int64, device=device)
            self.out = torch.empty_like(self.wire)
            self.info = torch.empty(n * ca.RECV_INFO.itemsize, dtype=torch.uint8, device=device)
            self.cap = cap
            self.payload_bytes = int(desc["len"].sum())
            self.alg_bytes = len(payload) + cap        # encode mask kernel: read payload + write wire
            self.kernel = "k_encode_mask"
            # the round trip's second half, k_decode: read wire + write out,
            # plus per frame its start (8 B) and wsg_recv_info (32 B); timed on
            # a context of its own so each half has its own HIP events
            self.dec_alg_bytes = 2 * cap + n * 40
            self.dec_codec = ca.Codec(device.index if device.index is not None else 0)
            self.workload = "C3 mask+unmask round trip: %d frames, payload uniform in [128, 65536] B" % n
            self.extra = {"frames": n, "wire_bytes": cap}
        elif self.cfg == "c4":
            k = args.frames or 10000
            length = args.size or 4096
            m = max(1, args.messages)
            # m messages of `length` bytes (one random arena) x k client keys
            rng = np.random.default_rng(4000 + rank)
            payload = wl.random_bytes(rng, m * length + 16)
            keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
            self.host = (payload, keys)
            self.m, self.length = m, length
            self.src_off = np.arange(m, dtype=np.uint64) * np.uint64(length)
            self.lens = np.full(m, length, dtype=np.uint64)
            self.ops = np.full(m, 0x82, dtype=np.uint8)
            self.payload = torch.from_numpy(payload).to(device)
            self.keys = torch.from_numpy(keys.view(np.int32)).to(device)
            fsz = ca.frame_size(0x82, True, length)
            per_msg = (fsz * k + 127) // 128 * 128
            self.wire = torch.empty(per_msg * m, dtype=torch.uint8, device=device)
            self.payload_bytes = m * length * k
            self.alg_bytes = m * (fsz * k + length + 4 * k)
            # frame sizes that are a multiple of 4 take the period kernel (wsg_kernels.hip launch_fanout_period)
            self.kernel = "k_fanout_period" if fsz % 4 == 0 else "k_fanout_flat"
            self.workload = ("C4 fan-out: one %d B payload masked with %d client keys" % (length, k) if m == 1 else
                             "C4 x %d messages: %d B payloads x %d client keys in one wsg_fanout_encode_many call"
                             % (m, length, k))
            self.extra = {"keys": k, "messages": m, "wire_bytes": fsz * k * m}
            # one fan-out per step through pre-bound C-ABI arguments (a
            # server's multicast loop): a launch is shorter than Python's
            # argument marshalling
            self.launch = codec.prepare_fanout(self.payload, self.keys, 0x82, True, self.wire, length=length) \
                if m == 1 else None
        else:  # c5: this rank's round-robin shard of 1 Mi x 16 KiB frames, encode
            world = int(os.environ.get("WORLD_SIZE", "1"))
            size = args.size or 16384
            n_total = args.frames or (1 << 20)
            from cppserver_amd import shard

            ids = shard.rank_frames(rank, world, n_total)
            # payloads are a function of the global frame index, made in HBM
            # (16 GiB at one GPU); the host regenerates any frame to check it
            self.payload = wl.c5_payload_torch(ids, size, device=device)
            desc = wl.c5_desc(ids, size)
            self.desc = ca.desc_to_tensor(desc, device)
            self.host = (ids, desc, size)
            n = len(desc)
            cap = n * ca.frame_size(0x82, True, size)
            self.wire = torch.empty(cap, dtype=torch.uint8, device=device)
            self.woff = torch.empty(n + 1, dtype=torch.int64, device=device)
            self.cap = cap
            self.payload_bytes = n * size
            self.alg_bytes = n * size + cap
            self.kernel = "k_encode_mask"
            self.workload = "C5 encode shard: %d x %d B frames of a %d-frame job (round-robin)" % (n, size, n_total)
            self.extra = {"frames_this_rank": n, "wire_bytes": cap}

    def close(self):
        """Free the device buffers (and C3's decode context) before the next leg."""
        if getattr(self, "dec_codec", None) is not None:
            self.dec_codec.close()
            self.dec_codec = None
        for name in ("wire", "fs", "out", "batches", "launch", "info", "payload", "desc", "woff", "keys"):
            if hasattr(self, name):
                setattr(self, name, None)

    def step(self):
        c = self.codec
        if self.cfg == "c2":
            self.launch[self.turn]()
            self.turn ^= 1
        elif self.cfg == "c3":
            c.encode_batch(self.payload, self.desc, wire=self.wire, wire_cap=self.cap, wire_off=self.woff)
            self.dec_codec.decode_batch(self.wire, self.woff[:-1], out=self.out, info=self.info)
        elif self.cfg == "c4":
            if self.m == 1:
                self.launch()
            else:
                c.fanout_many(self.payload, self.src_off, self.lens, self.ops, self.keys, wire=self.wire)
        else:
            c.encode_batch(self.payload, self.desc, wire=self.wire, wire_cap=self.cap, wire_off=self.woff)

    def spot_check(self):
        """One step's output at sampled frames against the oracle (the CPU
        restatement of ws.cpp), before the warm-up: c2 the unmasked payload
        and header bytes, c3 encode bytes and the decoded payload, c4 sampled
        fan-out frames, c5 sampled frames of the shard (payload regenerated
        on the host from the frame index)."""
        import oracle

        import cppserver_amd as ca

        self.step()
        self.codec.sync()
        if self.cfg == "c2":
            _, fs, _ = self.host
            win, out = self.batches[self.turn ^ 1]   # the batch the step above decoded
            n = len(fs)
            fsz = int(win.numel()) // n
            ok = True
            for i in (0, n // 2, n - 1):
                s = int(fs[i])
                rc, ref, _ = oracle.decode_batch(win[s: s + fsz].cpu().numpy(), np.zeros(1, np.uint64))
                ok &= rc == 0 and bool(np.array_equal(out[s: s + fsz].cpu().numpy(), ref))
            return bool(ok)
        if self.cfg == "c3":
            payload, desc = self.host
            n = len(desc)
            offs = self.woff.cpu().numpy()
            ok = True
            for i in (0, 1, n // 2, n - 1):
                d = desc[i: i + 1].copy()
                ref, _ = oracle.encode_batch(payload, d)
                a, b = int(offs[i]), int(offs[i + 1])
                got = self.wire[a: b].cpu().numpy()
                dec = self.out[a: b].cpu().numpy()
                p = payload[int(d["src_off"][0]): int(d["src_off"][0]) + int(d["len"][0])]
                ok &= bool(np.array_equal(got, ref)) and bool(np.array_equal(dec[len(dec) - len(p):], p))
            return bool(ok)
        if self.cfg == "c4":
            payload, keys = self.host
            fsz = ca.frame_size(0x82, True, self.length)
            k = len(keys)
            per_msg = (fsz * k + 127) // 128 * 128 if self.m > 1 else fsz * k
            ok = True
            for mi in sorted({0, self.m - 1}):
                msg = payload[mi * self.length: (mi + 1) * self.length]
                for j in (0, 1, k // 2, k - 1):
                    ref = oracle.fanout_encode(msg, keys[j: j + 1], 0x82, True)
                    a = mi * per_msg + j * fsz
                    ok &= bool(np.array_equal(self.wire[a: a + fsz].cpu().numpy(), ref))
            return bool(ok)
        ids, desc, size = self.host
        n = len(ids)
        fsz = ca.frame_size(0x82, True, size)
        ok = int(self.woff[-1].item()) == n * fsz
        for q in (0, 1, n // 2, n - 1):
            d = desc[q: q + 1].copy()
            d["src_off"] = 0
            ref, _ = oracle.encode_batch(wl_c5_payload(ids[q: q + 1], size), d)
            ok &= bool(np.array_equal(self.wire[q * fsz: (q + 1) * fsz].cpu().numpy(), ref))
        return bool(ok)


def wl_c5_payload(ids, size):
    from cppserver_amd import workloads as wl

    return wl.c5_payload_np(ids, size)


def cpu_baseline(w, seconds, cpu):
    """The oracle's faithful byte-loop restatement of the reference codec
    (ws.cpp:212-271 encode, :273-456 decode), timed on this host on a bounded
    sample of the same workload: one thread, then `cpu["threads"]` threads
    (one independent session per thread over a contiguous frame slice).
    Returns (one, many) baseline dicts in the unit of the line's metric."""
    import oracle

    threads = cpu["threads"]

    def pack(rate_1, rate_n, sample):
        base = {"unit": "GiB/s", "kind": "port", "sample": sample, "cpu_model": cpu["cpu_model"],
                "host_nproc": cpu["nproc"]}
        return (dict(base, value=rate_1, cores=1),
                dict(base, value=rate_n, cores=threads, sample=sample + "; one session per thread"))

    if w.cfg == "c2":
        wire, fs, _ = w.host
        n = len(fs)
        per_frame = w.payload_bytes // n
        t_probe = oracle.time_decode(wire, fs[: max(1, n // 16)], threads=1, iters=1)
        rate = (n // 16) * per_frame / max(t_probe, 1e-9)
        iters = max(3, int((seconds / 2) * rate / (n * per_frame)))
        t1 = oracle.time_decode(wire, fs, threads=1, iters=iters)
        tn = oracle.time_decode(wire, fs, threads=threads, iters=max(3, iters * threads // 2))
        sample = "%d frames x %d B (%.0f MiB), PrepareReceiveFrame per whole frame, median of %d passes" % (
            n, per_frame, n * per_frame / 2**20, iters)
        return pack(n * per_frame / t1 / GIB, n * per_frame / tn / GIB, sample)

    def enc_sample(payload, desc, budget):
        """First frames of the batch worth ~budget s of one-thread encode."""
        probe = desc[: max(1, min(len(desc), 256))]
        t = oracle.time_encode(payload, probe, threads=1, iters=1)
        per = float(probe["len"].sum()) / max(t, 1e-9)
        m, acc = 0, 0
        cap = budget * per
        while m < len(desc) and acc < cap:
            acc += int(desc["len"][m])
            m += 1
        return desc[: max(1, m)]

    if w.cfg == "c3":
        payload, desc = w.host
        sub = enc_sample(payload, desc, seconds / 4)
        wire, off = oracle.encode_batch(payload, sub)
        nb = float(sub["len"].sum())
        e1 = oracle.time_encode(payload, sub, threads=1, iters=3)
        d1 = oracle.time_decode(wire, off[:-1], threads=1, iters=3)
        en = oracle.time_encode(payload, sub, threads=threads, iters=3)
        dn = oracle.time_decode(wire, off[:-1], threads=threads, iters=3)
        sample = ("first %d of the %d C3 frames (%.0f MiB payload), PrepareSendFrame then PrepareReceiveFrame per "
                  "frame; rate = payload / (encode + decode time)" % (len(sub), len(desc), nb / 2**20))
        return pack(nb / (e1 + d1) / GIB, nb / (en + dn) / GIB, sample)
    if w.cfg == "c4":
        payload, keys = w.host
        k = len(keys)
        desc = np.zeros(k, dtype=oracle_desc_dtype())
        desc["len"] = w.length
        desc["key"] = keys
        desc["opcode"] = 0x82
        desc["mask"] = 1
        t1 = oracle.time_encode(payload, desc, threads=1, iters=5)
        tn = oracle.time_encode(payload, desc, threads=threads, iters=5)
        nb = float(k * w.length)
        sample = ("one message: %d x PrepareSendFrame(0x82, mask, %d B) with the key set per call (the client "
                  "path, SURVEY §3.3)" % (k, w.length))
        return pack(nb / t1 / GIB, nb / tn / GIB, sample)
    ids, desc, size = w.host
    sub_n = max(1, min(len(ids), int(seconds / 4 * 0.5 * GIB / size)))
    sub = desc[:sub_n].copy()
    payload = wl_c5_payload(ids[:sub_n], size)
    t1 = oracle.time_encode(payload, sub, threads=1, iters=3)
    tn = oracle.time_encode(payload, sub, threads=threads, iters=3)
    nb = float(sub_n * size)
    sample = "first %d of the shard's %d C5 frames (%.0f MiB), PrepareSendFrame per frame" % (
        sub_n, len(ids), nb / 2**20)
    return pack(nb / t1 / GIB, nb / tn / GIB, sample)


def oracle_desc_dtype():
    from cppserver_amd.layout import SEND_DESC

    return SEND_DESC


def torch_copy_rate(w, reps=10):
    """torch's device-to-device copy_ of the same byte count (read + write
    GB/s): the runtime's own copy, for scale only.  It is not the ceiling —
    k_decode beats it; the bare-copy ceiling of a 16-B-per-lane kernel is
    tools/membench.hip's."""
    t = w.torch
    src = w.wire
    dst = t.empty_like(src)
    for _ in range(2):
        dst.copy_(src)
    e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dst.copy_(src)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return 2 * src.numel() / (ms * 1e-3) / 1e9


def pcie_inclusive(w, reps=3):
    """Host wire -> H2D -> decode -> D2H rate (payload GiB/s), C2 only, through
    wsg_decode_batch_host's segmented 3-slot pipeline.  "pinned": host buffers
    in page-locked memory (a server's receive buffers); "pageable": plain
    numpy buffers, staged through pinned memory by the library."""
    if w.cfg != "c2":
        return None
    import cppserver_amd as ca

    wire, fs, _ = w.host
    res = {}
    pin_in = ca.pinned_empty(len(wire))
    pin_in[:] = wire
    pin_out = ca.pinned_empty(len(wire))
    for name, src, dst in (("pinned", pin_in, pin_out), ("pageable", wire, np.empty_like(wire))):
        rc, _, _ = w.codec.decode_batch_host(src, fs, out=dst)
        assert rc == 0
        t0 = time.perf_counter()
        for _ in range(reps):
            w.codec.decode_batch_host(src, fs, out=dst)
        res[name] = round(w.payload_bytes / ((time.perf_counter() - t0) / reps) / GIB, 2)
    # the send direction: the same 4096 x 64 KiB payloads encoded from host
    # memory (wsg_encode_batch_host), pinned buffers
    from cppserver_amd import workloads as wl

    rng = np.random.default_rng(7)
    desc, total = wl.ragged_desc(rng, np.full(len(fs), w.payload_bytes // len(fs)))
    pay = ca.pinned_empty(total)
    pay[:] = wl.random_bytes(rng, total)
    out = ca.pinned_empty(int(ca.frame_sizes(desc).sum()))
    rc, _, _ = w.codec.encode_batch_host(pay, desc, wire=out)
    assert rc == 0
    t0 = time.perf_counter()
    for _ in range(reps):
        w.codec.encode_batch_host(pay, desc, wire=out)
    res["encode_pinned"] = round(total / ((time.perf_counter() - t0) / reps) / GIB, 2)
    return res


def gpu_node_cpus(device_index=0):
    """The NUMA node the GPU hangs off (its PCI function's numa_node in sysfs)
    and that node's CPUs this process may use: (node, cpus) or (None, None).
    The host-side legs run there, as a deployment binds its IO threads to the
    GPU's node (numactl --cpunodebind): on the dual-socket GPU box a thread on
    the other socket crosses the socket link for every mailbox poll (the
    per-call echo 161 K vs 176 K msg/s, profiles/r5/numa_per_call_r5aa.log)."""
    try:
        import torch

        p = torch.cuda.get_device_properties(device_index)
        dev = "/sys/bus/pci/devices/%04x:%02x:%02x.0" % (p.pci_domain_id, p.pci_bus_id, p.pci_device_id)
        with open(os.path.join(dev, "numa_node")) as f:
            node = int(f.read().strip())
        if node < 0:
            return None, None
        with open("/sys/devices/system/node/node%d/cpulist" % node) as f:
            spec = f.read().strip()
        cpus = set()
        for part in spec.split(","):
            if "-" in part:
                a, b = part.split("-")
                cpus.update(range(int(a), int(b) + 1))
            elif part:
                cpus.add(int(part))
        cpus &= os.sched_getaffinity(0)
        return (node, cpus) if cpus else (None, None)
    except Exception:   # noqa: BLE001  (no sysfs entry: the legs run unbound)
        return None, None


def _run_leg(cmd, timeout, env=None):
    """A host-side leg's child process; a time-out is reported in the line
    (returncode 124) rather than ending the bench.  env: variables added to
    this process's environment for the child."""
    import subprocess

    try:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                              env=dict(os.environ, **env) if env else None)
    except subprocess.TimeoutExpired:
        return subprocess.CompletedProcess(cmd, 124, "", "no result within %d s" % timeout)


def session_batch_leg(timeout=240):
    """The batched session paths end to end on host
    buffers: C2's 4096 x 64 KiB frames spread over 1024 sessions, framed on
    the host (16 KiB reads), unmasked in one pipelined GPU pass, delivered
    through each session's callbacks; and the same frames queued for send and
    encoded in one pass.  Beside it, the per-call GPU path (one
    PrepareReceiveFrame / PrepareSendFrame per frame).  Runs
    tools/_build/bench_batch (product library only) as a child process."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "_build", "bench_batch")
    if not os.path.exists(exe):
        return None
    out = {}
    legs = (("rx", ["1024", "4", "65536", "16384", "3"]), ("tx", ["1024", "4", "65536", "0", "3"]),
            # echo-sized messages (32 B payload): 256 sessions x 64 frames
            ("rx_32B", ["256", "64", "32", "0", "3"]), ("tx_32B", ["256", "64", "32", "0", "3"]))
    for leg, args in legs:
        mode = leg.split("_")[0]
        r = _run_leg([exe, mode] + args, timeout)
        if r.returncode != 0:
            out[leg] = {"error": (r.stderr or r.stdout).strip()[-300:]}
            continue
        d = json.loads(r.stdout.strip().splitlines()[-1])
        out[leg] = {k: d[k] for k in ("batched_GiBps", "per_call_GiBps", "batched_frames_per_s",
                                       "per_call_frames_per_s", "delivered_ok")}
    out["workload"] = ("rx/tx: 1024 sessions x 4 frames x 64 KiB; *_32B: 256 sessions x 64 frames x 32 B; "
                       "host buffers (PCIe + host framing + callbacks inside)")
    return out


def echo_c1_leg(seconds=3.0, timeout=120):
    """BASELINE config C1 (ws_echo_client / ws_echo_server: 32-byte messages,
    1000 in flight per client) through the drop-in WSClient / WSSession API
    over in-memory transports (tools/_build/bench_echo, product library only;
    no sockets: the transport is out of scope).  per_read = the API's default
    (each read one batch scope), tick = one scope per event-loop pass,
    per_call = automatic batching off (one GPU round trip per masked frame);
    wss_* = the same through WSSClient / WSSSession over TLS 1.3 (wss_echo).
    Metric as ws_echo_client.cpp:191-201 (messages = echoed bytes / size)."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "_build", "bench_echo")
    if not os.path.exists(exe):
        return None
    out = {}
    legs = (("per_read_1c", ["per_read", "1", "1", "1000", "32"]),
            ("per_read_100c_4t", ["per_read", "100", "4", "1000", "32"]),
            ("tick_100c_1t", ["tick", "100", "1", "1000", "32"]),
            ("per_call_1c", ["per_call", "1", "1", "1000", "32"]),
            # wss_echo (performance/wss_echo_client.cpp): the same loop through
            # WSSClient / WSSSession over TLS 1.3 (OpenSSL record encryption)
            ("wss_per_read_1c", ["per_read", "1", "1", "1000", "32"]),
            ("wss_per_read_100c_4t", ["per_read", "100", "4", "1000", "32"]),
            ("wss_tick_100c_1t", ["tick", "100", "1", "1000", "32"]))
    for leg, args in legs:
        extra = ["tls"] if leg.startswith("wss_") else []
        r = _run_leg([exe] + args + [str(seconds)] + extra, timeout)
        if r.returncode != 0:
            out[leg] = {"error": (r.stderr or r.stdout).strip()[-300:]}
            continue
        d = json.loads(r.stdout.strip().splitlines()[-1])
        out[leg] = {k: d[k] for k in ("msg_per_s", "MiB_per_s", "latency_ns", "total_messages", "payload_ok")}
    # the same loop with the client's key 0 (tools/_build/echo_hostonly): no
    # frame has a key, so no GPU pass runs; the API's host work alone (framing,
    # delivery, queueing, hand-outs), i.e. what a per_read round costs besides
    # its two GPU passes
    ho = os.path.join(ROOT, "tools", "_build", "echo_hostonly")
    if os.path.exists(ho):
        r = _run_leg([ho, "per_read", "1", "1", "1000", "32", str(seconds)], timeout)
        if r.returncode == 0:
            d = json.loads(r.stdout.strip().splitlines()[-1])
            out["host_only_1c"] = {k: d[k] for k in ("msg_per_s", "latency_ns", "payload_ok")}
            out["host_only_1c"]["what"] = ("per_read_1c with client key 0: no GPU pass, the API's host work alone "
                                           "(not a product mode: client keys are rand(), ws.cpp:97)")
        else:
            out["host_only_1c"] = {"error": (r.stderr or r.stdout).strip()[-300:]}
    # the reference's algorithm in the SAME loop: the oracle's restatement of
    # PrepareSendFrame / PrepareReceiveFrame (CPU, no GPU) driving the same
    # in-memory echo (tools/_build/bench_echo_ref; the cpu_baseline side)
    ref = os.path.join(ROOT, "tools", "_build", "bench_echo_ref")
    if os.path.exists(ref):
        cr = {}
        for leg, a in (("1c_1t", ["1", "1", "1000", "32"]), ("100c_4t", ["100", "4", "1000", "32"])):
            r = _run_leg([ref] + a + [str(seconds)], timeout)
            if r.returncode != 0:
                cr[leg] = {"error": (r.stderr or r.stdout).strip()[-300:]}
                continue
            d = json.loads(r.stdout.strip().splitlines()[-1])
            cr[leg] = {k: d[k] for k in ("msg_per_s", "MiB_per_s", "latency_ns", "total_messages", "payload_ok")}
        cr["what"] = ("reference codec algorithm (oracle restatement of ws.cpp:212-456, CPU) in this same in-memory "
                      "echo loop; compare with per_read_1c / per_read_100c_4t")
        out["cpu_reference"] = cr
    # over real loopback TCP, the reference's own method (its drivers on
    # 127.0.0.1): the drop-in classes and the reference algorithm on the CPU,
    # same epoll loop (tools/_build/bench_echo_tcp; measurement-only sockets)
    tcp = os.path.join(ROOT, "tools", "_build", "bench_echo_tcp")
    if os.path.exists(tcp):
        tr = {}
        # gpu_100c_4t_hwq8: the same with GPU_MAX_HW_QUEUES=8 (round 4's
        # per-context lanes needed a hardware queue per IO thread; the one
        # lane per device of round 5 does not: the two should match)
        for leg, a, env in (("gpu_1c_1t", ["gpu", "1", "1"], None), ("gpu_100c_4t", ["gpu", "100", "4"], None),
                            ("gpu_100c_4t_hwq8", ["gpu", "100", "4"], {"GPU_MAX_HW_QUEUES": "8"}),
                            ("gpu_tick_100c_4t", ["gpu_tick", "100", "4"], None),
                            ("cpu_ref_1c_1t", ["cpu_ref", "1", "1"], None),
                            ("cpu_ref_100c_4t", ["cpu_ref", "100", "4"], None)):
            # the 100-client legs share the host's loopback stack with whatever
            # else runs on the machine: three runs each, the median reported
            # (the gpu and cpu_ref legs alike), every run's rate listed
            runs = []
            for _ in range(3 if a[1] == "100" and env is None else 1):
                r = _run_leg([tcp] + a + ["1000", "32", str(seconds)], timeout, env)
                if r.returncode != 0:
                    runs = [{"error": (r.stderr or r.stdout).strip()[-300:]}]
                    break
                runs.append(json.loads(r.stdout.strip().splitlines()[-1]))
            if "error" in runs[0]:
                tr[leg] = runs[0]
                continue
            d = sorted(runs, key=lambda x: x["msg_per_s"])[len(runs) // 2]
            tr[leg] = {k: d[k] for k in ("msg_per_s", "MiB_per_s", "latency_ns", "total_messages", "payload_ok")}
            tr[leg]["payload_ok"] = all(x["payload_ok"] for x in runs)
            if len(runs) > 1:
                tr[leg]["runs_msg_per_s"] = [x["msg_per_s"] for x in runs]
            if a[0] != "cpu_ref":   # socket reads, lane requests and launches of the reported run
                tr[leg]["lane"] = {k: d.get(k) for k in ("reads", "lane_requests", "lane_launches", "lane_state",
                                                           "lane_give_ups")}
        tr["what"] = ("ws_echo over TCP 127.0.0.1 (one process, server and client on their own epoll threads): "
                      "gpu = the drop-in WSClient/WSSession, cpu_ref = the oracle's restatement of the reference "
                      "codec (no GPU); 100-client legs: median of 3 runs (runs_msg_per_s); the published figures below are "
                      "this method on an i7-4790K")
        out["tcp_loopback"] = tr
    out["reference_published"] = {"msg_per_s_1c_1t": 160448, "msg_per_s_100c_4t": 594328,
                                  "wss_msg_per_s_1c_1t": 203343, "wss_msg_per_s_100c_4t": 818230,
                                  "hardware": "loopback sockets, i7-4790K (README.md:3312-3352, 3356-3396): "
                                              "not like-for-like with this in-memory loop"}
    out["transport"] = "in-memory pipes, no socket syscalls (sockets are out of scope)"
    return out


def multicast_leg(seconds=2.0, timeout=120):
    """ws_multicast (performance/ws_multicast_server.cpp:104-124: RATE
    MulticastBinary calls of 32 zero bytes per tick to every client;
    ws_multicast_client.cpp:48-51 counts received bytes) through the drop-in
    WSServer / WSClient over in-memory transports (tools/_build/
    bench_multicast).  Server frames have key 0, so the XOR is the identity
    (no GPU pass): this measures the API's framing and fan-out copies.
    per_call = each call on its own, tick = one BatchScope per tick."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "_build", "bench_multicast")
    if not os.path.exists(exe):
        return None
    out = {}
    for leg, args in (("per_call_1c", ["per_call", "1", "1000", "32"]),
                      ("tick_1c", ["tick", "1", "1000", "32"]),
                      ("per_call_100c", ["per_call", "100", "1000", "32"]),
                      ("tick_100c", ["tick", "100", "1000", "32"])):
        r = _run_leg([exe] + args + [str(seconds)], timeout)
        if r.returncode != 0:
            out[leg] = {"error": (r.stderr or r.stdout).strip()[-300:]}
            continue
        d = json.loads(r.stdout.strip().splitlines()[-1])
        out[leg] = {k: d[k] for k in ("msg_per_s", "MiB_per_s", "total_messages", "all_delivered")}
    out["reference_published"] = {"msg_per_s_1c_1t": 3148135, "msg_per_s_100c_4t": 3225965,
                                  "hardware": "loopback sockets, i7-4790K (README.md:3542-3580): not like-for-like "
                                              "with this in-memory loop"}
    out["gpu_work"] = ("none: server frames carry key 0 (ws.cpp:206), the XOR is the identity; this measures the "
                       "API's framing and fan-out copies (the keyed GPU fan-out is C4)")
    return out


def echo_size_leg(w, n=1 << 20, size=32, reps=20):
    """Echo-sized frames on the device batch paths (SURVEY C1's 32 B messages,
    38 B masked client frames): one batch of 1 Mi frames encoded
    (wsg_encode_batch: sizes scan + k_encode_small) and the resulting wire
    decoded (wsg_decode_batch: k_decode, staged tiles), each call timed back to
    back, inputs in HBM.  A context, not the headline."""
    import time

    import cppserver_amd as ca
    from cppserver_amd import workloads as wl

    t = w.torch
    c = w.codec
    payload, desc = wl.c3_batch(n, size, size, seed=77)
    dev = w.wire.device
    p = t.from_numpy(payload).to(dev)
    d = ca.desc_to_tensor(desc, dev)
    cap = n * ca.frame_size(0x82, True, size)
    wire = t.empty(cap, dtype=t.uint8, device=dev)
    woff = t.empty(n + 1, dtype=t.int64, device=dev)
    out = t.empty_like(wire)
    info = t.empty(n * ca.RECV_INFO.itemsize, dtype=t.uint8, device=dev)

    def timed(fn):
        for _ in range(3):
            fn()
        c.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        c.sync()
        return (time.perf_counter() - t0) / reps

    te = timed(lambda: c.encode_batch(p, d, wire=wire, wire_cap=cap, wire_off=woff))
    ok = int(woff[-1].item()) == cap
    td = timed(lambda: c.decode_batch(wire, woff[:-1], out=out, info=info))
    i = n // 2
    s0 = int(woff[i].item())
    ok = ok and t.equal(out[s0 + 6: s0 + 38].cpu(), p[i * size: (i + 1) * size].cpu())
    return {"workload": "%d frames x %d B payload, masked (echo size), device-resident" % (n, size),
            "encode_us": round(te * 1e6, 1), "decode_us": round(td * 1e6, 1),
            "encode_Gframes_per_s": round(n / te / 1e9, 2), "decode_Gframes_per_s": round(n / td / 1e9, 2),
            "roundtrip_ok": bool(ok)}


def fanout_graph_leg(w, per_graph=20, replays=10):
    """C4 is launch-latency sensitive: the same fan-out captured
    `per_graph` times in one HIP graph (torch.cuda.CUDAGraph over the
    library's launches on the capturing stream) and replayed; reports the
    fan-out time per call inside the graph next to the eager step."""
    t = w.torch
    c = w.codec
    wires = [w.wire, t.empty_like(w.wire)]
    for i in range(3):   # nothing is allocated inside a fan-out call; warm anyway
        c.fanout(w.payload, w.keys, 0x82, True, wire=wires[i & 1], length=w.length)
    t.cuda.synchronize()
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g):
        for i in range(per_graph):
            c.fanout(w.payload, w.keys, 0x82, True, wire=wires[i & 1], length=w.length)
    g.replay()
    t.cuda.synchronize()
    e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(replays):
        g.replay()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / (replays * per_graph)
    return {"fanouts_per_graph": per_graph, "us_per_fanout": round(us, 2),
            "GiBps": round(w.payload_bytes / (us * 1e-6) / GIB, 1)}


def _gather_tensors(wire, woff, group):
    """Device tensors for an RCCL group; host copies for the bench's own
    gloo group."""
    if group is None:
        n = int(woff[-1].item())
        return wire[:n].cpu(), woff.cpu()
    return wire, woff


def gather_root_check(parts, n_total, size, chunk=1024):
    """Root side of the C5 gather: reassemble the job in global frame order
    and check sampled frames against the oracle (payload regenerated from
    the frame index).  Returns (ok, job wire bytes)."""
    import oracle
    from cppserver_amd import shard
    from cppserver_amd import workloads as wl

    import cppserver_amd as ca

    job, job_off = shard.reassemble(parts, n_total, chunk)
    fsz = ca.frame_size(0x82, True, size)
    ok = int(job_off[-1].item()) == n_total * fsz
    for g in sorted({0, 1, chunk, n_total // 2 + 3, n_total - 1}):
        ids = np.array([g])
        ref, _ = oracle.encode_batch(wl.c5_payload_np(ids, size), wl.c5_desc(ids, size))
        ok &= bool(np.array_equal(job[g * fsz: (g + 1) * fsz].cpu().numpy(), ref))
    return bool(ok), int(job_off[-1].item())


def c5_rank_leg(world, rank, local, device, n_total=1 << 20, size=16384, chunk=1024, reps=3):
    """BASELINE config C5 beside the weak-scaling headline at N > 1, through
    the product's own multi-GPU entry in its one-process-per-GPU form (SURVEY
    §8b-3 / §8e): every torchrun rank joins a wsg_mgpu group
    (wsg_mgpu_create_rank; rank 0's wsg_mgpu_unique_id handed out over the
    host group) and calls wsg_mgpu_encode_gather on its round-robin shard of
    the 1 Mi x 16 KiB job (1024-frame chunks, payloads made in HBM): its GPU
    encodes the shard, then the library's grouped ncclSend / ncclRecv move
    every chunk straight to its place in rank 0's output (RCCL over xGMI),
    and k_rebase_offsets writes the job's frame offsets there.

    Per rank: the encode (HIP events on the group context's stream around
    wsg_encode_batch, and around k_encode_mask alone for the roofline) and
    the gather (events on the stream the transfers run on), each the max
    over ranks; root ingress GB/s beside SURVEY §8e's ~1.07 TB/s (7 xGMI
    links); the root's output against the oracle (sampled frames) and its
    offsets against the closed form."""
    import torch
    import torch.distributed as dist

    import cppserver_amd as ca
    from cppserver_amd import shard
    from cppserver_amd import workloads as wl

    group = None   # (the bench's gloo group: the id travels over host sockets)
    obj = [ca.MultiGPU.unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    g = ca.MultiGPU.rank(local, obj[0], rank, world)
    try:
        ids = shard.rank_frames(rank, world, n_total, chunk)
        payload = wl.c5_payload_torch(ids, size, device=device)
        desc = ca.desc_to_tensor(wl.c5_desc(ids, size), device)
        fsz = ca.frame_size(0x82, True, size)
        n_local = len(ids)
        wire = torch.empty(max(n_local * fsz, 16), dtype=torch.uint8, device=device)
        woff = torch.empty(n_local + 1, dtype=torch.int64, device=device)
        out = out_off = None
        if rank == 0:
            out = torch.empty(n_total * fsz, dtype=torch.uint8, device=device)
            out_off = torch.empty(n_total + 1, dtype=torch.int64, device=device)
        torch.cuda.synchronize()

        def call():
            return g.encode_gather(n_total, chunk, [payload], [desc], [wire], [woff], root=0, out=out,
                                   out_off=out_off)

        call()   # warm: RCCL connections, the library's scratch
        g.timing(True, every=1)
        g.timing_read(reset=True)
        enc, gat, wall = [], [], []
        for _ in range(reps):
            dist.barrier(group=group)
            t0 = time.perf_counter()
            e_ms, g_ms = call()
            wall.append((time.perf_counter() - t0) * 1e3)
            enc.append(e_ms)
            gat.append(g_ms)
        k_ms, k_n = g.timing_read(reset=True)
        g.timing(False)
        k_avg = k_ms / max(k_n, 1)
        enc_ms = max_over_ranks(min(enc), world, device)
        gat_ms = max_over_ranks(min(gat), world, device)
        wall_ms = max_over_ranks(min(wall), world, device)
        k_max = max_over_ranks(k_avg, world, device)
        k_min = -max_over_ranks(-k_avg, world, device)
        alg = n_local * (size + fsz)   # k_encode_mask: read payload + write frames (this rank)
        res = {"workload": "C5: %d x %d B frames round-robin (chunks of %d) over %d GPUs, gather to rank 0"
                           % (n_total, size, chunk, world),
               "path": "C-ABI rank form: wsg_mgpu_create_rank + wsg_mgpu_encode_gather (RCCL grouped send/recv)",
               "calls": reps, "encode_ms": round(enc_ms, 4),
               "encode_GiBps_job": round(n_total * size / (enc_ms * 1e-3) / GIB, 1),
               "gather_ms": round(gat_ms, 3), "wall_ms": round(wall_ms, 3),
               "roofline_per_rank": roofline_obj("k_encode_mask", alg, k_max, None,
                                                 "HIP events around k_encode_mask on each rank's group stream, "
                                                 "best of %d calls' average; slowest rank" % reps),
               "k_encode_mask_ms_fastest_rank": round(k_min, 5)}
        if rank == 0:
            moved = n_total * fsz - n_local * fsz
            res.update({"bytes_into_root": moved, "GBps_into_root": round(moved / (gat_ms * 1e-3) / 1e9, 1),
                        "root_ingress_expectation_GBps": root_ingress_expectation(world),
                        "job_bytes": n_total * fsz})
            ok = bool(torch.equal(out_off, torch.arange(n_total + 1, dtype=torch.int64, device=device) * fsz))
            import oracle

            for q in sorted({0, 1, chunk - 1, chunk, chunk * (world - 1) + 5, n_total // 2 + 3, n_total - 1}):
                if q >= n_total:
                    continue
                d = wl.c5_desc(np.array([q]), size)
                d["src_off"] = 0
                ref, _ = oracle.encode_batch(wl.c5_payload_np(np.array([q]), size), d)
                ok &= bool(np.array_equal(out[q * fsz: (q + 1) * fsz].cpu().numpy(), ref))
            res["root_check"] = bool(ok)
        del payload, wire, out
        torch.cuda.empty_cache()
        return res
    finally:
        g.close()


def c5_job_leg(world, rank, device, codec, n_total=1 << 20, size=16384, chunk=1024):
    """Cross-check of c5_rank_leg through torch.distributed instead of the
    product's entry: the same round-robin shards encoded per rank
    (wsg_encode_batch), the framed output moved to rank 0 by torch's RCCL
    group (cppserver_amd.shard.gather_frames), reassembled in frame order
    and sampled against the oracle.  Encode and gather times are max over
    ranks."""
    import torch

    import cppserver_amd as ca
    from cppserver_amd import shard
    from cppserver_amd import workloads as wl

    ids = shard.rank_frames(rank, world, n_total, chunk)
    payload = wl.c5_payload_torch(ids, size, device=device)
    desc = ca.desc_to_tensor(wl.c5_desc(ids, size), device)
    fsz = ca.frame_size(0x82, True, size)
    wire = torch.empty(len(ids) * fsz, dtype=torch.uint8, device=device)
    woff = torch.empty(len(ids) + 1, dtype=torch.int64, device=device)
    codec.encode_batch(payload, desc, wire=wire, wire_cap=wire.numel(), wire_off=woff)   # warm
    codec.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    e0.record()
    reps = 3
    for _ in range(reps):
        codec.encode_batch(payload, desc, wire=wire, wire_cap=wire.numel(), wire_off=woff)
    e1.record()
    e1.synchronize()
    codec.sync()
    enc_ms = max_over_ranks(e0.elapsed_time(e1) / reps, world, device)
    del payload
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    parts = shard.gather_frames(*_gather_tensors(wire, woff, rccl_group()), group=rccl_group())
    torch.cuda.synchronize()
    dt = max_over_ranks(time.perf_counter() - t0, world, device)
    res = {"workload": "C5: %d x %d B frames round-robin (chunks of %d) over %d GPUs, gather to rank 0"
                       % (n_total, size, chunk, world),
           "encode_ms": round(enc_ms, 3),
           "encode_GiBps_job": round(n_total * size / (enc_ms * 1e-3) / GIB, 1),
           "gather_ms": round(dt * 1e3, 3)}
    if parts is not None:
        moved = sum(int(p[1][-1].item()) for r, p in enumerate(parts) if r != 0)
        ok, total = gather_root_check(parts, n_total, size, chunk)
        res.update({"bytes_into_root": moved, "GBps_into_root": round(moved / dt / 1e9, 1), "job_bytes": total,
                    "root_check": ok})
    del parts, wire
    torch.cuda.empty_cache()
    return res


def pcie_all_ranks_leg(w, world, rank, device, reps=3):
    """The host-inclusive decode (pinned host wire -> H2D -> k_decode -> D2H,
    wsg_decode_batch_host) on every rank at once, each over its own GPU's
    PCIe link: the one-process-per-GPU form of a server decoding socket
    buffers on all GPUs.  Payload GiB/s over all ranks (max-over-ranks time)
    and one rank's own rate."""
    import cppserver_amd as ca

    # every rank reaches every collective below, whatever fails locally (a
    # rank that raised between them would leave the others waiting)
    wire, fs, _ = w.host
    err = None
    try:
        pin_in, pin_out = ca.pinned_empty(len(wire)), ca.pinned_empty(len(wire))
        pin_in[:] = wire
        rc, _, _ = w.codec.decode_batch_host(pin_in, fs, out=pin_out)   # warm (staging slots)
        if rc != 0:
            err = "wsg_decode_batch_host: %d" % rc
    except Exception as e:   # noqa: BLE001
        err = repr(e)[:200]
    barrier(world)
    t0 = time.perf_counter()
    if err is None:
        for _ in range(reps):
            rc, _, _ = w.codec.decode_batch_host(pin_in, fs, out=pin_out)
            if rc != 0:
                err = "wsg_decode_batch_host: %d" % rc
                break
    dt = time.perf_counter() - t0 if err is None else float("inf")
    mine = w.payload_bytes * reps / dt / GIB
    dt = max_over_ranks(dt, world, device)
    if err is not None or dt == float("inf"):
        return {"error": err or "another rank failed"}
    ok = bool(np.array_equal(pin_out[int(fs[0]): int(fs[0]) + 64], np.asarray(oracle_decode_head(wire, fs))))
    return {"workload": "every rank: %d x %d B frames from pinned host memory, decoded on its GPU"
                        % (len(fs), w.payload_bytes // len(fs)),
            "all_ranks_GiBps": round(world * w.payload_bytes * reps / dt / GIB, 2),
            "rank0_GiBps": round(mine, 2), "check": ok}


def oracle_decode_head(wire, fs):
    """The first 64 output bytes of frame 0 (the oracle's decode of it)."""
    import oracle

    a = int(fs[0])
    b = int(fs[1]) if len(fs) > 1 else len(wire)
    rc, ref, _ = oracle.decode_batch(np.ascontiguousarray(wire[a:b]), np.zeros(1, np.uint64))
    assert rc == 0
    return ref[:64]


def c5_capi_leg(world, rank, n_total=1 << 20, timeout=300):
    """C5 through the one-process multi-GPU C-ABI entry (SURVEY §8b-3:
    wsg_mgpu_create over all N GPUs, RCCL inside the library), what a C++
    server calls: tools/mgpu_c5.py, run by rank 0 in a child process under a
    time limit while the other ranks wait at a barrier (a collective that
    fails to start must not hold the bench line)."""
    import subprocess

    res = None
    if rank == 0:
        env = dict(os.environ)
        if os.environ.get("WSG_BENCH_SHARE_DEVICES") == "1":
            env["WSG_MGPU_ONE_DEVICE"] = "1"   # the rehearsal's ranks share a GPU: so do the tool's
        try:
            r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "mgpu_c5.py"), str(world), str(n_total)],
                               capture_output=True, text=True, timeout=timeout, env=env)
            if r.returncode == 0:
                res = json.loads(r.stdout.strip().splitlines()[-1])
            else:
                res = {"error": (r.stderr or r.stdout).strip()[-300:]}
        except subprocess.TimeoutExpired:
            res = {"error": "no result within %d s" % timeout}
    barrier(world)
    return res


def fanout_many_leg(w, m=16, reps=10):
    """The multicast tick (ws_multicast_server.cpp:104-114: `messages_rate`
    messages per tick, each to every client) as ONE wsg_fanout_encode_many
    call: m x C4 (4 KiB messages x 10000 client keys, 41 MB of frames each),
    timed back to back; per-message time next to the single fan-out step."""
    t = w.torch
    c = w.codec
    rng = np.random.default_rng(99)
    length, k = w.length, int(w.keys.numel())
    arena = t.from_numpy(rng.integers(0, 256, m * length, dtype=np.uint8)).to(w.keys.device)
    src = np.arange(m, dtype=np.uint64) * np.uint64(length)
    lens = np.full(m, length, dtype=np.uint64)
    ops = np.full(m, 0x82, dtype=np.uint8)
    wire, off = c.fanout_many(arena, src, lens, ops, w.keys)
    c.sync()
    e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        c.fanout_many(arena, src, lens, ops, w.keys, wire=wire)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    import cppserver_amd as ca

    fsz = ca.frame_size(0x82, True, length)
    bytes_out = m * k * fsz
    # the bare write stream of the same bytes on the same buffer (torch's
    # zero_: the runtime's fill), back to back like the calls above: the
    # write-only ceiling the fan-out's stores run against
    wire.zero_()
    e0.record()
    for _ in range(reps):
        wire.zero_()
    e1.record()
    e1.synchronize()
    fill_ms = e0.elapsed_time(e1) / reps
    return {"messages": m, "us_per_call": round(ms * 1e3, 2), "us_per_message": round(ms * 1e3 / m, 2),
            "write_GBps": round(bytes_out / (ms * 1e-3) / 1e9, 1), "frame_bytes": fsz,
            "bare_write_stream": {"us": round(fill_ms * 1e3, 2), "write_GBps": round(bytes_out / (fill_ms * 1e-3) / 1e9, 1),
                                  "fanout_vs_bare": round(fill_ms / ms, 4),
                                  "what": "zero_() of the same bytes, back to back (the runtime's fill)"}}


def c4_graph_leg(w, steps, reps=5):
    """C4 as a captured graph of `steps` fan-out launches, replayed `reps`
    times; HIP events around each replay.  Per-launch time and its frac."""
    import statistics

    t = w.torch
    st = t.cuda.Stream()
    g = t.cuda.CUDAGraph()
    with t.cuda.stream(st):
        w.launch()   # warm on the capture stream
        st.synchronize()
        with t.cuda.graph(g, stream=st):
            for _ in range(steps):
                w.launch()
    g.replay()
    t.cuda.synchronize()
    e0, e1 = t.cuda.Event(enable_timing=True), t.cuda.Event(enable_timing=True)
    us = []
    for _ in range(reps):
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        us.append(e0.elapsed_time(e1) * 1e3 / steps)
    med = statistics.median(us)
    return {"launches_per_replay": steps, "replays": reps, "us_per_launch": round(med, 3),
            "achieved_GBps": round(w.alg_bytes / (med * 1e-6) / 1e9, 1),
            "frac": round(w.alg_bytes / (med * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4),
            "value_GiBps": round(w.payload_bytes / (med * 1e-6) / GIB, 2)}


def roofline_obj(kernel, alg_bytes, avg_ms, traffic, timing, minmax=None):
    """The roofline object of one kernel: algorithmic bytes per launch over
    its average launch duration (HIP events on its launch stream), against
    the HBM peak; `traffic` = PMC HBM bytes per launch (profiles/), or None;
    `minmax` = (shortest, longest) timed launch, where each launch is timed."""
    achieved = alg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms else 0.0
    r = {"bound": "hbm", "kernel": kernel, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "alg_bytes_per_launch": alg_bytes,
         "avg_kernel_ms": round(avg_ms, 5), "kernel_timing": timing}
    if minmax is not None and avg_ms:
        r.update({"launch_min_ms": round(minmax[0], 5), "launch_max_ms": round(minmax[1], 5),
                  "launch_spread_pct": round(100 * (minmax[1] - minmax[0]) / avg_ms, 2)})
    return r


_ROCTX = []


def marker(name):
    """A roctx range around a leg's timed region (rocprofv3 --marker-trace
    lines the kernels of a trace up with the bench objects:
    tools/trace_split.py); a no-op where the roctx library is absent."""
    import contextlib
    import ctypes

    if not _ROCTX:
        try:
            lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            _ROCTX.append(lib)
        except OSError:
            _ROCTX.append(None)

    @contextlib.contextmanager
    def rng():
        lib = _ROCTX[0]
        if lib is not None:
            lib.roctxRangePushA(name.encode())
        try:
            yield
        finally:
            if lib is not None:
                lib.roctxRangePop()

    return rng()


def timed_region(w, steps, world, device):
    """EXACTLY `steps` steps between barrier + torch.cuda.synchronize() on
    both sides (wall clock, max over ranks), with the dominant kernels' HIP
    events.  C2/C4 steps are ONE launch of the dominant kernel, so two events
    around the region on its launch stream (torch's current stream) give its
    average duration without adding anything between launches; C3/C5 steps
    launch several kernels, so the library times the dominant one of every
    `every`-th call (each event pair costs a few us: every 8th call for long
    regions, every call for the short sub-config regions)."""
    import torch

    single = w.cfg in ("c2", "c4")
    codecs = [w.codec] + ([w.dec_codec] if w.cfg == "c3" else [])
    every = 1 if steps <= 20 else 8
    if not single:
        for c in codecs:
            c.timing(True, every=every)
            c.timing_read(reset=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # torch creates the HIP events at their first record(): do that here, not
    # inside the timed region (a first hipEventCreate costs tens of us)
    e0.record()
    e1.record()
    barrier(world)
    torch.cuda.synchronize()
    # no Python garbage collection inside the region (a full collection of the
    # interpreter's objects is a host stall of milliseconds, unrelated to the
    # path measured).  Not gc.collect() here: a collection right before t0
    # leaves the host's caches cold and adds ~100 us to a 20-step region
    # (tools/region_gap.py: wall - events 22 us without it, 119 us with it)
    gc.disable()
    try:
        with marker("bench.%s.timed" % w.cfg):
            t0 = time.perf_counter()
            e0.record()
            for _ in range(steps):
                w.step()
            e1.record()
            t_sub = time.perf_counter()
            torch.cuda.synchronize()
            # the clock stops at this rank's synchronize; the closing barrier
            # only lines the ranks up again (max over ranks takes the slowest)
            elapsed = time.perf_counter() - t0
    finally:
        gc.enable()
    barrier(world)
    region_ms = e0.elapsed_time(e1)
    if single:
        kern, spread = [(region_ms, steps)], [None]
        note = "HIP events around the timed region / steps (one launch per step)"
    else:
        kern, spread = [], []
        for c in codecs:
            spread.append(c.timing_minmax())
            kern.append(c.timing_read(reset=True))
            c.timing(False)
        note = ("HIP events around the dominant kernel of every call in the timed region" if every == 1 else
                "HIP events around the dominant kernel of every %dth call in the timed region" % every)
    w.codec.sync()
    elapsed = max_over_ranks(elapsed, world, device)
    avgs = [max_over_ranks(ms / max(k, 1), world, device) for ms, k in kern]
    return {"elapsed": elapsed, "region_event_ms": region_ms, "kernel_avg_ms": avgs, "timing": note,
            "minmax": spread, "submit_ms": (t_sub - t0) * 1e3}


# CPU baselines run after every GPU leg and host leg: a baseline loads every
# core for seconds, and the legs timed right after it ran slower (a C4
# region 12.6 us per launch after C3's 16-thread baseline against 8.0 us
# with none before it, profiles/r4/c4_after_cpu_baseline.log)
_DEFERRED_CPU = []


def defer_cpu_baseline(obj, w, seconds):
    import types

    snap = types.SimpleNamespace(cfg=w.cfg, host=w.host, payload_bytes=w.payload_bytes,
                                 length=getattr(w, "length", None))
    _DEFERRED_CPU.append((obj, snap, seconds))


def run_deferred_cpu_baselines(cpu):
    while _DEFERRED_CPU:
        obj, snap, seconds = _DEFERRED_CPU.pop(0)
        try:
            obj["cpu_baseline"], obj["cpu_baseline_mt"] = cpu_baseline(snap, seconds, cpu)
        except Exception as e:   # noqa: BLE001  (reported; the GPU numbers stand)
            obj["cpu_baseline"] = {"error": repr(e)[:300]}


def config_obj(args, cfg, codec, rank, world, device, steps, warmup, cpu):
    """One BASELINE config measured in this run: its own workload, spot check
    against the oracle, warm-up, timed region, roofline per dominant kernel
    (C3: both halves of the round trip), and the CPU baseline beside it."""
    import argparse as _ap

    sub = _ap.Namespace(**dict(vars(args), config=cfg, frames=None, size=None, messages=1))
    w = Workload(sub, codec, rank, device)
    try:
        ok = w.spot_check()
        # warm-up by time: after the seconds of host work above (input
        # generation, the oracle spot check) the GPU has sat idle, and the
        # first ~15 ms of load run up to 25 % slower (tools/c3_dec.py:
        # C3's decode 0.88 -> 0.69 ms over its first 20 launches)
        warmup = warm_up(w, warmup, WARM_SECONDS)
        r = timed_region(w, steps, world, device)
        ms_step = r["elapsed"] / steps * 1e3
        obj = {"workload": w.workload, "value": round(world * w.payload_bytes * steps / r["elapsed"] / GIB, 2),
               "unit": "GiB/s", "steps": steps, "warmup": warmup, "ms_per_step": round(ms_step, 4),
               "event_ms_per_step": round(r["region_event_ms"] / steps, 4)}
        obj.update(w.extra)
        rf = roofline_obj(w.kernel, w.alg_bytes, r["kernel_avg_ms"][0], pmc_traffic(args.pmc, cfg), r["timing"],
                          r["minmax"][0])
        if cfg == "c3":
            dec = roofline_obj("k_decode", w.dec_alg_bytes, r["kernel_avg_ms"][1], pmc_traffic(args.pmc, "c3_dec"),
                               r["timing"], r["minmax"][1])
            both = w.alg_bytes + w.dec_alg_bytes
            t = sum(r["kernel_avg_ms"])
            rf = dict(dec, halves=[rf, dec],
                      round_trip={"alg_bytes": both, "kernel_ms": round(t, 5),
                                  "achieved": round(both / (t * 1e-3) / 1e9, 1),
                                  "frac": round(both / (t * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)})
        obj["roofline"] = rf
        if cfg == "c3":
            obj["k_decode_per_launch"] = decode_launches(w)
        if cfg == "c4":
            # C4 is launch-latency sensitive, report it with a graph
            # of repeats too: the same prepared launch captured `steps` times
            # and replayed once (a Python call per launch costs ~6-7 us, close
            # to the 8 us kernel, and can bound the eager region on a slow host)
            obj["graph_replay"] = c4_graph_leg(w, steps)
            # the ws_multicast tick's form: 16 such messages in ONE launch
            # (wsg_fanout_encode_many), where one 41 MB fan-out is too short
            # to reach the write rate on its own
            many = fanout_many_leg(w)
            per_msg = w.alg_bytes   # one message: frames + payload + keys
            many["frac"] = round(per_msg / (many["us_per_message"] * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
            obj["multicast_tick_16"] = many
        if cpu is not None and rank == 0:
            # timed at the end of the run (defer_cpu_baseline)
            defer_cpu_baseline(obj, w, args.cpu_seconds * 0.6)
        obj["spot_check"] = ok
        return obj
    finally:
        w.close()


def decode_launches(w, launches=60, warm=30):
    """C3's decode half launch by launch: k_decode alone
    on the round trip's wire, HIP events between launches (one launch per
    decode_batch call), after the timed region, behind `warm` untimed
    launches of its own (the synchronize before it idles the GPU, and the
    first ~15 ms of load after an idle GPU run slow: with 10 warm launches,
    7 ms, round 5's first_5_ms were 0.72-0.74 ms against a 0.676 median;
    30 cover the ramp)."""
    import statistics

    t = w.torch
    ev = [t.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
    for e in ev:
        e.record()
    t.cuda.synchronize()
    for _ in range(warm):
        w.dec_codec.decode_batch(w.wire, w.woff[:-1], out=w.out, info=w.info)
    ev[0].record()
    for i in range(launches):
        w.dec_codec.decode_batch(w.wire, w.woff[:-1], out=w.out, info=w.info)
        ev[i + 1].record()
    t.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(launches)]
    med = statistics.median(ms)
    srt = sorted(ms)
    p10, p90 = srt[launches // 10], srt[(9 * launches) // 10]
    return {"launches": launches, "median_ms": round(med, 5), "min_ms": round(min(ms), 5),
            "max_ms": round(max(ms), 5), "p10_ms": round(p10, 5), "p90_ms": round(p90, 5),
            "stdev_ms": round(statistics.pstdev(ms), 5), "spread_pct": round(100 * (max(ms) - min(ms)) / med, 2),
            "p10_p90_spread_pct": round(100 * (p90 - p10) / med, 2),
            "first_5_ms": [round(x, 4) for x in ms[:5]], "warm_launches": warm,
            "frac_at_median": round(w.dec_alg_bytes / (med * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}


SUB_CONFIGS = (("c3", 20, 3), ("c4", 200, 3), ("c5", 10, 3))   # (config, steps, min warm-up steps): bounded legs
WARM_SECONDS = 0.25


def warm_up(w, min_steps, seconds):
    """Untimed steps: at least `min_steps`, and until `seconds` of them have
    run on the GPU.  Returns the number of steps."""
    import torch

    done = 0
    t0 = time.perf_counter()
    while done < min_steps or time.perf_counter() - t0 < seconds:
        for _ in range(max(1, min_steps)):
            w.step()
        done += max(1, min_steps)
        torch.cuda.synchronize()
    w.codec.sync()
    return done


CHECK_KEYS = ("spot_check", "root_check", "check", "payload_ok", "delivered_ok", "roundtrip_ok", "all_delivered",
              "wire_ok", "off_ok")


def failed_checks(obj, path=""):
    """Every parity / delivery check in the line's legs that is false, and
    every leg that recorded an error, as dotted paths (the run exits non-zero
    when there is any)."""
    out = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            p = path + "." + k if path else k
            if k in CHECK_KEYS and v is not True:
                out.append("%s=%s" % (p, v))
            elif k == "error":
                out.append("%s: %s" % (path or k, str(v)[:120]))
            else:
                out.extend(failed_checks(v, p))
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            out.extend(failed_checks(v, "%s[%d]" % (path, i)))
    return out


def main():
    args = parse()
    check_world(args)   # (--gpus N > 1 without a launch: starts the ranks and exits)
    if args.dry_run:
        return dry_run(args)
    failed = []
    import torch

    import cppserver_amd as ca

    rank, world, local = dist_setup(args)
    device = torch.device("cuda", local)
    codec = ca.Codec(local)
    w = Workload(args, codec, rank, device)

    # the spot check (one step, then seconds of host-side oracle work with the
    # GPU idle) comes first, so that the warm-up steps run right before the
    # timed region: the first launch after an idle GPU takes 150-165 us
    # instead of 86 (tools/ramp.py), 4 % of a 20-step region
    ok = w.spot_check()
    for _ in range(args.warmup):
        w.step()
    codec.sync()

    r = timed_region(w, args.steps, world, device)
    elapsed = r["elapsed"]
    ms_per_step = elapsed / args.steps * 1e3
    value = world * w.payload_bytes * args.steps / elapsed / GIB
    k_avg_ms = r["kernel_avg_ms"][0]
    pmc_key = w.cfg + ("x%d" % w.m if w.cfg == "c4" and w.m > 1 else "")
    traffic = pmc_traffic(args.pmc, pmc_key) if args.frames is None and args.size is None else None
    roof = roofline_obj(w.kernel, w.alg_bytes, k_avg_ms, traffic, r["timing"], r["minmax"][0])
    if w.cfg == "c3":
        dec = roofline_obj("k_decode", w.dec_alg_bytes, r["kernel_avg_ms"][1],
                           pmc_traffic(args.pmc, "c3_dec") if traffic is not None else None, r["timing"],
                           r["minmax"][1])
        roof = dict(dec, halves=[roof, dec])

    extras = {"event_ms_per_step": round(r["region_event_ms"] / args.steps, 4),
              # where the wall clock's excess over the events goes: the host's
              # time to submit the region (launches queue behind a busy GPU
              # after the first) and the rest, first-launch latency + wake-up
              "region_host": {"submit_ms": round(r["submit_ms"], 4),
                              "wall_minus_events_ms": round(elapsed * 1e3 - r["region_event_ms"], 4)}}
    if w.cfg == "c5" and world > 1:
        # the exchange step: the job's shards encoded and gathered to rank 0
        # by the product's rank form (RCCL inside the library)
        try:
            extras["c5_job"] = c5_rank_leg(world, rank, local, device)
        except Exception as e:   # noqa: BLE001
            extras["c5_job"] = {"error": repr(e)[:300]}
    if w.cfg == "c2" and world > 1 and not args.no_extras:
        try:
            extras["pcie_inclusive_all_ranks"] = pcie_all_ranks_leg(w, world, rank, device)
        except Exception as e:   # noqa: BLE001  (reported; the headline stands)
            extras["pcie_inclusive_all_ranks"] = {"error": repr(e)[:300]}
    if w.cfg == "c2" and world > 1 and not args.no_c5_job:
        # C5 (BASELINE configs[4]) on the same GPUs through the product's RCCL
        # rank form; a failure is reported in the line (and fails the run, see
        # failed_checks), it does not take the headline's numbers with it
        c5_frames = int(os.environ.get("WSG_C5_FRAMES", 1 << 20))
        try:
            extras["c5_job"] = c5_rank_leg(world, rank, local, device, n_total=c5_frames)
        except Exception as e:   # noqa: BLE001
            extras["c5_job"] = {"error": repr(e)[:300]}
        torch.cuda.empty_cache()
        if os.environ.get("WSG_BENCH_CAPI_RCCL", "1") != "0":
            # the one-process form of the same entry (wsg_mgpu_create over all
            # N GPUs, device / xGMI peer copies), in a child process
            capi = c5_capi_leg(world, rank, n_total=c5_frames)
            if capi is not None:
                extras["c5_job_one_process"] = capi
        if os.environ.get("WSG_BENCH_TORCH_GATHER") == "1":
            # labelled cross-check, only when asked and after the product's
            # legs: the same job gathered by torch.distributed's own RCCL
            # (a second RCCL stack in the rank from here on)
            try:
                extras["c5_job_torch_crosscheck"] = c5_job_leg(world, rank, device, codec, n_total=c5_frames)
            except Exception as e:   # noqa: BLE001
                extras["c5_job_torch_crosscheck"] = {"error": repr(e)[:300]}
    cpu = host_cpu() if (rank == 0 and world == 1 and not args.no_cpu) else None
    headline_cpu = {}
    if cpu is not None:
        defer_cpu_baseline(headline_cpu, w, args.cpu_seconds)
    if rank == 0 and world == 1 and not args.no_extras:
        extras["torch_copy_GBps"] = round(torch_copy_rate(w), 1)   # for scale, not a ceiling (torch_copy_rate)
        pc = pcie_inclusive(w)
        if pc is not None:
            extras["pcie_inclusive_GiBps"] = pc
        if w.cfg == "c4" and w.m == 1:
            extras["hip_graph"] = fanout_graph_leg(w)
            extras["fanout_many"] = fanout_many_leg(w)
        if w.cfg == "c2":
            extras["echo_size_device"] = echo_size_leg(w)
    headline_cfg = w.cfg
    workload_name, workload_extra = w.workload, w.extra
    w.close()
    del w
    torch.cuda.empty_cache()
    # the other BASELINE configs (C3 round trip, C4 fan-out, C5 1 Mi x 16 KiB
    # job on this GPU), each a bounded leg with its own roofline and CPU
    # baseline, after the headline's own region (its inputs are freed first)
    if headline_cfg == "c2" and world == 1 and not args.no_configs:
        for cfg, steps, warm in SUB_CONFIGS:
            try:
                extras[cfg] = config_obj(args, cfg, codec, rank, world, device, steps, warm, cpu)
            except Exception as e:   # noqa: BLE001  (reported; the headline stands)
                extras[cfg] = {"error": repr(e)[:300]}
            torch.cuda.empty_cache()
    # the host-side legs run child processes of the product library;
    # $WSG_BENCH_HOST_LEGS=0 skips them (the rocprofv3 trace run: the
    # profiler follows child processes, and tracing their ~1e5 small launches
    # per second takes minutes; the GPU legs above are unchanged by it)
    host_legs = os.environ.get("WSG_BENCH_HOST_LEGS", "1") != "0"
    if rank == 0 and world == 1 and not args.no_extras and headline_cfg == "c2" and host_legs:
        # the legs' processes on the GPU's NUMA node (inherited affinity;
        # the reference-algorithm legs alike), this thread's mask restored after
        node, cpus = gpu_node_cpus(local)
        mask = os.sched_getaffinity(0)
        if cpus:
            os.sched_setaffinity(0, cpus)
        try:
            sb = session_batch_leg()
            if sb is not None:
                extras["session_batch"] = sb
            c1 = echo_c1_leg()
            if c1 is not None:
                extras["echo_c1"] = c1
            mc = multicast_leg()
            if mc is not None:
                extras["ws_multicast"] = mc
        finally:
            if cpus:
                os.sched_setaffinity(0, mask)
        extras["host_legs_cpus"] = {"numa_node": node, "cpus": len(cpus) if cpus else None,
                                    "what": "session / echo / multicast legs bound to the GPU's NUMA node "
                                            "(both the drop-in and the reference-algorithm legs)"}
    if cpu is not None:
        run_deferred_cpu_baselines(cpu)
    cpu1, cpu_mt = headline_cpu.get("cpu_baseline"), headline_cpu.get("cpu_baseline_mt")

    if world > 1:
        import torch.distributed as dist

        okt = torch.tensor([1 if ok else 0])
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    if rank == 0:
        cfg = args.config
        line = {
            "metric": METRIC if cfg == "c2" else "WS payload GiB/s (device-resident), " + cfg.upper(),
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if cfg == "c5" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded random payloads and keys)",
            "config": dict({"workload": workload_name,
                            "parallelism": ("1 Mi-frame job split round-robin over %d GPUs" % world) if cfg == "c5"
                            else "independent batch per GPU (dp%d)" % world}, **workload_extra),
            "roofline": roof,
            "cpu_baseline": cpu1,
            "cpu_baseline_mt": cpu_mt,
            "spot_check": ok,
        }
        line.update(extras)
        failed = failed_checks(extras)
        if not ok:
            failed.insert(0, "spot_check (headline)")
        # the top-level spot_check is every leg's parity check and root check
        # together; the headline's own stays beside it
        line["spot_check_headline"] = ok
        line["spot_check"] = not failed
        line["failed_checks"] = failed
        print(json.dumps(line), flush=True)
        if failed:
            print("bench.py: %d failed check(s) or leg error(s): %s" % (len(failed), "; ".join(failed)),
                  file=sys.stderr, flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    codec.close()
    if rank == 0 and failed:
        sys.exit(1)


if __name__ == "__main__":
    main()
