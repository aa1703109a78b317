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

Other configs (--config c3|c4|c5) are available for tracking; the headline
line is c2.
"""
import argparse
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
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="budget of the CPU baseline leg")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip copy-ceiling and PCIe-inclusive legs")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return ap.parse_args()


def dist_setup(args):
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist

        # $WSG_BENCH_BACKEND=gloo rehearses the N-rank path on fewer GPUs
        # (ranks share devices round-robin); the real run is RCCL, one GPU per rank
        backend = os.environ.get("WSG_BENCH_BACKEND", "nccl")
        if backend != "nccl":
            local = local % torch.cuda.device_count()
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(local)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def max_over_ranks(x, world, device):
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=device)
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
            self.workload = "C3 mask+unmask round trip: %d frames, payload uniform in [128, 65536] B" % n
            self.extra = {"frames": n, "wire_bytes": cap}
        elif self.cfg == "c4":
            k = args.frames or 10000
            length = args.size or 4096
            payload, keys = wl.c4_fanout(length, k, seed=4000 + rank)
            self.payload = torch.from_numpy(payload).to(device)
            self.keys = torch.from_numpy(keys.view(np.int32)).to(device)
            fsz = ca.frame_size(0x82, True, length)
            self.wire = torch.empty(fsz * k, dtype=torch.uint8, device=device)
            self.payload_bytes = length * k
            self.alg_bytes = fsz * k + length + 4 * k
            # frame sizes that are a multiple of 4 take the period kernel (wsg_kernels.hip launch_fanout_period)
            self.kernel = "k_fanout_period" if fsz % 4 == 0 else "k_fanout_flat"
            self.workload = "C4 fan-out: one %d B payload masked with %d client keys" % (length, k)
            self.extra = {"keys": k, "wire_bytes": fsz * k}
        else:  # c5: this rank's round-robin shard of 1 Mi x 16 KiB frames, encode
            world = int(os.environ.get("WORLD_SIZE", "1"))
            size = args.size or 16384
            payload, desc, ids = wl.c5_shard(rank, world, n_total=args.frames or (1 << 20), size=size,
                                             max_frames=None)
            self.payload = torch.from_numpy(payload).to(device)
            self.desc = ca.desc_to_tensor(desc, device)
            n = len(desc)
            cap = n * ca.frame_size(0x82, True, size)
            self.wire = torch.empty(cap, dtype=torch.uint8, device=device)
            self.woff = torch.empty(n + 1, dtype=torch.int64, device=device)
            self.cap = cap
            self.payload_bytes = n * size
            self.alg_bytes = n * size + cap
            self.kernel = "k_encode_mask"
            self.workload = "C5 encode shard: %d x %d B frames of a 1 Mi-frame job (round-robin)" % (n, size)
            self.extra = {"frames_this_rank": n, "wire_bytes": cap}

    def step(self):
        c = self.codec
        if self.cfg == "c2":
            wire, out = self.batches[self.turn]
            self.turn ^= 1
            c.decode_batch(wire, self.fs, out=out, info=self.info)
        elif self.cfg == "c3":
            c.encode_batch(self.payload, self.desc, wire=self.wire, wire_cap=self.cap, wire_off=self.woff)
            c.decode_batch(self.wire, self.woff[:-1], out=self.out, info=self.info)
        elif self.cfg == "c4":
            c.fanout(self.payload, self.keys, 0x82, True, wire=self.wire)
        else:
            c.encode_batch(self.payload, self.desc, wire=self.wire, wire_cap=self.cap, wire_off=self.woff)

    def spot_check(self):
        """Cheap self-check of one step's output (not the oracle)."""
        if self.cfg != "c2":
            return True
        wire, fs, keys = self.host
        self.codec.decode_batch(self.wire, self.fs, out=self.out, info=self.info)
        self.codec.sync()
        out = self.out.cpu().numpy()
        n = len(fs)
        fsz = len(wire) // n
        ok = True
        for i in (0, n // 2, n - 1):
            s = int(fs[i])
            hdr = fsz - (self.payload_bytes // n)
            p = wire[s + hdr: s + fsz]
            kb = np.frombuffer(int(keys[i]).to_bytes(4, "little"), np.uint8)
            ok &= bool(np.array_equal(out[s + hdr: s + fsz], p ^ np.resize(kb, len(p))))
            ok &= bool(np.array_equal(out[s: s + hdr], wire[s: s + hdr]))
        return ok


def cpu_baseline(w, seconds):
    """The oracle's faithful byte-loop restatement of the reference codec,
    timed on this host on a bounded sample of the same workload."""
    import oracle

    if w.cfg != "c2":
        return None, None
    wire, fs, _ = w.host
    n = len(fs)
    per_frame = w.payload_bytes // n
    # sample: the first m frames; size it so 1 thread runs ~seconds/2 in total
    t_probe = oracle.time_decode(wire, fs[: max(1, n // 16)], threads=1, iters=1)
    rate = (n // 16) * per_frame / max(t_probe, 1e-9)
    m = n
    iters = max(3, int((seconds / 2) * rate / (m * per_frame)))
    fs_s = fs[:m]
    t1 = oracle.time_decode(wire, fs_s, threads=1, iters=iters)
    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    tn = oracle.time_decode(wire, fs_s, threads=threads, iters=max(3, iters * threads // 2))
    sample = "%d frames x %d B (%.0f MiB), PrepareReceiveFrame per whole frame, median of %d passes" % (
        m, per_frame, m * per_frame / 2**20, iters)
    one = {"value": m * per_frame / t1 / GIB, "unit": "GiB/s", "cores": 1, "kind": "port", "sample": sample}
    mt = {"value": m * per_frame / tn / GIB, "unit": "GiB/s", "cores": threads, "kind": "port",
          "sample": sample + "; one session per thread over a contiguous frame slice"}
    return one, mt


def copy_ceiling(w, reps=10):
    """torch device-to-device copy of the same byte count (measured ceiling)."""
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
        r = subprocess.run([exe, mode] + args, capture_output=True, text=True, timeout=timeout)
        if r.returncode != 0:
            out[leg] = {"error": (r.stderr or r.stdout).strip()[-300:]}
            continue
        d = json.loads(r.stdout.strip().splitlines()[-1])
        out[leg] = {k: d[k] for k in ("batched_GiBps", "per_call_GiBps", "batched_frames_per_s",
                                       "per_call_frames_per_s", "delivered_ok")}
    out["workload"] = ("rx/tx: 1024 sessions x 4 frames x 64 KiB; *_32B: 256 sessions x 64 frames x 32 B; "
                       "host buffers (PCIe + host framing + callbacks inside)")
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
        c.fanout(w.payload, w.keys, 0x82, True, wire=wires[i & 1])
    t.cuda.synchronize()
    g = t.cuda.CUDAGraph()
    with t.cuda.graph(g):
        for i in range(per_graph):
            c.fanout(w.payload, w.keys, 0x82, True, wire=wires[i & 1])
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


def gather_leg(w, world, device):
    """C5's exchange step: every rank's framed output to rank 0 over RCCL
    (variable-size grouped send/recv, cppserver_amd.shard.gather_frames),
    timed once after the encode steps; reported beside the kernel rate."""
    import torch

    from cppserver_amd import shard

    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    parts = shard.gather_frames(w.wire, w.woff)
    torch.cuda.synchronize()
    barrier(world)
    dt = time.perf_counter() - t0
    moved = None
    if parts is not None:
        moved = sum(int(p[1][-1].item()) for r, p in enumerate(parts) if r != 0)
    dt = max_over_ranks(dt, world, device)
    return {"ms": round(dt * 1e3, 3), "bytes_into_root": moved,
            "GBps_into_root": round(moved / dt / 1e9, 1) if moved else None}


def main():
    args = parse()
    import torch

    import cppserver_amd as ca

    rank, world, local = dist_setup(args)
    device = torch.device("cuda", local)
    codec = ca.Codec(local)
    w = Workload(args, codec, rank, device)

    for _ in range(args.warmup):
        w.step()
    codec.sync()
    ok = w.spot_check()

    # Kernel time, live over the timed region, on the stream the kernels are
    # launched on (torch's current stream).  C2 and C4 steps are ONE launch
    # of the dominant kernel, so two events around the region give its
    # average duration (launch gaps included: an upper bound) without adding
    # anything between launches.  C3/C5 steps launch several kernels: HIP
    # events around the dominant one of every 8th step (each event packet
    # costs a few us, so timing every step would slow the step itself).
    single = w.cfg in ("c2", "c4")
    if not single:
        codec.timing(True, every=8)
        codec.timing_read(reset=True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record()
    for _ in range(args.steps):
        w.step()
    e1.record()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    if single:
        kernel_ms, launches = e0.elapsed_time(e1), args.steps
    else:
        kernel_ms, launches = codec.timing_read(reset=True)
        codec.timing(False)
    codec.sync()

    elapsed = max_over_ranks(elapsed, world, device)
    ms_per_step = elapsed / args.steps * 1e3
    value = world * w.payload_bytes * args.steps / elapsed / GIB
    k_avg_ms = kernel_ms / max(launches, 1)
    k_avg_ms = max_over_ranks(k_avg_ms, world, device)
    achieved = w.alg_bytes / (k_avg_ms * 1e-3) / 1e9
    traffic = pmc_traffic(args.pmc, w.cfg) if args.frames is None and args.size is None else None

    extras = {}
    if w.cfg == "c5" and world > 1:
        extras["gather"] = gather_leg(w, world, device)
    if rank == 0 and world == 1 and not args.no_extras:
        extras["copy_ceiling_GBps"] = round(copy_ceiling(w), 1)
        pc = pcie_inclusive(w)
        if pc is not None:
            extras["pcie_inclusive_GiBps"] = pc
        if w.cfg == "c4":
            extras["hip_graph"] = fanout_graph_leg(w)
        if w.cfg == "c2":
            extras["echo_size_device"] = echo_size_leg(w)
            sb = session_batch_leg()
            if sb is not None:
                extras["session_batch"] = sb
    cpu1 = cpu_mt = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu1, cpu_mt = cpu_baseline(w, args.cpu_seconds)

    if world > 1:
        import torch.distributed as dist

        okt = torch.tensor([1 if ok else 0], device=device)
        dist.all_reduce(okt, op=dist.ReduceOp.MIN)
        ok = bool(okt.item())

    if rank == 0:
        line = {
            "metric": METRIC if w.cfg == "c2" else "WS payload GiB/s (device-resident), " + w.cfg.upper(),
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong" if w.cfg == "c5" else "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded random payloads and keys)",
            "config": dict({"workload": w.workload,
                            "parallelism": ("1 Mi-frame job split round-robin over %d GPUs" % world) if w.cfg == "c5"
                            else "independent batch per GPU (dp%d)" % world}, **w.extra),
            "roofline": {
                "bound": "hbm",
                "kernel": w.kernel,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 4),
                "traffic": traffic,
                "alg_bytes_per_launch": w.alg_bytes,
                "avg_kernel_ms": round(k_avg_ms, 5),
                "kernel_timing": ("HIP events around the timed region / steps (one launch per step)" if single
                                  else "HIP events around every 8th launch in the timed region"),
            },
            "cpu_baseline": cpu1,
            "cpu_baseline_mt": cpu_mt,
            "spot_check": ok,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()
    codec.close()


if __name__ == "__main__":
    main()
