"""C3's ragged decode, launch by launch (round 3): k_decode
per-launch times (HIP events between launches) over the C3 wire (65536
frames, payload uniform in [128, 65536]) for several seeds, against uniform
frames of the same total size (32 KiB + 64 B payload), so that what the
ragged tables cost is told apart from the footprint.  Diagnostic only.

usage: python tools/c3_dec.py [launches]   ($WSG_C3_WARM=seconds of warm-up
launches before each measured series; a device copy of the same wire gives
the jitter the footprint has without the codec)
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def encoded(c, payload, desc):
    cap = int(ca.frame_sizes(desc).sum())
    p = torch.from_numpy(payload).cuda()
    d = ca.desc_to_tensor(desc, "cuda")
    wire = torch.empty(cap, dtype=torch.uint8, device="cuda")
    woff = torch.empty(len(desc) + 1, dtype=torch.int64, device="cuda")
    c.encode_batch(p, d, wire=wire, wire_cap=cap, wire_off=woff)
    c.sync()
    return wire, woff


WARM = float(os.environ.get("WSG_C3_WARM", "0"))   # seconds of launches before the measured ones


def warm(fn):
    import time

    t_end = time.perf_counter() + WARM
    while time.perf_counter() < t_end:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()


def per_launch(c, wire, woff, launches, alt=None):
    out = torch.empty_like(wire)
    n = woff.numel() - 1
    info = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    bufs = [(wire, woff)] + ([alt] if alt is not None else [])
    for i in range(3):
        w, o = bufs[i % len(bufs)]
        c.decode_batch(w, o[:-1], out=out if w is wire else torch.empty_like(w), info=info)
    c.sync()
    warm(lambda: c.decode_batch(wire, woff[:-1], out=out, info=info))
    outs = [out] + ([torch.empty_like(alt[0])] if alt is not None else [])
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
    ev[0].record()
    for i in range(launches):
        j = i % len(bufs)
        c.decode_batch(bufs[j][0], bufs[j][1][:-1], out=outs[j], info=info)
        ev[i + 1].record()
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) for i in range(launches)]


def copy_launch(src, launches):
    """The same bytes through a plain device copy (hipMemcpyAsync), launch by
    launch: the jitter the hardware shows for this footprint without the codec."""
    dst = torch.empty_like(src)
    dst.copy_(src)
    torch.cuda.synchronize()
    warm(lambda: dst.copy_(src))
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
    ev[0].record()
    for i in range(launches):
        dst.copy_(src)
        ev[i + 1].record()
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) for i in range(launches)]


def show(name, ms, alg):
    med = statistics.median(ms)
    print("%-34s median %.4f ms (frac %.3f)  min %.4f  max %.4f  spread %.1f%%  stdev %.4f" % (
        name, med, alg / med / 8e9 * 1e3, min(ms), max(ms), 100 * (max(ms) - min(ms)) / med,
        statistics.pstdev(ms)), flush=True)


def main():
    launches = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    c = ca.Codec(0)
    for seed in (3000, 3001, 3002):
        payload, desc = wl.c3_batch(65536, 128, 65536, seed=seed)
        wire, woff = encoded(c, payload, desc)
        alg = 2 * wire.numel() + 40 * len(desc)
        ms = per_launch(c, wire, woff, launches)
        show("ragged seed %d (same wire)" % seed, ms, alg)
        if seed == 3000:
            print("   per launch:", " ".join("%.3f" % x for x in ms), flush=True)
            cp = copy_launch(wire, launches)
            show("device copy of the same wire", cp, 2 * wire.numel())
            print("   per launch:", " ".join("%.3f" % x for x in cp), flush=True)
            p2, d2 = wl.c3_batch(65536, 128, 65536, seed=seed + 100)
            alt = encoded(c, p2, d2)
            ms = per_launch(c, wire, woff, launches, alt=alt)
            show("ragged seed %d (two wires in turn)" % seed, ms, alg)
            del alt
        del wire, woff
        torch.cuda.empty_cache()
    rng = np.random.default_rng(5)
    desc, total = wl.ragged_desc(rng, np.full(65536, 32832))
    payload = wl.random_bytes(rng, total)
    wire, woff = encoded(c, payload, desc)
    alg = 2 * wire.numel() + 40 * len(desc)
    show("uniform 32832 B frames", per_launch(c, wire, woff, launches), alg)
    c.close()


if __name__ == "__main__":
    main()
