"""Where bench.py's C2 wall clock goes beyond the kernel (round 3, VERDICT
item 6): the timed region as bench.py runs it (barrier + synchronize on both
sides, K prepared wsg_decode_batch launches) against the HIP events around
it, for K = 0 (fixed cost), 20 (the driver's K) and 200, with the final wait
done by torch.cuda.synchronize() directly or after polling the end event;
then per-launch events of a 20-launch region.  Diagnostic only.

usage: python tools/gap.py
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def spin_sync():
    """$WSG_SPIN=1: hipDeviceScheduleSpin on the HIP runtime torch loaded,
    before the device is initialised (the host spins in synchronize instead
    of yielding / sleeping)."""
    import ctypes
    import glob

    libs = glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*"))
    hip = ctypes.CDLL(libs[0] if libs else "libamdhip64.so")
    rc = hip.hipSetDeviceFlags(ctypes.c_uint(1))   # hipDeviceScheduleSpin
    print("hipSetDeviceFlags(spin) ->", rc, libs[:1], flush=True)


def main():
    if os.environ.get("WSG_SPIN") == "1":
        spin_sync()
    n, size = 4096, 65536
    wire, fs, _ = wl.c2_wire(n, size, seed=1)
    ws = [torch.from_numpy(wire).cuda(), torch.from_numpy(wl.c2_wire(n, size, seed=2)[0]).cuda()]
    outs = [torch.empty_like(ws[0]) for _ in ws]
    f = torch.from_numpy(fs.view(np.int64)).cuda()
    info = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    c = ca.Codec(0)
    launch = [c.prepare_decode(ws[i], f, outs[i], info) for i in range(2)]

    def region(k, poll, pause=0.0):
        if pause:
            time.sleep(pause)   # bench.py's spot check leaves the GPU idle for seconds
        for i in range(5):
            launch[i & 1]()
        c.sync()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for i in range(k):
            launch[i & 1]()
        e1.record()
        t_sub = time.perf_counter()
        if poll:
            while not e1.query():
                pass
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        return (t1 - t0) * 1e6, e0.elapsed_time(e1) * 1e3, (t_sub - t0) * 1e6

    for poll in (False, True):
        for k in (0, 1, 20, 200):
            rows = [region(k, poll) for _ in range(7)]
            wall = sorted(r[0] for r in rows)[3]
            ev = sorted(r[1] for r in rows)[3]
            sub = sorted(r[2] for r in rows)[3]
            print("poll=%d K=%3d  wall %9.1f us  events %9.1f us  gap %7.1f us  (%.2f us/step)  submit %8.1f us"
                  % (poll, k, wall, ev, wall - ev, (wall - ev) / max(k, 1), sub), flush=True)

    # as bench.py meets it: a pause, 5 warm-up steps, 20 timed
    rows = [region(20, False, pause=1.5) for _ in range(5)]
    for wall, ev, sub in rows:
        print("after 1.5 s idle: K= 20  wall %8.1f us  events %8.1f us  gap %6.1f us (%.2f%%)" % (
            wall, ev, wall - ev, 100 * (wall - ev) / ev), flush=True)
    # per-launch events over a 20-launch region
    for trial in range(3):
        for i in range(5):
            launch[i & 1]()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
        ev[0].record()
        for i in range(20):
            launch[i & 1]()
            ev[i + 1].record()
        torch.cuda.synchronize()
        us = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(20)]
        print("trial %d per-launch us: %s" % (trial, " ".join("%.1f" % x for x in us)), flush=True)
    c.close()


if __name__ == "__main__":
    main()
