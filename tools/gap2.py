"""bench.py's C2 region, one region per trial as the bench runs it (seconds
of host work with the GPU idle, 5 warm-up launches, then K launches between
synchronizes), for variants of how the host starts and ends the region:

  base   torch's current stream resolved per launch, blocking synchronize
  bound  the stream bound once when the launch is prepared
  poll   bound, and the host polls the end event before the synchronize
  warm   bound + poll, after a time-based warm-up (0.25 s of launches)

Prints wall - events per region (median, max over trials) for each.
Diagnostic only.  usage: python tools/gap2.py [trials] [K]
"""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def host_work(seconds):
    t0 = time.perf_counter()
    x = 0
    while time.perf_counter() - t0 < seconds:
        x += sum(range(1000))
    return x


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    if os.environ.get("GAP_ROCTX") == "1":   # load roctx and open/close one range, as bench.marker does
        import ctypes

        lib = ctypes.CDLL("librocprofiler-sdk-roctx.so.1")
        lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        lib.roctxRangePushA(b"gap2")
        lib.roctxRangePop()
        print("roctx loaded", flush=True)
    n, size = 4096, 65536
    wire, fs, _ = wl.c2_wire(n, size, seed=1)
    ws = [torch.from_numpy(wire).cuda(), torch.from_numpy(wl.c2_wire(n, size, seed=2)[0]).cuda()]
    outs = [torch.empty_like(ws[0]) for _ in ws]
    f = torch.from_numpy(fs.view(np.int64)).cuda()
    info = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    c = ca.Codec(0)
    cur = torch.cuda.current_stream()
    free = [c.prepare_decode(ws[i], f, outs[i], info) for i in range(2)]
    bound = [c.prepare_decode(ws[i], f, outs[i], info, stream=cur) for i in range(2)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    e1.record()
    torch.cuda.synchronize()

    def region(variant):
        launch = free if variant == "base" else bound
        host_work(1.0)
        if variant == "warm":
            t = time.perf_counter()
            while time.perf_counter() - t < 0.25:
                for i in range(5):
                    launch[i & 1]()
                torch.cuda.synchronize()
        for i in range(5):
            launch[i & 1]()
        c.sync()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for i in range(k):
            launch[i & 1]()
        e1.record()
        if variant in ("poll", "warm"):
            while not e1.query():
                pass
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e6
        ev = e0.elapsed_time(e1) * 1e3
        return wall - ev, ev / k

    res = {v: [] for v in ("base", "bound", "poll", "warm")}
    for _ in range(trials):
        for v in res:
            res[v].append(region(v))
    for v, rows in res.items():
        gaps = [g for g, _ in rows]
        per = [p for _, p in rows]
        print("%-5s K=%d  wall-events median %6.1f us  max %6.1f us  (%.2f %% of the region)  kernel %.2f us"
              % (v, k, statistics.median(gaps), max(gaps), 100 * statistics.median(gaps) / (k * statistics.median(per)),
                 statistics.median(per)), flush=True)
    c.close()


if __name__ == "__main__":
    main()
