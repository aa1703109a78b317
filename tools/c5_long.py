"""C5 encode over a long back-to-back run (round 3): per-call times of
wsg_encode_batch (HIP events between calls) for 1/8 of the job and the whole
job, to tell a footprint effect from one of sustained load (the chip's clock
and power management; MI355X_MICROARCH.md "DVFS give-back").  Diagnostic only.

usage: python tools/c5_long.py [seconds_per_size]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def main():
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 0.25
    c = ca.Codec(0)
    size = 16384
    fsz = ca.frame_size(0x82, True, size)
    for frac in (8, 1, 8):
        n = (1 << 20) // frac
        ids = np.arange(n, dtype=np.int64)
        payload = wl.c5_payload_torch(ids, size, device="cuda")
        desc = ca.desc_to_tensor(wl.c5_desc(ids, size), "cuda")
        wire = torch.empty(n * fsz, dtype=torch.uint8, device="cuda")
        woff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        alg = n * size + n * fsz
        c.encode_batch(payload, desc, wire=wire, wire_cap=wire.numel(), wire_off=woff)
        c.sync()
        launches = max(10, int(secs / (6.4e-3 / frac)))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
        ev[0].record()
        for i in range(launches):
            c.encode_batch(payload, desc, wire=wire, wire_cap=wire.numel(), wire_off=woff)
            ev[i + 1].record()
        torch.cuda.synchronize()
        ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(launches)]
        k = max(1, launches // 10)
        segs = [sum(ms[a: a + k]) / len(ms[a: a + k]) for a in range(0, launches, k)]
        print("frames=%7d (1/%d) %d calls: per-call ms by tenth of the run: %s" % (
            n, frac, launches, " ".join("%.4f" % x for x in segs)), flush=True)
        print("   first tenth %.0f GB/s (frac %.3f), last tenth %.0f GB/s (frac %.3f)" % (
            alg / segs[0] / 1e6, alg / segs[0] / 8e6, alg / segs[-1] / 1e6, alg / segs[-1] / 8e6), flush=True)
        del payload, desc, wire, woff
        torch.cuda.empty_cache()
    c.close()


if __name__ == "__main__":
    main()
