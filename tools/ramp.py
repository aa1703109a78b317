"""C2 decode after an idle pause: per-launch k_decode times (HIP events
between launches) for the first launches after the GPU sat idle, to tell
whether a short timed region (the driver's --steps 20) starts on a GPU that
is still ramping.  Diagnostic only.

usage: python tools/ramp.py [pause_s] [launches]
"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def main():
    pause = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    launches = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    n, size = 4096, 65536
    wire, fs, _ = wl.c2_wire(n, size, seed=1)
    ws = [torch.from_numpy(wire).cuda(), torch.from_numpy(wl.c2_wire(n, size, seed=2)[0]).cuda()]
    outs = [torch.empty_like(ws[0]) for _ in ws]
    f = torch.from_numpy(fs.view(np.int64)).cuda()
    info = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    c = ca.Codec(0)
    for i in range(4):
        c.decode_batch(ws[i & 1], f, out=outs[i & 1], info=info)
    c.sync()
    for trial in range(3):
        time.sleep(pause)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(launches + 1)]
        ev[0].record()
        for i in range(launches):
            c.decode_batch(ws[i & 1], f, out=outs[i & 1], info=info)
            ev[i + 1].record()
        torch.cuda.synchronize()
        us = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(launches)]
        print("pause %.1fs trial %d: first 10 %s" % (pause, trial, " ".join("%.1f" % x for x in us[:10])))
        for a, b in ((0, 5), (5, 25), (25, 45), (45, launches)):
            seg = us[a:b]
            if seg:
                print("  launches %2d-%2d avg %.2f us" % (a, b - 1, sum(seg) / len(seg)))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
