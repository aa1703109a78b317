"""C2 decode: eager Python-driven steps vs the same steps captured in one HIP
graph vs the C++ loop of tools/decbench (interleaved, one box).  Tells how
much of bench.py's per-step time is the Python launch path.

usage: python tools/graph_ab.py [reps]
"""
import os
import statistics
import subprocess
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    n, size, steps = 4096, 65536, 200
    wire, fs, _ = wl.c2_wire(n, size, seed=1)
    ws = [torch.from_numpy(wire).cuda(), torch.from_numpy(wl.c2_wire(n, size, seed=2)[0]).cuda()]
    outs = [torch.empty_like(ws[0]) for _ in ws]
    f = torch.from_numpy(fs.view(np.int64)).cuda()
    info = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    c = ca.Codec(0)
    for i in range(4):
        c.decode_batch(ws[i & 1], f, out=outs[i & 1], info=info)
    c.sync()
    s = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for i in range(steps):
            c.decode_batch(ws[i & 1], f, out=outs[i & 1], info=info)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = {"eager": [], "graph": []}
    for _ in range(reps):
        torch.cuda.synchronize()
        e0.record()
        for i in range(steps):
            c.decode_batch(ws[i & 1], f, out=outs[i & 1], info=info)
        e1.record()
        e1.synchronize()
        res["eager"].append(e0.elapsed_time(e1) * 1e3 / steps)
        torch.cuda.synchronize()
        e0.record()
        g.replay()
        e1.record()
        e1.synchronize()
        res["graph"].append(e0.elapsed_time(e1) * 1e3 / steps)
    c.sync()
    alg = 2 * len(wire) + n * 40
    for k, v in res.items():
        m = statistics.median(v)
        print("%-6s %d steps: %.2f us per step (median of %d), %.1f GB/s, frac %.4f" % (
            k, steps, m, reps, alg / m / 1e3, alg / m / 1e3 / 8000))
    exe = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "decbench")
    if os.path.exists(exe):
        r = subprocess.run([exe, str(n), str(size)], capture_output=True, text=True, timeout=120)
        print("\n".join(x for x in r.stdout.splitlines() if "libwsg" in x or x.startswith("bare copy (")))


if __name__ == "__main__":
    main()
