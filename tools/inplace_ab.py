"""k_decode on the C2 batch out of place (wire -> out, the bench's headline
step) against in place (out = wire: a server unmasking its receive arena
where it lies; decoding twice restores the masked wire, so every launch
has valid input), two batches alternating as in bench.py, HIP events per
region of K launches, interleaved trials.  Diagnostic only.

usage: python tools/inplace_ab.py [trials] [K]
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    n, size = 4096, 65536
    wires = [torch.from_numpy(wl.c2_wire(n, size, seed=s)[0]).cuda() for s in (1, 2)]
    fs = torch.from_numpy(wl.c2_wire(n, size, seed=1)[1].view(np.int64)).cuda()
    outs = [torch.empty_like(w) for w in wires]
    info = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    c = ca.Codec(0)
    variants = {
        "out_of_place": [c.prepare_decode(wires[i], fs, outs[i], info) for i in range(2)],
        "in_place": [c.prepare_decode(wires[i], fs, wires[i], info) for i in range(2)],
    }
    alg = 2 * wires[0].numel() + n * 40
    res = {v: [] for v in variants}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(trials):
        for v, launch in variants.items():
            for i in range(20):
                launch[i & 1]()
            torch.cuda.synchronize()
            e0.record()
            for i in range(k):
                launch[i & 1]()
            e1.record()
            e1.synchronize()
            res[v].append(e0.elapsed_time(e1) * 1e3 / k)
    # the in-place pair decoded an even number of times per batch: masked again
    ref = wl.c2_wire(n, size, seed=1)[0]
    ok = bool(np.array_equal(wires[0].cpu().numpy(), ref))
    for v, xs in res.items():
        med = statistics.median(xs)
        print("%-13s k_decode %.2f us per launch (median of %d regions of %d)  %.0f GB/s  frac %.4f  [%s]"
              % (v, med, trials, k, alg / med / 1e3, alg / med / 1e3 / 8000, " ".join("%.2f" % x for x in xs)),
              flush=True)
    print("in-place wire restored after an even number of decodes:", ok, flush=True)
    c.close()


if __name__ == "__main__":
    main()
