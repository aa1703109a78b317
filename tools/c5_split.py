"""C5 encode split into sub-batches (round 3): the whole 1 Mi x 16 KiB job in
one wsg_encode_batch call against the same job as k calls over consecutive
frame slices (same buffers, same bytes out), and single slices at the start
and at the end of the buffers.  Tells whether the whole job's lower rate
comes from the buffers' size (placement, translation) or from one launch
covering it.  Kernel times: the library's HIP events around k_encode_mask.
Diagnostic only.

usage: python tools/c5_split.py
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
    c = ca.Codec(0)
    size = 16384
    n = 1 << 20
    fsz = ca.frame_size(0x82, True, size)
    ids = np.arange(n, dtype=np.int64)
    payload = wl.c5_payload_torch(ids, size, device="cuda")
    desc_np = wl.c5_desc(ids, size)
    desc = ca.desc_to_tensor(desc_np, "cuda")
    wire = torch.empty(n * fsz, dtype=torch.uint8, device="cuda")
    woff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    D = ca.SEND_DESC.itemsize

    def run(slices):
        """Encode the frame ranges `slices` back to back; kernel ms summed."""
        for a, b in slices:
            c.encode_batch(payload, desc[a * D: b * D], wire=wire[a * fsz:], wire_cap=(b - a) * fsz,
                           wire_off=woff[a:])
        c.sync()
        c.timing(True, 1)
        c.timing_read()
        reps = 4
        for _ in range(reps):
            for a, b in slices:
                c.encode_batch(payload, desc[a * D: b * D], wire=wire[a * fsz:], wire_cap=(b - a) * fsz,
                               wire_off=woff[a:])
        ms, k = c.timing_read()
        c.timing(False)
        return ms / reps

    cases = [("whole job, 1 call", [(0, n)]),
             ("8 calls of 1/8", [(i * n // 8, (i + 1) * n // 8) for i in range(8)]),
             ("2 calls of 1/2", [(0, n // 2), (n // 2, n)]),
             ("32 calls of 1/32", [(i * n // 32, (i + 1) * n // 32) for i in range(32)]),
             ("first 1/8 only", [(0, n // 8)]),
             ("last 1/8 only", [(7 * n // 8, n)])]
    res = {name: [] for name, _ in cases}
    for rep in range(3):
        for name, sl in cases:
            res[name].append(run(sl))
    for name, sl in cases:
        frames = sum(b - a for a, b in sl)
        m = statistics.median(res[name])
        alg = frames * (size + fsz)
        print("%-20s frames=%7d  k_encode_mask total %.4f ms  %.0f GB/s  frac %.3f" % (
            name, frames, m, alg / m / 1e6, alg / m / 8e6), flush=True)
    c.close()


if __name__ == "__main__":
    main()
