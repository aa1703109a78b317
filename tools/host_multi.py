"""PCIe-inclusive C2 decode / encode (host buffers, pinned) through one
context vs several (wsg_*_batch_host_multi) on the GPUs given, payload
GiB/s.  With all contexts on one GPU it tells whether one host pipeline
leaves that GPU's link idle; over N GPUs it is the multi-link rate.

usage: python tools/host_multi.py [devices, e.g. 0,0 or 0,1,2,3] [reps]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def rate(fn, nbytes, reps):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        rc = fn()
        assert rc == 0, rc
    return round(nbytes * reps / (time.perf_counter() - t0) / 2**30, 2)


def main():
    devs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0,0").split(",")]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    codecs = [ca.Codec(d) for d in devs]   # first: torch's HIP runtime before any pinned allocation
    n, size = 4096 * max(1, len(set(devs))), 65536
    wire, fs, _ = wl.c2_wire(n, size, seed=1)
    pin_in, pin_out = ca.pinned_empty(len(wire)), ca.pinned_empty(len(wire))
    pin_in[:] = wire
    res = {"devices": devs, "workload": "%d x %d B masked frames, pinned host buffers" % (n, size)}
    for k in sorted({1, len(codecs)}):
        res["decode_%dctx_GiBps" % k] = rate(
            lambda: ca.decode_batch_host_multi(codecs[:k], pin_in, fs, out=pin_out)[0], n * size, reps)
    rng = np.random.default_rng(7)
    desc, total = wl.ragged_desc(rng, np.full(n, size))
    pay = ca.pinned_empty(total)
    pay[:] = wl.random_bytes(rng, total)
    out = ca.pinned_empty(int(ca.frame_sizes(desc).sum()))
    for k in sorted({1, len(codecs)}):
        res["encode_%dctx_GiBps" % k] = rate(
            lambda: ca.encode_batch_host_multi(codecs[:k], pay, desc, wire=out)[0], total, reps)
    print(json.dumps(res), flush=True)
    for c in codecs:
        c.close()


if __name__ == "__main__":
    main()
