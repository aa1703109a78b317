"""Per-call time of host batches (by default the C1 echo's: 1000 masked
frames of 32-byte payloads, page-locked buffers: the replies' encode and the
reads' decode), through the host lane and through the launch path
($WSG_LANE_MAX=0).
Median of many calls, microseconds.  Prints one JSON line per batch shape.
Diagnostic only.
usage: python tools/lane_ab.py [FRAMES=1000] [SIZE=32] [CALLS=3000]
       python tools/lane_ab.py sweep [CALLS=1000]   (echo-sized to 2 MiB batches)"""
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402



def timed(fn, calls):
    for _ in range(200):
        fn()
    v = []
    for _ in range(calls):
        t = time.perf_counter()
        fn()
        v.append((time.perf_counter() - t) * 1e6)
    v.sort()
    return round(statistics.median(v), 2), round(v[int(len(v) * 0.9)], 2)


SWEEP = [(1000, 32), (1700, 33), (4000, 32), (8000, 32), (16000, 32), (30000, 32), (60, 16000), (120, 8000),
         (250, 8000), (500, 2000), (1000, 1000), (1900, 1000)]


def main():
    """usage: lane_ab.py [FRAMES [SIZE [CALLS]]] | lane_ab.py sweep [CALLS]:
    the lane (default $WSG_LANE_MAX) against the launch path per batch shape"""
    import torch

    assert torch.cuda.is_available()   # torch's HIP init before the library's first host allocation
    if len(sys.argv) > 1 and sys.argv[1] == "sweep":
        calls = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
        shapes = SWEEP
    else:
        n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
        size = int(sys.argv[2]) if len(sys.argv) > 2 else 32
        calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
        shapes = [(n, size)]
    rng = np.random.default_rng(1)
    codecs = {}
    for name, env in (("lane", {}), ("launch", {"WSG_LANE_MAX": "0"})):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        codecs[name] = ca.Codec(0)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for n, size in shapes:
        desc, total = wl.ragged_desc(rng, np.full(n, size))
        pay = ca.pinned_empty(total)
        pay[:] = wl.random_bytes(rng, total)
        fsz = int(ca.frame_sizes(desc).sum())
        wire = ca.pinned_empty(fsz)
        out = ca.pinned_empty(fsz)
        res = {"frames": n, "payload": size, "wire_bytes": fsz, "calls": calls}
        for name, c in codecs.items():
            r0, _, _ = c.lane_stats()
            rc, w, off = c.encode_batch_host(pay, desc, wire=wire)
            assert rc == 0
            fs = off[:-1].copy()
            enc = timed(lambda: c.encode_batch_host(pay, desc, wire=wire), calls)
            dec = timed(lambda: c.decode_batch_host(wire, fs, out=out), calls)
            r1, _, _ = c.lane_stats()
            res[name] = {"encode_us_median_p90": enc, "decode_us_median_p90": dec, "lane_requests": r1 - r0}
        print(json.dumps(res), flush=True)
    for c in codecs.values():
        c.close()


if __name__ == "__main__":
    main()
