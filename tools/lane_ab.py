"""Per-call time of the small host batches of the C1 echo (1000 masked
frames of 32-byte payloads, page-locked buffers: the replies' encode and the
reads' decode), through the host lane and through the launch path
($WSG_LANE_MAX=0), and through timing-only lane builds (tools/build_variant.sh:
lane_d1 answers without the work, lane_d2 does the per-frame phase only).
Median of many calls, microseconds.  Prints one JSON line.  Diagnostic only.
usage: python tools/lane_ab.py [FRAMES=1000] [SIZE=32] [CALLS=3000]"""
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

VAR = os.path.join(ROOT, "cppserver_amd", "_build", "var")


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


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    size = int(sys.argv[2]) if len(sys.argv) > 2 else 32
    calls = int(sys.argv[3]) if len(sys.argv) > 3 else 3000
    import torch

    assert torch.cuda.is_available()   # torch's HIP init before the library's first host allocation
    rng = np.random.default_rng(1)
    desc, total = wl.ragged_desc(rng, np.full(n, size))
    pay = ca.pinned_empty(total)
    pay[:] = wl.random_bytes(rng, total)
    fsz = int(ca.frame_sizes(desc).sum())
    wire = ca.pinned_empty(fsz)
    out = ca.pinned_empty(fsz)
    variants = {"lane": (None, {}), "launch": (None, {"WSG_LANE_MAX": "0"})}
    for v in ("lane_d1", "lane_d2"):
        if os.path.exists(os.path.join(VAR, v, "libwsg.so")):
            variants[v] = (os.path.join(VAR, v, "libwsg.so"), {})
    res = {"frames": n, "payload": size, "wire_bytes": fsz, "calls": calls}
    for name, (lib, env) in variants.items():
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        c = ca.Codec(0, lib_path=lib)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        rc, w, off = c.encode_batch_host(pay, desc, wire=wire)
        assert rc == 0
        fs = off[:-1].copy()
        enc = timed(lambda: c.encode_batch_host(pay, desc, wire=wire), calls)
        dec = timed(lambda: c.decode_batch_host(wire, fs, out=out), calls)
        res[name] = {"encode_us_median_p90": enc, "decode_us_median_p90": dec}
        c.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
