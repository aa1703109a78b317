"""Echo-sized frames (32 B payload, 38 B masked frames) on the
device batch paths: N frames encoded with wsg_encode_batch and the wire
decoded with wsg_decode_batch, REPS times each, round trip checked.  For
rocprofv3 kernel traces of the small-frame kernels (profiles/).

usage: FRAMES=1048576 SIZE=32 REPS=20 python tools/echo_size.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def main():
    n = int(os.environ.get("FRAMES", 1 << 20))
    size = int(os.environ.get("SIZE", 32))
    reps = int(os.environ.get("REPS", 20))
    c = ca.Codec(0)
    payload, desc = wl.c3_batch(n, size, size, seed=77)
    p = torch.from_numpy(payload).cuda()
    d = ca.desc_to_tensor(desc, "cuda")
    cap = n * ca.frame_size(0x82, True, size)
    wire = torch.empty(cap, dtype=torch.uint8, device="cuda")
    woff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    out = torch.empty_like(wire)
    info = torch.empty(n * ca.RECV_INFO.itemsize, dtype=torch.uint8, device="cuda")
    res = {}
    for name, fn in (("encode", lambda: c.encode_batch(p, d, wire=wire, wire_cap=cap, wire_off=woff)),
                     ("decode", lambda: c.decode_batch(wire, woff[:-1], out=out, info=info))):
        for _ in range(3):
            fn()
        c.sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        c.sync()
        res[name] = (time.perf_counter() - t0) / reps * 1e6
    hdr = ca.frame_size(0x82, True, size) - size
    o = out.view(n, hdr + size)[:, hdr:].reshape(-1)
    ok = bool(torch.equal(o, p[: n * size]))
    print("frames=%d size=%d encode %.1f us  decode %.1f us  round trip %s" % (n, size, res["encode"], res["decode"],
                                                                              "ok" if ok else "MISMATCH"))
    c.close()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
