"""Host-staged C2 decode (wsg_decode_batch_host) from pageable and from
page-locked buffers, and the encode from pageable payloads, for one library
build (round 5: the parallel staging copies, WSG_COPY_WORKERS builds from
tools/build_variant.sh).  Prints one JSON line of payload GiB/s.

usage: python tools/pcie_pageable.py [path/to/libwsg.so] ($REPS)"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
import oracle  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402

GIB = float(1 << 30)


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else None
    reps = int(os.environ.get("REPS", 5))
    c = ca.Codec(0, lib_path=lib)
    wire, fs, _ = wl.c2_wire(4096, 65536, seed=3)
    payload = 4096 * 65536
    rc_o, out_o, _ = oracle.decode_batch(wire[: 64 * 65550], fs[:64])
    res = {"lib": lib or "in-tree"}
    pin_in, pin_out = ca.pinned_empty(len(wire)), ca.pinned_empty(len(wire))
    pin_in[:] = wire
    for name, src, dst in (("pinned", pin_in, pin_out), ("pageable", wire, np.empty_like(wire))):
        rc, out, _ = c.decode_batch_host(src, fs, out=dst)
        assert rc == 0 and np.array_equal(out[: 64 * 65550], out_o), name
        t0 = time.perf_counter()
        for _ in range(reps):
            c.decode_batch_host(src, fs, out=dst)
        res[name] = round(payload / ((time.perf_counter() - t0) / reps) / GIB, 2)
    rng = np.random.default_rng(7)
    desc, total = wl.ragged_desc(rng, np.full(4096, 65536))
    pay = wl.random_bytes(rng, total)
    rc, w, off = c.encode_batch_host(pay, desc)
    assert rc == 0
    t0 = time.perf_counter()
    for _ in range(reps):
        c.encode_batch_host(pay, desc, wire=w)
    res["encode_pageable"] = round(total / ((time.perf_counter() - t0) / reps) / GIB, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
