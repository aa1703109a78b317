"""A/B of the host-staged pipelines ($WSG_PIPE=slots vs the role streams) on
C2's wire (decode) and a C5-like batch (encode), pinned and pageable host
buffers.  Prints payload GiB/s per variant (best of REPS)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402

GIB = float(1 << 30)


def best(fn, reps):
    fn()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        t.append(time.perf_counter() - t0)
    return min(t)


def main():
    reps = int(os.environ.get("REPS", 5))
    codec = ca.Codec(0)
    wire, fs, _ = wl.c2_wire()
    payload_bytes = 4096 * 65536
    pin_in = ca.pinned_empty(len(wire))
    pin_in[:] = wire
    pin_out = ca.pinned_empty(len(wire))
    pag_out = np.empty_like(wire)
    pay, desc, _ = wl.c5_shard(0, 64, n_total=1 << 20)   # 16384 x 16 KiB = 256 MiB
    cap = int(np.sum([ca.frame_size(0x82, True, int(x)) for x in desc["len"]]))
    pin_pay = ca.pinned_empty(len(pay))
    pin_pay[:] = pay
    pin_wire = ca.pinned_empty(cap)
    pag_wire = np.empty(cap, np.uint8)
    for mb in os.environ.get("STAGE_MB", "32").split(","):
        os.environ["WSG_STAGE_MB"] = mb
        for pipe in ("slots", "roles"):
            os.environ["WSG_PIPE"] = pipe
            r = {}
            r["dec_pinned"] = payload_bytes / best(lambda: codec.decode_batch_host(pin_in, fs, out=pin_out), reps) / GIB
            r["dec_pageable"] = payload_bytes / best(lambda: codec.decode_batch_host(wire, fs, out=pag_out), reps) / GIB
            r["enc_pinned"] = len(pay) / best(lambda: codec.encode_batch_host(pin_pay, desc, wire=pin_wire), reps) / GIB
            r["enc_pageable"] = len(pay) / best(lambda: codec.encode_batch_host(pay, desc, wire=pag_wire), reps) / GIB
            print("stage=%sMiB pipe=%-5s " % (mb, pipe) + "  ".join("%s %.1f" % kv for kv in r.items()), flush=True)
    rc, out, _ = codec.decode_batch_host(pin_in, fs, out=pin_out)
    assert rc == 0


if __name__ == "__main__":
    main()
