"""Host batch decode time per call for the status-pass shapes: many small
frames in place (page-locked, one k_decode launch) and staged (pageable,
the segmented pipeline), and C2's 4096 x 64 KiB staged, through the product
library or a variant (tools/build_variant.sh; e.g. one built from an older
wsg_capi.hip with $CSRC).  One library per process.  Diagnostic only.
usage: python tools/latch_ab.py [LIB] [CALLS=20]   (prints one JSON line)"""
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


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "-" else None
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    import torch

    assert torch.cuda.is_available()
    rng = np.random.default_rng(2)
    c = ca.Codec(0, lib_path=lib)
    res = {"lib": lib or "product", "calls": calls}
    for name, n, size, pinned in (("inplace_100k_x32", 100000, 32, True), ("staged_1m_x32", 1 << 20, 32, False),
                                  ("staged_c2_4096_x64k", 4096, 65536, False)):
        desc, total = wl.ragged_desc(rng, np.full(n, size))
        desc["mask"] = True
        desc["key"] = rng.integers(1, 2**32, n, dtype=np.uint64).astype(np.uint32)
        pay = wl.random_bytes(rng, total)
        rc, wire, off = c.encode_batch_host(pay, desc)
        assert rc == 0
        fs = off[:-1].copy()
        if pinned:
            w = ca.pinned_empty(len(wire))
            w[:] = wire
            out = ca.pinned_empty(len(wire))
        else:
            w = np.array(wire)
            out = np.empty_like(w)
        v = []
        for i in range(calls + 3):
            t = time.perf_counter()
            rc, o, info = c.decode_batch_host(w, fs, out=out)
            dt = (time.perf_counter() - t) * 1e6
            assert rc == 0
            if i >= 3:
                v.append(dt)
        res[name] = {"us_median": round(statistics.median(v), 1), "us_min": round(min(v), 1),
                     "payload_GiBps": round(n * size / (statistics.median(v) * 1e-6) / 2**30, 2)}
    c.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
