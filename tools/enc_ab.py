"""Interleaved A/B of encode launch settings (round 3) on the whole C5 job,
a 1/8 share of it and the C3 batch: each variant is a context made with its
environment (WSG_ENC_BLOCKS_PER_CU, WSG_ENC_LAUNCH_PIECES, ...), every
variant runs on the same buffers in turn; k_encode_mask time from the
library's HIP events (all of a call's launches).  Diagnostic only.

usage: python tools/enc_ab.py "NAME=V[,NAME=V]" ...   ("" = defaults)
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402

KNOBS = ("WSG_ENC_BLOCKS_PER_CU", "WSG_ENC_LAUNCH_PIECES")


def make(spec):
    for k in KNOBS:
        os.environ.pop(k, None)
    for kv in filter(None, spec.split(",")):
        k, _, v = kv.partition("=")
        os.environ[k] = v
    c = ca.Codec(0)
    for k in KNOBS:
        os.environ.pop(k, None)
    return c


def batches():
    size = 16384
    for name, n in (("C5 whole job", 1 << 20), ("C5 1/8", 1 << 17)):
        ids = np.arange(n, dtype=np.int64)
        yield name, wl.c5_payload_torch(ids, size, device="cuda"), wl.c5_desc(ids, size)
    payload, desc = wl.c3_batch(65536, 128, 65536, seed=3000)
    yield "C3 65536 ragged", torch.from_numpy(payload).cuda(), desc


def main():
    specs = sys.argv[1:] or [""]
    codecs = [make(s) for s in specs]
    for name, payload, desc_np in batches():
        desc = ca.desc_to_tensor(desc_np, "cuda")
        cap = int(ca.frame_sizes(desc_np).sum())
        wire = torch.empty(cap, dtype=torch.uint8, device="cuda")
        woff = torch.empty(len(desc_np) + 1, dtype=torch.int64, device="cuda")
        alg = int(desc_np["len"].sum()) + cap
        reps = 3 if cap > (8 << 30) else 10
        # warm the clocks: ~0.1 s of encodes
        for _ in range(max(3, int(0.1 / (cap / 3e12)))):
            codecs[0].encode_batch(payload, desc, wire=wire, wire_cap=cap, wire_off=woff)
        res = [[] for _ in specs]
        for rep in range(5):
            for i, c in enumerate(codecs):
                c.encode_batch(payload, desc, wire=wire, wire_cap=cap, wire_off=woff)
                c.timing(True, 1)
                c.timing_read()
                for _ in range(reps):
                    c.encode_batch(payload, desc, wire=wire, wire_cap=cap, wire_off=woff)
                ms, k = c.timing_read()
                c.timing(False)
                res[i].append(ms / k)
        ok = int(woff[-1].item()) == cap
        for s, r in zip(specs, res):
            m = statistics.median(r)
            print("%-18s %-45s %.4f ms  %.0f GB/s  frac %.4f  spread %.1f%%  offsets_ok=%s" % (
                name, s or "(defaults)", m, alg / m / 1e6, alg / m / 8e9 * 1e3 / 1e3,
                100 * (max(r) - min(r)) / m, ok), flush=True)
        del payload, desc, wire, woff
        torch.cuda.empty_cache()
    for c in codecs:
        c.close()


if __name__ == "__main__":
    main()
