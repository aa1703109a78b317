"""Interleaved A/B timing of encode variants (libwsg.so builds) on C5/C3-like batches.

usage: CFG=c5|c3|c4 python tools/tune_enc.py [NAME=VALUE@]path/to/libwsg.so ...
(NAME=VALUE is set in the environment before that library's context is made)
"""
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def make_codec(spec):
    if spec and "@" in spec:
        env, _, spec = spec.partition("@")
        name, _, value = env.partition("=")
        os.environ[name] = value
    return ca.Codec(0, lib_path=spec or None)


def main():
    libs = sys.argv[1:] or [None]
    cfg = os.environ.get("CFG", "c5")
    if cfg == "c4":
        return fanout(libs)
    if cfg == "c5":
        payload, desc, _ = wl.c5_shard(0, 8, n_total=1 << 20)      # one rank's share of 8: 131072 x 16 KiB
    else:   # $FRAMES frames, payload uniform in [$LO, $HI] (default: C3-like)
        payload, desc = wl.c3_batch(int(os.environ.get("FRAMES", 16384)), int(os.environ.get("LO", 128)),
                                    int(os.environ.get("HI", 65536)), seed=3)
    cap = int(np.sum([ca.frame_size(0x82, True, int(x)) for x in desc["len"]]))
    n = len(desc)
    p = [torch.from_numpy(payload).cuda() for _ in range(2)]
    d = ca.desc_to_tensor(desc, "cuda")
    wires = [torch.empty(cap, dtype=torch.uint8, device="cuda") for _ in range(2)]
    woff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
    codecs = [make_codec(l) for l in libs]
    kern = [[] for _ in libs]
    step = [[] for _ in libs]   # whole wsg_encode_batch (scan included), 32 calls back to back, wall clock
    for rep in range(int(os.environ.get("REPS", 5))):
        for ci, c in enumerate(codecs):
            for it in range(3):
                c.encode_batch(p[it & 1], d, wire=wires[it & 1], wire_cap=cap, wire_off=woff)
            c.timing(True, 1)
            c.timing_read()
            for it in range(8):
                c.encode_batch(p[it & 1], d, wire=wires[it & 1], wire_cap=cap, wire_off=woff)
            ms, k = c.timing_read()
            c.timing(False)
            kern[ci].append(ms / k)
            c.sync()
            t0 = time.perf_counter()
            for it in range(32):
                c.encode_batch(p[it & 1], d, wire=wires[it & 1], wire_cap=cap, wire_off=woff)
            c.sync()
            step[ci].append((time.perf_counter() - t0) / 32 * 1e3)
    alg = len(payload) + cap
    for l, k, st in zip(libs, kern, step):
        m = statistics.median(k)
        print("%-50s encode kernel %.4f ms  %.0f GB/s  spread %.1f%%  | whole call %.4f ms" % (
            l, m, alg / m / 1e6, 100 * (max(k) - min(k)) / m, statistics.median(st)))


def fanout(libs):
    payload, keys = wl.c4_fanout(int(os.environ.get("LEN", 4096)), int(os.environ.get("KEYS", 10000)))
    fsz = ca.frame_size(0x82, True, len(payload))
    p = torch.from_numpy(payload).cuda()
    kt = torch.from_numpy(keys.view(np.int32)).cuda()
    wires = [torch.empty(fsz * len(keys), dtype=torch.uint8, device="cuda") for _ in range(2)]
    codecs = [make_codec(l) for l in libs]
    kern = [[] for _ in libs]
    for rep in range(int(os.environ.get("REPS", 5))):
        for ci, c in enumerate(codecs):
            for it in range(3):
                c.fanout(p, kt, 0x82, True, wire=wires[it & 1])
            c.timing(True, 1)
            c.timing_read()
            for it in range(20):
                c.fanout(p, kt, 0x82, True, wire=wires[it & 1])
            ms, k = c.timing_read()
            c.timing(False)
            kern[ci].append(ms / k)
    alg = len(payload) + 4 * len(keys) + fsz * len(keys)
    for l, k in zip(libs, kern):
        m = statistics.median(k)
        print("%-50s fanout kernel %.4f ms  %.0f GB/s  spread %.1f%%" % (l, m, alg / m / 1e6,
                                                                       100 * (max(k) - min(k)) / m))


if __name__ == "__main__":
    main()
