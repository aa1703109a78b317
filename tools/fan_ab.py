"""Fan-out library variants A/B (round 5; built by tools/build_variant.sh),
each checked against the oracle first (C4, the 16-message tick, other frame
geometries), then timed interleaved over rounds:

* c4_us: one C4 fan-out (4 KiB x 10000 keys) per launch, K launches captured
  in a graph and replayed (as bench.py's graph_replay leg);
* tick_us: 16 x C4 in one wsg_fanout_encode_many call, back to back (as
  bench.py's multicast_tick_16), with the runtime's fill of the same bytes.

Used for profiles/r5/fan_run_ab.log (a run kernel, since removed: each wave
writing U consecutive rows with per-chunk L2 loads, 17-22 us per C4), and
fan_cap_ab.log (the period kernel's workgroups per CU capped).

usage: python tools/fan_ab.py NAME=path/to/libwsg.so ...   ($K, $ROUNDS, $M: messages per tick, 16)
(one variant per process: each library's initial-exec TLS)"""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
import oracle  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def parity(c):
    rng = np.random.default_rng(5)
    bad = []
    for length, k, op in ((4096, 10000, 0x82), (4092, 7, 0x82), (4088, 5, 0x81), (122, 1000, 0x82), (58, 33, 0x82),
                          (8190, 130, 0x89), (65538, 40, 0x82), (9, 50, 0x82), (10, 3000, 0x82), (1000, 777, 0x8A)):
        for mask in (True, False):
            m = 3
            keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
            lens = np.full(m, length)
            ops = np.full(m, op)
            src = np.zeros(m, np.uint64)
            src[1:] = np.cumsum(lens[:-1] + 5)
            arena = wl.random_bytes(rng, int(src[-1] + lens[-1] + 16))
            wire, off = c.fanout_many(torch.from_numpy(arena).cuda(), src, lens, ops,
                                      torch.from_numpy(keys.view(np.int32)).cuda(), mask=mask)
            c.sync()
            got = wire.cpu().numpy()
            for i in range(m):
                ref = oracle.fanout_encode(arena[int(src[i]): int(src[i]) + length], keys, op, mask)
                a = int(off[i])
                if not np.array_equal(got[a: a + len(ref)], ref):
                    bad.append((length, k, op, mask, i))
    return bad


def main():
    specs = [a.split("=", 1) for a in sys.argv[1:]]
    K = int(os.environ.get("K", 200))
    rounds = int(os.environ.get("ROUNDS", 3))
    payload, keys = wl.c4_fanout(4096, 10000)
    fsz = ca.frame_size(0x82, True, len(payload))
    p = torch.from_numpy(payload).cuda()
    kt = torch.from_numpy(keys.view(np.int32)).cuda()
    m = int(os.environ.get("M", 16))
    arena = torch.from_numpy(np.random.default_rng(99).integers(0, 256, m * 4096, dtype=np.uint8)).cuda()
    src = np.arange(m, dtype=np.uint64) * np.uint64(4096)
    lens = np.full(m, 4096, dtype=np.uint64)
    ops = np.full(m, 0x82, dtype=np.uint8)
    var = []
    for name, path in specs:
        c = ca.Codec(0, lib_path=path)
        bad = parity(c)
        w = torch.empty(fsz * len(keys), dtype=torch.uint8, device="cuda")
        launch = c.prepare_fanout(p, kt, 0x82, True, w)
        launch()
        torch.cuda.synchronize()
        ref = oracle.fanout_encode(payload, keys, 0x82, True)
        c4_ok = bool(np.array_equal(w.cpu().numpy(), ref))
        st = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            launch()
            st.synchronize()
            with torch.cuda.graph(g, stream=st):
                for _ in range(K):
                    launch()
        wire, off = c.fanout_many(arena, src, lens, ops, kt)
        c.sync()
        var.append(dict(name=name, c=c, g=g, wire=wire, bad=bad, c4_ok=c4_ok, c4=[], tick=[], fill=[]))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(rounds):
        for v in var:
            v["g"].replay()
            torch.cuda.synchronize()
            e0.record()
            v["g"].replay()
            e1.record()
            e1.synchronize()
            v["c4"].append(e0.elapsed_time(e1) * 1e3 / K)
            c = v["c"]
            for _ in range(2):
                c.fanout_many(arena, src, lens, ops, kt, wire=v["wire"])
            e0.record()
            for _ in range(10):
                c.fanout_many(arena, src, lens, ops, kt, wire=v["wire"])
            e1.record()
            e1.synchronize()
            v["tick"].append(e0.elapsed_time(e1) * 1e3 / 10)
            e0.record()
            for _ in range(10):
                v["wire"].zero_()
            e1.record()
            e1.synchronize()
            v["fill"].append(e0.elapsed_time(e1) * 1e3 / 10)
    for v in var:
        c4 = statistics.median(v["c4"])
        tick = statistics.median(v["tick"])
        fill = statistics.median(v["fill"])
        print(json.dumps({"variant": v["name"], "m": m, "parity_bad": v["bad"][:5], "c4_ok": v["c4_ok"],
                          "c4_us": round(c4, 3), "c4_frac": round(41040000 / (c4 * 1e-6) / 8e12, 4),
                          "tick_us": round(tick, 2), "fill_us": round(fill, 2), "tick_vs_fill": round(fill / tick, 4),
                          "c4_all": [round(x, 3) for x in v["c4"]], "tick_all": [round(x, 1) for x in v["tick"]]}),
              flush=True)


if __name__ == "__main__":
    main()
