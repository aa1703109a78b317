"""ws_multicast's tick as one wsg_fanout_encode_many call (16 x C4: 4 KiB
messages x 10000 client keys, 656 MB of frames) under launch-shape variants
(VERDICT r3 item 5), interleaved: waves per CU per message
($WSG_FAN_WAVES_PER_CU) and waves per workgroup ($WSG_FAN_WPB); beside them
the bare write stream of the same bytes (hipMemsetAsync through torch's
zero_) and the single C4 launch.  HIP events around back-to-back calls.
Prints one JSON line.  Diagnostic only.

usage: python tools/fan_many_ab.py ["WSG_FAN_WAVES_PER_CU=4,WSG_FAN_WPB=4" ...]
"""
import json
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402

KNOBS = ("WSG_FAN_WAVES_PER_CU", "WSG_FAN_WPB")


VAR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cppserver_amd", "_build", "var")


def make(spec):
    """spec: "NAME=V,..." environment knobs, or "lib:<variant>" (a build of
    tools/build_variant.sh under cppserver_amd/_build/var)."""
    lib = None
    for k in KNOBS:
        os.environ.pop(k, None)
    for kv in filter(None, spec.split(",")):
        if kv.startswith("lib:"):
            lib = os.path.join(VAR, kv[4:], "libwsg.so")
            continue
        k, _, v = kv.partition("=")
        os.environ[k] = v
    c = ca.Codec(0, lib_path=lib)
    for k in KNOBS:
        os.environ.pop(k, None)
    return c


def timed(fn, reps=10, rounds=7):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(rounds):
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        e1.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / reps)
    return statistics.median(out)


def main():
    specs = sys.argv[1:] or ["", "WSG_FAN_WAVES_PER_CU=4", "WSG_FAN_WAVES_PER_CU=3", "WSG_FAN_WAVES_PER_CU=2",
                             "WSG_FAN_WAVES_PER_CU=1", "WSG_FAN_WPB=4", "WSG_FAN_WAVES_PER_CU=2,WSG_FAN_WPB=4",
                             "WSG_FAN_WAVES_PER_CU=8,WSG_FAN_WPB=8"]
    m, length, k = 16, 4096, 10000
    rng = np.random.default_rng(99)
    arena = torch.from_numpy(rng.integers(0, 256, m * length, dtype=np.uint8)).cuda()
    keys = torch.from_numpy(rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32).view(np.int32)).cuda()
    src = np.arange(m, dtype=np.uint64) * np.uint64(length)
    lens = np.full(m, length, dtype=np.uint64)
    ops = np.full(m, 0x82, dtype=np.uint8)
    fsz = ca.frame_size(0x82, True, length)
    per_msg = m and (fsz * k + length + 4 * k)
    codecs = [make(s) for s in specs]
    wire, off = codecs[0].fanout_many(arena, src, lens, ops, keys)
    one = torch.empty(fsz * k, dtype=torch.uint8, device="cuda")
    bytes_out = m * k * fsz
    fill = wire[:bytes_out]
    res = {"messages": m, "frame_bytes": fsz, "bytes_out": bytes_out, "variants": {}}
    for _ in range(20):   # clocks up
        codecs[0].fanout_many(arena, src, lens, ops, keys, wire=wire)
    torch.cuda.synchronize()
    per = {s: [] for s in specs}
    fills = []
    for rnd in range(3):
        fills.append(timed(lambda: fill.zero_()))
        for s, c in zip(specs, codecs):
            per[s].append(timed(lambda: c.fanout_many(arena, src, lens, ops, keys, wire=wire)))
    res["bare_write_us"] = round(statistics.median(fills), 2)
    res["bare_write_TBps"] = round(bytes_out / (statistics.median(fills) * 1e-6) / 1e12, 3)
    for s, c in zip(specs, codecs):
        us = statistics.median(per[s])
        res["variants"][s or "default"] = {
            "us_per_call": round(us, 2), "write_TBps": round(bytes_out / (us * 1e-6) / 1e12, 3),
            "frac": round(m * per_msg / (us * 1e-6) / 8e12, 4),
            "vs_bare_write": round(res["bare_write_us"] / us, 4),
            "single_c4_us": round(timed(lambda: c.fanout(arena[:length], keys, 0x82, True, wire=one), reps=50), 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
