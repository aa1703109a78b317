"""One case of test_gpu_lane.py::test_lane_timeout_waits_for_the_lane, in a
process of its own (the lane given up is the process's, for good).  The
environment holds the lane back ($WSG_TEST_LANE_DELAY_US) longer than a
request may wait ($WSG_LANE_TIMEOUT_MS):

* drained: the lane leaves within $WSG_LANE_DRAIN_MS, so the call decodes on
  the launch path and returns the oracle's bytes; nothing is written into the
  buffers after it returned (the late lane saw `stop` and did not take the
  request); the next batch in the same buffers (launch path) is exact too;
* lost: the lane does not leave in time: the call fails (WSG_EHIP) without
  the buffers being touched — not by the launch path, and not by the late
  lane once it runs — and the context refuses further calls.

Prints one JSON line {"ok": bool, ...}."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import cppserver_amd as ca  # noqa: E402
import oracle  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402

WSG_EHIP = -5


def batch(seed):
    rng = np.random.default_rng(seed)
    desc, total = wl.ragged_desc(rng, rng.integers(0, 200, 300))
    desc["mask"] = True
    payload = wl.random_bytes(rng, total + 16)
    wire, off = oracle.encode_batch(payload, desc)
    return wire, off[:-1].copy()


def main():
    case = sys.argv[1]
    res = {"case": case}
    c = ca.Codec(0)
    wire, fs = batch(1)
    rc_o, out_o, info_o = oracle.decode_batch(wire, fs)
    pin_in, pin_out = ca.pinned_empty(len(wire)), ca.pinned_empty(len(wire))
    pin_in[:] = wire
    pin_out[:] = 0xEE
    t0 = time.perf_counter()
    rc, out, info = c.decode_batch_host(pin_in, fs, out=pin_out)
    res["call_s"] = round(time.perf_counter() - t0, 3)
    res["rc"] = rc
    res["running"] = c.lane_stats()[2]
    if case == "drained":
        first = rc == rc_o and np.array_equal(out, out_o) and np.array_equal(info["key"], info_o["key"])
        snap = np.array(pin_out)
        time.sleep(1.0)   # the late lane has long run by now
        untouched_after = np.array_equal(np.array(pin_out), snap)
        wire2, fs2 = batch(2)
        rc2_o, out2_o, _ = oracle.decode_batch(wire2, fs2)
        pin_in[: len(wire2)] = wire2
        rc2, out2, _ = c.decode_batch_host(pin_in[: len(wire2)], fs2, out=pin_out)
        second = rc2 == rc2_o and np.array_equal(out2, out2_o)
        res.update(first=first, untouched_after=untouched_after, second=second)
        res["ok"] = bool(first and untouched_after and second and res["running"] == -1)
    else:
        time.sleep(1.5)   # the late lane starts (0.9 s) and must leave without the request
        untouched = bool(np.all(np.array(pin_out) == 0xEE))
        rc2, _, _ = c.decode_batch_host(pin_in, fs, out=pin_out)
        res.update(untouched=untouched, rc_after=rc2)
        res["ok"] = bool(rc == WSG_EHIP and untouched and rc2 == WSG_EHIP)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
