"""One case of test_gpu_lane.py::test_lane_timeout_waits_for_the_lane (or
test_lane_inline_answers_across_the_tag_wrap), in a process of its own (the
lane is the process's).  The environment holds the lane's first launch back
($WSG_TEST_LANE_DELAY_US, $WSG_TEST_LANE_DELAY_GENS) longer than a request
may wait ($WSG_LANE_TIMEOUT_MS):

* drained: the lane leaves within $WSG_LANE_DRAIN_MS, so the call decodes on
  the launch path and returns the oracle's bytes; nothing is written into the
  buffers after it returned (the late lane saw `stop` and did not take the
  request); then the lane comes back: the next batch in the same buffers and
  200 per-call XORs are lane requests of a new launch, all exact;
* lost: the lane does not leave in time: the call fails (WSG_EHIP) without
  the buffers being touched — not by the launch path, and not by the late
  lane once it runs — and the context refuses further calls.

* handover: the lane made to hand over constantly ($WSG_LANE_YIELD_US and
  $WSG_LANE_IDLE_US of tens of microseconds) while eight threads, each with
  its own context, decode, encode and XOR through it: every result exact,
  hundreds of launches, no request lost across a hand-over.

* churn: the same eight threads while every few launches of the lane start
  late ($WSG_TEST_LANE_DELAY_EVERY) past the request time-out: the lane is
  given up and brought back again and again (wsg_lane_events), requests in
  flight at each give-up are redone on the launch paths, tasks the old lane
  never took are skipped; every result exact, and the lane answers after.

* wrap: see wrap() below.

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


def xor_ref(data, key, phase):
    """ws.cpp:264-270 (and :402-403): byte i ^ key byte (phase + i) % 4."""
    kb = np.frombuffer(int(key).to_bytes(4, "little"), np.uint8)
    return np.frombuffer(bytes(data), np.uint8) ^ kb[(np.arange(len(data)) + phase) % 4]


def wrap(res):
    """Tickets from just below 2^32 ($WSG_TEST_LANE_TICKET_BASE) with every
    slot's inline answer units left as a task 2^32 tickets earlier would have
    left them ($WSG_TEST_LANE_STALE_XRES): per-call XORs of up to 40 bytes
    (answered inline) and larger ones, across the 2^32 mark and round the
    ring more than once — every result the request's own bytes."""
    c = ca.Codec(0)
    rng = np.random.default_rng(11)
    req0 = c.lane_stats()[0]
    bad = []
    n = 3000
    for i in range(n):
        ln = int(rng.integers(1, 41)) if i % 5 else int(rng.integers(41, 300))
        data = bytes(wl.random_bytes(rng, ln))
        key, phase = int(rng.integers(0, 2**32)), int(rng.integers(0, 4))
        got = np.frombuffer(c.xor_host(data, key, phase), np.uint8)
        if not np.array_equal(got, xor_ref(data, key, phase)):
            bad.append((i, ln))
    req1, launches, running = c.lane_stats()
    res.update(bad=bad[:10], n_bad=len(bad), requests=req1 - req0, launches=launches, running=running)
    res["ok"] = bool(not bad and req1 - req0 == n and running != -1)
    c.close()
    print(json.dumps(res))


def handover(res, churn=False):
    import threading

    import oracle as orc

    n_threads, rounds = 8, 40
    codecs = [ca.Codec(0) for _ in range(n_threads)]
    errors = []

    def work(i):
        try:
            c = codecs[i]
            rng = np.random.default_rng(700 + i)
            pin_p, pin_w = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
            pin_in, pin_out = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
            for it in range(rounds):
                desc, total = wl.ragged_desc(rng, rng.integers(0, 300, int(rng.integers(1, 1500))))
                desc["mask"] = rng.random(len(desc)) < 0.9
                payload = wl.random_bytes(rng, total + 16)
                wire_o, off_o = orc.encode_batch(payload, desc)
                if len(wire_o) > 60000:
                    continue
                pin_p[: len(payload)] = payload
                rc, wire, off = c.encode_batch_host(pin_p[: len(payload)], desc, wire=pin_w)
                if rc != 0 or not np.array_equal(wire, wire_o):
                    errors.append(("encode", i, it, rc))
                    return
                fs = off_o[:-1].copy()
                rc_o, out_o, _ = orc.decode_batch(wire_o, fs)
                pin_in[: len(wire_o)] = wire_o
                rc, out, _ = c.decode_batch_host(pin_in[: len(wire_o)], fs, out=pin_out)
                if rc != rc_o or not np.array_equal(out[: len(wire_o)], out_o):
                    errors.append(("decode", i, it, rc))
                    return
                data = bytes(wl.random_bytes(rng, int(rng.integers(1, 100))))
                key = int(rng.integers(0, 2**32))
                kb = np.frombuffer(key.to_bytes(4, "little"), np.uint8)
                ref = np.frombuffer(data, np.uint8) ^ kb[np.arange(len(data)) % 4]
                if not np.array_equal(np.frombuffer(c.xor_host(data, key, 0), np.uint8), ref):
                    errors.append(("xor", i, it))
                    return
        except Exception as e:
            errors.append(("exception", i, repr(e)))

    threads = [threading.Thread(target=work, args=(i,)) for i in range(n_threads)]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    stats = [c.lane_stats() for c in codecs]
    res.update(errors=errors[:5], alive=sum(th.is_alive() for th in threads), launches=stats[0][1],
               requests=sum(s[0] for s in stats), running=stats[0][2])
    res["ok"] = bool(not errors and res["alive"] == 0 and res["launches"] >= 50 and res["running"] != -1)
    if churn:
        # given up and brought back again and again under the eight threads,
        # every result still exact; and the lane serves requests afterwards
        r0 = codecs[0].lane_stats()[0]
        time.sleep(0.3)   # past the last hold-off
        data = bytes(range(40))
        back = bool(np.array_equal(np.frombuffer(codecs[0].xor_host(data, 0x01020304, 1), np.uint8),
                                   xor_ref(data, 0x01020304, 1)))
        back &= codecs[0].lane_stats()[0] > r0 and codecs[0].lane_stats()[2] != -1
        give_ups, rearms = codecs[0].lane_events()
        res.update(give_ups=give_ups, rearms=rearms, lane_back=back)
        res["ok"] = bool(not errors and res["alive"] == 0 and give_ups >= 2 and rearms >= 2 and back)
    for c in codecs:
        c.close()
    print(json.dumps(res))


def main():
    case = sys.argv[1]
    if case == "handover":
        return handover({"case": case})
    if case == "churn":
        return handover({"case": case}, churn=True)
    if case == "wrap":
        return wrap({"case": case})
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
        req0, launches0, _ = c.lane_stats()
        # the lane comes back (hold-off passed, it has left, nothing in
        # flight; only its first launch was held back): the next batches and
        # per-call XORs are lane requests of a new launch, exact
        wire2, fs2 = batch(2)
        rc2_o, out2_o, _ = oracle.decode_batch(wire2, fs2)
        pin_in[: len(wire2)] = wire2
        rc2, out2, _ = c.decode_batch_host(pin_in[: len(wire2)], fs2, out=pin_out)
        second = rc2 == rc2_o and np.array_equal(out2, out2_o)
        rng = np.random.default_rng(3)
        xor_ok = True
        for i in range(200):
            data = bytes(wl.random_bytes(rng, int(rng.integers(1, 200))))
            key, phase = int(rng.integers(0, 2**32)), i % 4
            xor_ok &= bool(np.array_equal(np.frombuffer(c.xor_host(data, key, phase), np.uint8),
                                          xor_ref(data, key, phase)))
        req1, launches1, running1 = c.lane_stats()
        back = req1 - req0 >= 201 and launches1 > launches0 and running1 != -1
        res.update(first=first, untouched_after=untouched_after, second=second, xor_ok=xor_ok,
                   lane_back=bool(back), requests=[req0, req1], launches=[launches0, launches1],
                   running_after=running1)
        res["ok"] = bool(first and untouched_after and second and xor_ok and back and res["running"] == -1)
    else:
        time.sleep(1.5)   # the late lane starts (0.9 s) and must leave without the request
        untouched = bool(np.all(np.array(pin_out) == 0xEE))
        rc2, _, _ = c.decode_batch_host(pin_in, fs, out=pin_out)
        res.update(untouched=untouched, rc_after=rc2)
        c.close()   # (a dead context: its buffers are left to the process's end, not freed under the lane)
        res["ok"] = bool(rc == WSG_EHIP and untouched and rc2 == WSG_EHIP)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
