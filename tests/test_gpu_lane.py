"""The host lane (wsg_lane_stats, wsg_internal.h): page-locked host batches
of at most $WSG_LANE_MAX wire bytes, and the per-call path's XORs, go to the
device's resident lane — one kernel shared by every context of the process,
a mailbox per workgroup in host memory — instead of a launch per call.  Its
bytes and per-frame fields must be those of the launch path and of the
oracle, bit-exact:

* many rounds through the SAME page-locked buffers with new bytes each time
  (the lane never returns between requests: a stale cache line would show),
  decode out of place and in place, encode, small frames to 64 KiB batches;
* frame tables with errors (truncated last frame, a length running into the
  next frame, a start past the wire) and tables the lane must not take
  (not strictly increasing: the launch path);
* the lane leaving after its idle limit and being launched again;
* the lane against the launch path ($WSG_LANE_MAX=0) on the same batches;
* several contexts on several threads sharing the one lane;
* a request the lane does not answer in time (tests/lane_timeout_job.py, its
  own process): the caller waits for the lane to leave before it uses the
  buffers, and a lane that starts late does not take the abandoned request."""
import os
import time

import numpy as np
import pytest

import oracle

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
from tests.test_gpu_parity import INFO_FIELDS  # noqa: E402

OPCODES = [0x81, 0x82, 0x01, 0x88, 0x89, 0x8A, 0xC2]


def _codec(**env):
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return ca.Codec(0)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


@pytest.fixture(scope="module")
def lane():
    c = _codec(WSG_LANE_MAX=65536)
    yield c
    c.close()


@pytest.fixture(scope="module")
def launch():
    c = _codec(WSG_LANE_MAX=0)
    yield c
    c.close()


def _small_batch(rng, max_wire=60000):
    n = int(rng.choice([1, 3, 40, 300, 1000, 1700]))
    cls = rng.random(n)
    lens = np.where(cls < 0.7, rng.integers(0, 126, n), np.where(cls < 0.97, rng.integers(126, 600, n),
                                                                 rng.integers(600, 9000, n)))
    while True:
        desc, total = wl.ragged_desc(rng, lens)
        desc["opcode"] = rng.choice(OPCODES, n)
        desc["mask"] = rng.random(n) < 0.9
        desc["status"] = np.where(rng.random(n) < 0.2, rng.integers(0, 70000, n), 0)
        desc["src_off"] += rng.integers(0, 16, n).astype(np.uint64)
        if int(ca.frame_sizes(desc).sum()) <= max_wire or n == 1:
            break
        lens = lens // 2
    payload = wl.random_bytes(rng, total + 16)
    return payload, desc


def _check_decode(c, pin_in, wire, fs, pin_out=None):
    rc_o, out_o, info_o = oracle.decode_batch(wire, fs)
    pin_in[: len(wire)] = wire
    rc, out, info = c.decode_batch_host(pin_in[: len(wire)], fs, out=pin_out if pin_out is not None else pin_in)
    assert rc == rc_o
    assert np.array_equal(out[: len(wire)], out_o)
    for f in INFO_FIELDS:
        assert np.array_equal(info[f], info_o[f]), f


def test_lane_rounds_same_buffers(lane):
    rng = np.random.default_rng(11)
    pin_p, pin_w = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
    pin_in, pin_out = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
    r0, _, _ = lane.lane_stats()
    for it in range(300):
        payload, desc = _small_batch(rng)
        wire_o, off_o = oracle.encode_batch(payload, desc)
        pin_p[: len(payload)] = payload
        rc, wire, off = lane.encode_batch_host(pin_p[: len(payload)], desc, wire=pin_w)
        assert rc == 0 and np.array_equal(off, off_o) and np.array_equal(wire, wire_o), it
        fs = off_o[:-1].copy()
        _check_decode(lane, pin_in, wire_o, fs, pin_out)   # out of place
        _check_decode(lane, pin_in, wire_o, fs)            # in place
    r1, launches, running = lane.lane_stats()
    assert r1 - r0 >= 3 * 300 - 5   # (a batch over the lane's size takes the launch path)
    assert running in (0, 1)


def test_lane_errors_and_tables(lane, launch):
    rng = np.random.default_rng(5)
    payload, desc = _small_batch(rng, max_wire=20000)
    wire_o, off_o = oracle.encode_batch(payload, desc)
    fs = off_o[:-1].copy()
    pin = ca.pinned_empty(1 << 16)
    pout = ca.pinned_empty(1 << 16)
    cases = {
        "truncated last": (wire_o[:-3], fs),
        "start past the wire": (wire_o, np.concatenate([fs, [len(wire_o) + 40]]).astype(np.uint64)),
        "frame runs into the next": (wire_o, np.sort(np.concatenate([fs, fs[-1:] + 1])).astype(np.uint64)),
        "first frame not at 0": (np.concatenate([np.zeros(7, np.uint8), wire_o]), fs + np.uint64(7)),
        "garbage starts": (wire_o, np.sort(rng.choice(len(wire_o), min(len(fs), 50), replace=False)).astype(np.uint64)),
        "not increasing (launch path)": (wire_o, fs[::-1].copy()),
        "repeated start (launch path)": (wire_o, np.concatenate([fs[:1], fs]).astype(np.uint64)),
        "empty wire": (np.zeros(0, np.uint8), np.zeros(3, np.uint64)),
    }
    for name, (w, f) in cases.items():
        rc_o, out_o, info_o = oracle.decode_batch(w, f)
        contract = bool(np.all(np.diff(f.astype(np.int64)) > 0))
        for c in (lane, launch):
            pin[: len(w)] = w
            rc, out, info = c.decode_batch_host(pin[: len(w)], f, out=pout)
            assert rc == rc_o, name
            if contract:
                assert np.array_equal(out[: len(w)], out_o), name
                for fld in INFO_FIELDS:
                    assert np.array_equal(info[fld], info_o[fld]), (name, fld)
            else:
                # a table that is not strictly increasing breaks the decode
                # contract (include/wsg_capi.h): the status and every frame's
                # error are the oracle's, the valid frames' fields too; the
                # output bytes are unspecified (test_decode_garbage_starts_match_oracle)
                assert np.array_equal(info["error"], info_o["error"]), name
                ok = info_o["error"] == 0
                for fld in INFO_FIELDS:
                    assert np.array_equal(info[fld][ok], info_o[fld][ok]), (name, fld)


def test_lane_idle_relaunch():
    c = _codec(WSG_LANE_MAX=65536)
    try:
        rng = np.random.default_rng(9)
        pin_in, pin_out = ca.pinned_empty(1 << 16), ca.pinned_empty(1 << 16)
        _, l0, _ = c.lane_stats()
        for it in range(6):
            payload, desc = _small_batch(rng, max_wire=30000)
            wire_o, off_o = oracle.encode_batch(payload, desc)
            _check_decode(c, pin_in, wire_o, off_o[:-1].copy(), pin_out)
            time.sleep(0.03)   # 15 x the idle limit (2 ms): the lane has left
        req, launches, running = c.lane_stats()
        assert req == 6 and launches - l0 >= 5, (req, launches, l0)
    finally:
        c.close()


def test_lane_matches_launch_path_echo_shape(lane, launch):
    """The C1 echo's batches (1000 masked 38-byte frames; the replies of 1000
    32-byte payloads) through both paths, bytes and fields equal."""
    rng = np.random.default_rng(3)
    desc, total = wl.ragged_desc(rng, np.full(1000, 32))
    payload = wl.random_bytes(rng, total)
    pin_p = ca.pinned_empty(total)
    pin_p[:] = payload
    outs = []
    for c in (lane, launch):
        pw = ca.pinned_empty(int(ca.frame_sizes(desc).sum()))
        rc, w, off = c.encode_batch_host(pin_p, desc, wire=pw)
        assert rc == 0
        outs.append(np.array(w))
    assert np.array_equal(outs[0], outs[1])
    wire_o, off_o = oracle.encode_batch(payload, desc)
    assert np.array_equal(outs[0], wire_o)
    pin_in, pin_out = ca.pinned_empty(len(wire_o)), ca.pinned_empty(len(wire_o))
    for c in (lane, launch):
        _check_decode(c, pin_in, wire_o, off_o[:-1].copy(), pin_out)


def test_lane_payload_arenas(lane):
    """Encode reads its payloads from an LDS copy of the arena when the
    arena's 16-B blocks fit LANE_PSTAGE (64 KiB), else from host memory: both
    sides of that limit, arenas not 16-B aligned, frames scattered over a
    large arena, and zero-length payloads, against the oracle."""
    rng = np.random.default_rng(21)
    big = ca.pinned_empty(1 << 19)
    pin_w = ca.pinned_empty(1 << 17)
    for arena in (0, 17, 65536 - 32, 65536 - 16, 65536 - 1, 65536, 65536 + 40, 300000):
        for mis in (0, 1, 7, 15):
            n = int(rng.integers(1, 1200))
            lens = rng.integers(0, 60, n) if arena else np.zeros(n, np.int64)
            lens = np.minimum(lens, arena)
            desc = np.zeros(n, dtype=ca.SEND_DESC)
            desc["len"] = lens
            desc["src_off"] = [int(rng.integers(0, arena - int(ln) + 1)) for ln in lens]
            # the first and last byte of the arena are read by some frame
            if arena and n > 1 and lens[0] > 0:
                desc["src_off"][0] = 0
                desc["len"][-1] = min(int(lens[-1]) or 1, arena)
                desc["src_off"][-1] = arena - int(desc["len"][-1])
            desc["key"] = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
            desc["opcode"] = rng.choice(OPCODES, n)
            desc["mask"] = rng.random(n) < 0.9
            desc["status"] = np.where(rng.random(n) < 0.1, rng.integers(0, 70000, n), 0)
            payload = wl.random_bytes(rng, arena)
            view = big[mis: mis + arena]
            view[:] = payload
            wire_o, off_o = oracle.encode_batch(payload, desc)
            assert len(wire_o) <= 65536
            rc, wire, off = lane.encode_batch_host(view, desc, wire=pin_w)
            assert rc == 0 and np.array_equal(off, off_o), (arena, mis)
            assert np.array_equal(wire, wire_o), (arena, mis)


def _batch_of(rng, lens, mask=0.9):
    n = len(lens)
    desc, total = wl.ragged_desc(rng, np.asarray(lens))
    desc["opcode"] = rng.choice(OPCODES, n)
    desc["mask"] = rng.random(n) < mask
    desc["status"] = np.where(rng.random(n) < 0.05, rng.integers(0, 70000, n), 0)
    return wl.random_bytes(rng, total + 16), desc


def test_lane_byte_groups_large_batches():
    """Batches past one group's LDS stage (64 KiB) up to the lane's request
    limit ($WSG_LANE_MAX: 512 KiB by default, 2 MiB here) are cut into groups of about equal
    wire bytes, each a run of whole frames whose range fits the stage (decode)
    or whose payload span usually does (encode): many echo-sized frames,
    a few frames just under the stage, ragged mixes, and the cases that leave
    the lane — a frame larger than the stage (decode; encode keeps it, a group
    alone), more frames than the lane's groups hold, a batch over the limit.
    Encode, decode out of place and in place, against the oracle; the lane's
    request count shows which went to the lane."""
    c = _codec(WSG_LANE_MAX=2 << 20)
    try:
        rng = np.random.default_rng(77)
        cap = 4 << 20
        pin_p, pin_w = ca.pinned_empty(cap), ca.pinned_empty(cap)
        pin_in, pin_out = ca.pinned_empty(cap), ca.pinned_empty(cap)
        stage = 65536
        cases = {   # name: (payload lengths, encode on the lane, decode on the lane)
            "echo frames 760 KB": (np.full(20000, 32), True, True),
            "frames just under the stage": (np.full(30, stage - 200), True, True),
            "ragged 1.2 MB": (rng.integers(0, 2000, 1200), True, True),
            "1.9 MB of 1000 B frames": (np.full(1900, 1000), True, True),
            "one frame over the stage": (np.concatenate([np.full(500, 40), [100000], np.full(500, 40)]), True, False),
            "over the frame limit": (np.zeros(40000, np.int64), False, False),
            "over the request limit": (np.full(3000, 1000), False, False),
            "65 KB just over one group": (np.full(1700, 33), True, True),
        }
        for name, (lens, enc_lane, dec_lane) in cases.items():
            payload, desc = _batch_of(rng, lens)
            wire_o, off_o = oracle.encode_batch(payload, desc)
            assert len(wire_o) <= cap and len(payload) <= cap
            pin_p[: len(payload)] = payload
            r0, _, _ = c.lane_stats()
            rc, wire, off = c.encode_batch_host(pin_p[: len(payload)], desc, wire=pin_w)
            assert rc == 0 and np.array_equal(off, off_o) and np.array_equal(wire, wire_o), name
            r1, _, _ = c.lane_stats()
            assert (r1 - r0 == 1) == enc_lane, (name, "encode", r1 - r0)
            fs = off_o[:-1].copy()
            _check_decode(c, pin_in, wire_o, fs, pin_out)
            _check_decode(c, pin_in, wire_o, fs)
            r2, _, _ = c.lane_stats()
            assert (r2 - r1 == 2) == dec_lane and (r2 - r1) in (0, 2), (name, "decode", r2 - r1)
    finally:
        c.close()


def _latch_cases(rng, n):
    payload, desc = _batch_of(rng, rng.integers(0, 90, n))
    wire_o, off_o = oracle.encode_batch(payload, desc)
    fs = off_o[:-1].copy()
    mid = n // 2
    return wire_o, fs, {
        "truncated last": (wire_o[:-3], fs),
        "runs into the next": (wire_o, np.sort(np.concatenate([fs, fs[mid:mid + 1] + 1])).astype(np.uint64)),
        "start past the wire": (wire_o, np.concatenate([fs, [len(wire_o) + 40]]).astype(np.uint64)),
        "first frame's header garbage": (np.concatenate([np.full(2, 0x7F, np.uint8), wire_o[2:]]), fs),
    }


def _latch_check(c, name, ww, ff, pin=None, pout=None):
    rc_o, out_o, info_o = oracle.decode_batch(ww, ff)
    if pin is not None:   # page-locked: in place on the launch path
        pin[: len(ww)] = ww
        rc, out, info = c.decode_batch_host(pin[: len(ww)], ff, out=pout)
    else:                 # pageable: the staged pipeline
        rc, out, info = c.decode_batch_host(np.array(ww), ff)
    assert rc == rc_o, name
    assert np.array_equal(out[: len(ww)], out_o), name
    for fld in INFO_FIELDS:
        assert np.array_equal(info[fld], info_o[fld]), (name, fld)


def test_launch_path_status_from_the_latch(launch):
    """Decodes of 4096 frames or more read the error latch back and skip the
    status pass over the records when no frame erred — in place on the
    launch path (page-locked buffers) and through the staged pipeline
    (pageable buffers, 1 MiB segments: the frames cut into four): clean
    batches around a truncated last frame, a frame running into the next
    (ETRUNC turned EINVAL by the pass), a start past the wire and a garbage
    header (each followed by a clean batch: the latch re-armed), rc / bytes /
    records against the oracle."""
    rng = np.random.default_rng(31)
    wire_o, fs, bad = _latch_cases(rng, 6000)
    pin, pout = ca.pinned_empty(len(wire_o) + 64), ca.pinned_empty(len(wire_o) + 64)
    for name, (w, f) in bad.items():
        for ww, ff in ((wire_o, fs), (w, f), (wire_o, fs)):
            _latch_check(launch, name, ww, ff, pin, pout)
    staged = _codec(WSG_STAGE_MB=1)
    try:
        wire_o, fs, bad = _latch_cases(rng, 70000)
        assert len(wire_o) > 3 << 20
        for name, (w, f) in bad.items():
            for ww, ff in ((wire_o, fs), (w, f), (wire_o, fs)):
                _latch_check(staged, name, ww, ff)
    finally:
        staged.close()


@pytest.mark.parametrize("groups", [1, 3, 32])
def test_lane_group_counts(groups):
    """A request is cut into frame groups ($WSG_LANE_GROUPS at most; one per
    idle workgroup), each staged and written by one workgroup: one group, an
    odd count, more groups than workgroups (a workgroup taking several of one
    request); decode in and out of place, encode, against the oracle."""
    c = _codec(WSG_LANE_MAX=65536, WSG_LANE_GROUPS=groups)
    try:
        rng = np.random.default_rng(100 + groups)
        pin_p, pin_w = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
        pin_in, pin_out = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
        r0, _, _ = c.lane_stats()
        for it in range(40):
            if it % 4 == 0:   # many tiny frames: several groups per workgroup
                n = int(rng.integers(2000, 4000))
                desc, total = wl.ragged_desc(rng, rng.integers(0, 9, n))
                desc["mask"] = True
                payload = wl.random_bytes(rng, total + 16)
            else:
                payload, desc = _small_batch(rng)
            wire_o, off_o = oracle.encode_batch(payload, desc)
            pin_p[: len(payload)] = payload
            rc, wire, off = c.encode_batch_host(pin_p[: len(payload)], desc, wire=pin_w)
            assert rc == 0 and np.array_equal(off, off_o) and np.array_equal(wire, wire_o), (groups, it)
            fs = off_o[:-1].copy()
            _check_decode(c, pin_in, wire_o, fs, pin_out)
            _check_decode(c, pin_in, wire_o, fs)
        r1, _, _ = c.lane_stats()
        assert r1 - r0 >= 3 * 40 - 6, (r0, r1)
    finally:
        c.close()


def test_lane_periodic_relaunch_and_device_sync():
    """A launch of the lane ends after $WSG_LANE_YIELD_US of running (2 ms)
    and the next call launches it again behind it: results stay exact across
    the hand-overs, and a device-wide synchronize from another thread (what
    hipFree / hipHostFree do) waits for one hand-over, not for the busy lane
    to go idle."""
    import threading

    c = _codec(WSG_LANE_MAX=65536)
    busy = _codec(WSG_LANE_MAX=65536)
    try:
        rng = np.random.default_rng(17)
        pin_in, pin_out = ca.pinned_empty(1 << 16), ca.pinned_empty(1 << 16)
        r0, _, _ = c.lane_stats()
        for it in range(40):
            payload, desc = _small_batch(rng, max_wire=30000)
            wire_o, off_o = oracle.encode_batch(payload, desc)
            _check_decode(c, pin_in, wire_o, off_o[:-1].copy(), pin_out)
        r1, _, _ = c.lane_stats()
        assert r1 - r0 == 40, (r1 - r0)

        # another thread keeps the lane answering; this one synchronizes
        payload, desc = _small_batch(np.random.default_rng(2), max_wire=30000)
        wire_o, off_o = oracle.encode_batch(payload, desc)
        fs = off_o[:-1].copy()
        b_in, b_out = ca.pinned_empty(len(wire_o)), ca.pinned_empty(len(wire_o))
        b_in[:] = wire_o
        rc_o, out_o, _ = oracle.decode_batch(wire_o, fs)
        stop = threading.Event()
        errors = []

        def hammer():
            try:
                while not stop.is_set():
                    rc, out, _ = busy.decode_batch_host(b_in, fs, out=b_out)
                    if rc != rc_o or not np.array_equal(out, out_o):
                        errors.append(rc)
                        return
            except Exception as e:  # pragma: no cover - reported below
                errors.append(e)

        th = threading.Thread(target=hammer)
        th.start()
        try:
            time.sleep(0.3)
            _, l0, _ = busy.lane_stats()
            waits = []
            for _ in range(5):
                t0 = time.perf_counter()
                torch.cuda.synchronize()
                waits.append(time.perf_counter() - t0)
                time.sleep(0.02)
            _, l1, _ = busy.lane_stats()
        finally:
            stop.set()
            th.join(timeout=30)
        assert not th.is_alive() and not errors, errors
        # a hand-over every 2 ms while the other thread keeps ringing; the
        # idle limit alone would never come
        assert l1 - l0 >= 10, (l0, l1)
        assert max(waits) < 0.25, waits
    finally:
        busy.close()
        c.close()


def test_lane_shared_by_contexts():
    """Eight threads, each with its own context (as a server's IO threads
    have), decode and encode through the one lane of the device at once:
    every batch bit-exact against the oracle, one set of launches for all."""
    import threading

    n_threads, rounds = 8, 60
    codecs = [_codec(WSG_LANE_MAX=65536) for _ in range(n_threads)]
    errors = []

    def work(i):
        try:
            c = codecs[i]
            rng = np.random.default_rng(300 + i)
            pin_p, pin_w = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
            pin_in, pin_out = ca.pinned_empty(1 << 17), ca.pinned_empty(1 << 17)
            for it in range(rounds):
                payload, desc = _small_batch(rng)
                wire_o, off_o = oracle.encode_batch(payload, desc)
                pin_p[: len(payload)] = payload
                rc, wire, off = c.encode_batch_host(pin_p[: len(payload)], desc, wire=pin_w)
                if rc != 0 or not np.array_equal(off, off_o) or not np.array_equal(wire, wire_o):
                    errors.append(("encode", i, it, rc))
                    return
                fs = off_o[:-1].copy()
                rc_o, out_o, info_o = oracle.decode_batch(wire_o, fs)
                pin_in[: len(wire_o)] = wire_o
                rc, out, info = c.decode_batch_host(pin_in[: len(wire_o)], fs, out=pin_out)
                if rc != rc_o or not np.array_equal(out[: len(wire_o)], out_o) or any(
                        not np.array_equal(info[f], info_o[f]) for f in INFO_FIELDS):
                    errors.append(("decode", i, it, rc))
                    return
                data = wl.random_bytes(rng, int(rng.integers(1, 3000)))
                key, phase = int(rng.integers(0, 2**32)), int(rng.integers(0, 4))
                if not np.array_equal(np.frombuffer(c.xor_host(data, key, phase), np.uint8), _xor_ref(data, key, phase)):
                    errors.append(("xor", i, it))
                    return
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("exception", i, repr(e)))

    try:
        r0 = [c.lane_stats()[0] for c in codecs]
        threads = [threading.Thread(target=work, args=(i,)) for i in range(n_threads)]
        for th in threads:
            th.start()
        for th in threads:
            th.join(timeout=120)
        assert not any(th.is_alive() for th in threads)
        assert not errors, errors[:5]
        stats = [c.lane_stats() for c in codecs]
        # every context put its requests on the lane, and they all see the same
        # lane (one count of launches)
        assert all(s[0] - r >= 3 * rounds - 5 for s, r in zip(stats, r0)), (stats, r0)
        assert len({s[1] for s in stats}) == 1, stats
    finally:
        for c in codecs:
            c.close()


def _xor_ref(data, key, phase):
    kb = np.frombuffer(int(key).to_bytes(4, "little"), np.uint8)
    idx = (np.arange(len(data)) + phase) % 4
    return np.frombuffer(bytes(data), np.uint8) ^ kb[idx]


def test_lane_per_call_xor(lane, launch):
    """The per-call path's XOR (wsg_xor_host: PrepareSendFrame /
    PrepareReceiveFrame outside a batch scope) on the lane up to 64 KiB, the
    launch path above, and with the lane off: every length class, every key
    phase, against a numpy restatement of ws.cpp:264-270."""
    rng = np.random.default_rng(41)
    r0, _, _ = lane.lane_stats()
    lens = [1, 2, 3, 15, 16, 17, 31, 32, 33, 39, 40, 41, 63, 64, 125, 126, 1000, 4095, 4096, 4097, 16383, 16384,
            16385, 65535, 65536, 65537, 200000]   # (up to 40: the payload inside the task)
    for ln in lens:
        for phase in range(4):
            data = wl.random_bytes(rng, ln)
            key = int(rng.integers(0, 2**32))
            ref = _xor_ref(data, key, phase)
            for c in (lane, launch):
                got = np.frombuffer(bytes(c.xor_host(data, key, phase)), np.uint8)
                assert np.array_equal(got, ref), (ln, phase)
    r1, _, _ = lane.lane_stats()
    assert r1 - r0 == 4 * sum(1 for ln in lens if ln <= 65536), (r0, r1)


def _lane_job(case, env):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    job = os.path.join(root, "tests", "lane_timeout_job.py")
    e = dict(os.environ, **env)
    r = subprocess.run([sys.executable, job, case], env=e, capture_output=True, text=True, timeout=90, cwd=root)
    assert r.returncode == 0, (case, r.stdout[-2000:], r.stderr[-2000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["ok"], (case, json.dumps(res))


def test_lane_inline_answers_across_the_tag_wrap():
    """An inline XOR's answer units carry the low 32 bits of its ticket, which
    recur in a slot every 2^32 tickets: the host marks the slot's units stale
    before each task goes out.  In a process of its own, tickets start just
    below 2^32 with every slot's units left as the task 2^32 tickets earlier
    would have left them; 3000 per-call XORs cross the mark and the ring
    several times, every one on the lane and equal to ws.cpp:264-270's
    bytes."""
    _lane_job("wrap", {"WSG_TEST_LANE_TICKET_BASE": str(2**32 - 300), "WSG_TEST_LANE_STALE_XRES": "1"})


def test_lane_timeout_waits_for_the_lane():
    """A request the lane leaves unanswered ($WSG_LANE_TIMEOUT_MS; the lane
    held back by $WSG_TEST_LANE_DELAY_US) in a process of its own: the caller
    gives the lane up and waits for it to leave before the launch path reuses
    the buffers; the late lane does not take the abandoned request (nothing
    written after the call returned), and the lane comes back for the next
    calls (a new launch, every result exact); and when the lane does not leave in
    time, the call fails without touching the buffers and the context refuses
    further calls.  And the lane handing over every few tens of
    microseconds while eight threads' contexts use it: every result exact,
    no request lost across a hand-over; and the same while the lane is given
    up and brought back again and again (churn)."""
    for case, env in (("drained", {"WSG_LANE_TIMEOUT_MS": "150", "WSG_TEST_LANE_DELAY_US": "500000",
                                   "WSG_TEST_LANE_DELAY_GENS": "1", "WSG_LANE_DRAIN_MS": "3000"}),
                      ("lost", {"WSG_LANE_TIMEOUT_MS": "100", "WSG_TEST_LANE_DELAY_US": "900000",
                                "WSG_LANE_DRAIN_MS": "100"}),
                      ("handover", {"WSG_LANE_YIELD_US": "40", "WSG_LANE_IDLE_US": "20"}),
                      ("churn", {"WSG_LANE_YIELD_US": "400", "WSG_LANE_IDLE_US": "200", "WSG_LANE_TIMEOUT_MS": "30",
                                 "WSG_TEST_LANE_DELAY_US": "60000", "WSG_TEST_LANE_DELAY_EVERY": "4",
                                 "WSG_LANE_DRAIN_MS": "3000"})):
        _lane_job(case, env)
