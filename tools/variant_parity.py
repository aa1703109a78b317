"""Bit-exactness of an A/B build of the library (tools/build_variant.sh)
before it can replace the default: the device encode and decode of the
differential-fuzz batches (tests/test_gpu_fuzz.py's generator) and the full
C3 batch through the variant, every byte and offset against the oracle.
usage: python tools/variant_parity.py VARIANT [SEEDS]   -> one JSON line"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
from tests.test_gpu_fuzz import _batch  # noqa: E402


def encode(codec, payload, desc):
    p = torch.from_numpy(payload).cuda()
    d = ca.desc_to_tensor(desc, "cuda")
    cap = int(ca.frame_sizes(desc).sum())
    wire = torch.full((max(cap, 16) + 64,), 0xA5, dtype=torch.uint8, device="cuda")
    w, off = codec.encode_batch(p, d, wire=wire, wire_cap=cap)
    codec.sync()
    got = w.cpu().numpy()
    return got[:cap], off.cpu().numpy().view(np.uint64), bool((got[cap:] == 0xA5).all())


def fanout_parity(c, seeds, wpc_env):
    """Fan-outs of the differential fuzz (tests/test_gpu_fuzz.py's shapes),
    C4, and 16 x C4 in one wsg_fanout_encode_many call, vs the oracle."""
    from tests.test_gpu_fuzz import OPCODES

    bad = []
    for seed in range(seeds):
        rng = np.random.default_rng(7000 + seed)
        length = int(rng.choice([int(rng.integers(0, 126)), int(rng.integers(126, 9000)),
                                 int(rng.integers(60000, 70000))]))
        k = int(rng.integers(1, 30000 if length < 9000 else 60))
        opcode = int(rng.choice(OPCODES))
        mask = bool(rng.random() < 0.8)
        payload, keys = wl.c4_fanout(length, k, seed=seed)
        ref = oracle.fanout_encode(payload, keys, opcode, mask)
        wire = torch.full((len(ref) + 48,), 0xA5, dtype=torch.uint8, device="cuda")
        c.fanout(torch.from_numpy(payload).cuda(), torch.from_numpy(keys.view(np.int32)).cuda(), opcode, mask,
                 wire=wire, length=length)
        c.sync()
        got = wire.cpu().numpy()
        if not (np.array_equal(got[: len(ref)], ref) and (got[len(ref):] == 0xA5).all()):
            bad.append(seed)
    m, length, k = 16, 4096, 10000
    rng = np.random.default_rng(99)
    arena = rng.integers(0, 256, m * length, dtype=np.uint8)
    keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
    w, off = c.fanout_many(torch.from_numpy(arena).cuda(), np.arange(m, dtype=np.uint64) * np.uint64(length),
                           np.full(m, length, dtype=np.uint64), np.full(m, 0x82, dtype=np.uint8),
                           torch.from_numpy(keys.view(np.int32)).cuda())
    c.sync()
    got = w.cpu().numpy()
    many_ok = True
    for i in range(m):
        ref = oracle.fanout_encode(arena[i * length: (i + 1) * length], keys, 0x82, True)
        many_ok &= bool(np.array_equal(got[int(off[i]): int(off[i]) + len(ref)], ref))
    return {"fanout_seeds": seeds, "fanout_bad": bad, "many16_ok": many_ok, "env": wpc_env}


def main():
    name = sys.argv[1]
    seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    c = ca.Codec(0, lib_path=os.path.join(ROOT, "cppserver_amd", "_build", "var", name, "libwsg.so"))
    if "--fanout" in sys.argv:
        print(json.dumps(dict(variant=name, **fanout_parity(c, seeds, None))),
              flush=True)
        return
    bad = []
    for seed in range(seeds):
        payload, desc = _batch(1000 + seed)
        ref, ref_off = oracle.encode_batch(payload, desc)
        got, off, tail = encode(c, payload, desc)
        if not (np.array_equal(got, ref) and np.array_equal(off, ref_off) and tail):
            bad.append(seed)
    payload, desc = wl.c3_batch(65536, 128, 65536, seed=3000)
    ref, ref_off = oracle.encode_batch(payload, desc)
    got, off, tail = encode(c, payload, desc)
    c3 = bool(np.array_equal(got, ref) and np.array_equal(off, ref_off) and tail)
    print(json.dumps({"variant": name, "fuzz_seeds": seeds, "fuzz_bad": bad, "c3_full": c3}), flush=True)


if __name__ == "__main__":
    main()
