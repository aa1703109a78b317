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


def main():
    name = sys.argv[1]
    seeds = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    c = ca.Codec(0, lib_path=os.path.join(ROOT, "cppserver_amd", "_build", "var", name, "libwsg.so"))
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
