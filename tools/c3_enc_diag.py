"""Where the ragged C3 encode loses against C5's uniform frames (VERDICT r3
item 4).  Interleaved A/B over library builds (tools/build_variant.sh):
  base   the in-tree library
  diag1  no edge chunks (header / shared chunks not written: timing only)
  diag4  shared chunks stored whole instead of byte by byte (timing only)
  diag2  no source funnel (misaligned loads taken as aligned: timing only)
  eu8 / eu2   8 KiB / 2 KiB pieces
on the C3 batch (65536 frames, 128 B - 64 KiB), C3's bytes as uniform
frames, and a C5 rank share; k_encode_mask time from each library's HIP
events.  Also the piece-occupancy of each batch (pieces per frame, bytes of
a piece used).  Prints one JSON line.  Diagnostic only (not a parity check).
"""
import json
import os
import statistics
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402

VAR = os.path.join(ROOT, "cppserver_amd", "_build", "var")


def occupancy(desc, piece=4096, align=128):
    sizes = ca.frame_sizes(desc).astype(np.int64)
    off = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    lead = off % align
    pieces = (sizes + lead + piece - 1) // piece
    return {"frames": int(len(desc)), "pieces": int(pieces.sum()), "pieces_per_frame": round(float(pieces.mean()), 3),
            "bytes_per_piece": round(float(sizes.sum() / pieces.sum()), 1),
            "fill": round(float(sizes.sum() / (pieces.sum() * piece)), 4)}


def batches():
    payload, desc = wl.c3_batch(65536, 128, 65536, seed=3000)
    yield "C3", payload, desc
    n = 65536
    mean = int(desc["len"].mean()) // 16 * 16
    rng = np.random.default_rng(5)
    d2, total = wl.ragged_desc(rng, np.full(n, mean))
    yield "C3 bytes as uniform %d B frames" % mean, wl.random_bytes(rng, total), d2
    ids = np.arange(1 << 17)
    yield "C5 1/8 share", None, (ids, wl.c5_desc(ids, 16384))


def main():
    want = sys.argv[1:] or ["diag1", "diag4", "diag2", "eu8", "eu2"]
    names = ["base"] + [v for v in want if os.path.exists(os.path.join(VAR, v, "libwsg.so"))]
    codecs = {n: ca.Codec(0) if n == "base" else ca.Codec(0, lib_path=os.path.join(VAR, n, "libwsg.so")) for n in names}
    out = {"variants": names, "batches": []}
    for name, payload, desc in batches():
        if payload is None:
            ids, desc = desc
            p = wl.c5_payload_torch(ids, 16384, device="cuda")
        else:
            p = torch.from_numpy(payload).cuda()
        d = ca.desc_to_tensor(desc, "cuda")
        cap = int(ca.frame_sizes(desc).sum())
        wire = torch.empty(cap, dtype=torch.uint8, device="cuda")
        woff = torch.empty(len(desc) + 1, dtype=torch.int64, device="cuda")
        alg = int(desc["len"].sum()) + cap
        for c in codecs.values():   # warm-up ~0.2 s
            for _ in range(40):
                c.encode_batch(p, d, wire=wire, wire_cap=cap, wire_off=woff)
        torch.cuda.synchronize()
        res = {n: [] for n in names}
        for rep in range(8):
            for n, c in codecs.items():
                c.timing(True, every=1)
                c.timing_read(reset=True)
                for _ in range(5):
                    c.encode_batch(p, d, wire=wire, wire_cap=cap, wire_off=woff)
                ms, k = c.timing_read(reset=True)
                c.timing(False)
                res[n].append(ms / max(k, 1))
        b = {"batch": name, "alg_bytes": alg, "occupancy": occupancy(desc)}
        for n in names:
            med = statistics.median(res[n])
            b[n] = {"ms": round(med, 4), "frac": round(alg / (med * 1e-3) / 8e12, 4)}
        out["batches"].append(b)
        print(json.dumps(b), file=sys.stderr, flush=True)
        del p, d, wire, woff
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
