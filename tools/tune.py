"""Interleaved A/B timing of decode variants on the GPU box (medians).

usage: python tools/tune.py [bpc[:tiles_per_block][@lib.so] ...]
(env WSG_BLOCKS_PER_CU / WSG_DEC_TILES_PER_BLOCK per context)
Each context is created with its own WSG_BLOCKS_PER_CU; runs are interleaved
so clock/thermal drift hits every setting alike (guide §5.4 rule 24).
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def main():
    # settings: "BPC" or "BPC@path/to/libwsg.so"
    settings = sys.argv[1:] or ["8", "16", "32"]
    n, size = int(os.environ.get("FRAMES", 4096)), int(os.environ.get("SIZE", 65536))
    # ROT distinct batches, used in turn, so no step finds its input in the
    # 256 MiB Infinity Cache left warm by the previous step
    rot = int(os.environ.get("ROT", 1))
    ragged = os.environ.get("RAGGED")   # "lo,hi": C3-style ragged frames (payload uniform in [lo, hi])
    if ragged:
        lo, hi = (int(x) for x in ragged.split(","))
        rot = 1   # a ragged batch (GBs) is far larger than the Infinity Cache anyway
        enc = ca.Codec(0)
        payload, desc = wl.c3_batch(n, lo, hi, seed=3)
        w_, off = enc.encode_batch(torch.from_numpy(payload).cuda(), ca.desc_to_tensor(desc, "cuda"),
                                   wire_cap=int(ca.frame_sizes(desc).sum()))
        enc.sync()
        enc.close()
        ws, f = [w_], off[:-1].clone()
        wire = ws[0].cpu().numpy()
        size = len(wire) // n
    else:
        wire, fs, _ = wl.c2_wire(n, size, seed=1)
        ws = [torch.from_numpy(wire).cuda()] + [torch.from_numpy(wl.c2_wire(n, size, seed=2 + r)[0]).cuda()
                                               for r in range(rot - 1)]
        f = torch.from_numpy(fs.view(np.int64)).cuda()
    outs = [torch.empty_like(ws[0]) for _ in range(rot)]
    if os.environ.get("INPLACE") == "1":   # out aliases the wire (a receive buffer unmasked where it lies)
        outs = list(ws)
    if os.environ.get("ARENA") == "1":
        # every wire and output carved from ONE allocation (16 KiB-aligned
        # slots), as a server's preallocated batch arena would hold them
        slot = (ws[0].numel() + 16383) // 16384 * 16384
        arena = torch.empty(2 * rot * slot, dtype=torch.uint8, device="cuda")
        for r in range(rot):
            a = arena[2 * r * slot: 2 * r * slot + ws[0].numel()]
            a.copy_(ws[r])
            ws[r] = a
            outs[r] = arena[(2 * r + 1) * slot: (2 * r + 1) * slot + ws[0].numel()]
    info = torch.empty(n * 32, dtype=torch.uint8, device="cuda")
    it = [0]

    def step1(c):
        k = it[0] % rot
        it[0] += 1
        c.decode_batch(ws[k], f, out=outs[k], info=info)
    codecs = {}
    for b in settings:
        # "BPC[:TPB][@lib]": blocks per CU cap, and tiles per block (0: off)
        grid, _, path = b.partition("@")
        bpc, _, tpb = grid.partition(":")
        os.environ["WSG_BLOCKS_PER_CU"] = bpc
        os.environ["WSG_DEC_TILES_PER_BLOCK"] = tpb or "0"
        codecs[b] = ca.Codec(0, lib_path=path or None)
    every = int(os.environ.get("EVERY", 1))
    kern = {b: [] for b in settings}
    step = {b: [] for b in settings}
    bare = {b: [] for b in settings}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(int(os.environ.get("REPS", 7))):
        for b in settings:
            c = codecs[b]
            for _ in range(3):
                step1(c)
            e0.record()
            for _ in range(20):
                step1(c)
            e1.record()
            e1.synchronize()
            bare[b].append(e0.elapsed_time(e1) / 20)
            c.timing(True, every)
            c.timing_read()
            e0.record()
            for _ in range(20):
                step1(c)
            e1.record()
            e1.synchronize()
            ms, k = c.timing_read()
            c.timing(False)
            kern[b].append(ms / k)
            step[b].append(e0.elapsed_time(e1) / 20)
    alg = 2 * len(wire)
    print("batches in rotation: %d x %.0f MB wire" % (rot, len(wire) / 1e6))
    for b in settings:
        km, sm, bm = statistics.median(kern[b]), statistics.median(step[b]), statistics.median(bare[b])
        print("%-40s kernel %.4f ms (%.0f GB/s)  step %.4f ms (%.0f GiB/s)  untimed step %.4f ms (%.0f GiB/s)  spread %.1f%%" % (
            b, km, alg / km / 1e6, sm, n * size / (sm * 1e-3) / 2**30, bm, n * size / (bm * 1e-3) / 2**30,
            100 * (max(kern[b]) - min(kern[b])) / km))


if __name__ == "__main__":
    main()
