"""C5 through the one-process multi-GPU C-ABI entry (wsg_mgpu_create over
several GPUs): the 1 Mi x 16 KiB job dealt round-robin in
1024-frame chunks to the GPUs, every GPU encodes its shard,
wsg_mgpu_encode_gather moves the framed chunks to device 0 (xGMI peer
copies, every sender on its own link into the root); the root checks
sampled frames against the oracle.  Prints one JSON object.  bench.py runs
it from rank 0 at N > 1 (in its own process, under a time limit).
$WSG_MGPU_ONE_DEVICE=1 puts every rank on device 0 (a rehearsal of the
N-rank flow on a one-GPU box).

usage: python tools/mgpu_c5.py NGPUS [n_total] [size] [chunk]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
import oracle  # noqa: E402  (the checker)
from cppserver_amd import shard  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def host_leg(g, ngpu, reps=3):
    """The PCIe-inclusive decode (host wire in pinned memory -> GPUs -> host)
    of ngpu x 4096 x 64 KiB frames: on device 0 alone, then split over every
    GPU of the group (wsg_mgpu_decode_batch_host: a run per GPU, each on its
    own link); payload GiB/s, sampled frames checked against the oracle."""
    n, size = 4096 * ngpu, 65536
    wire, fs, _ = wl.c2_wire(n, size, seed=5)
    pin_in, pin_out = ca.pinned_empty(len(wire)), ca.pinned_empty(len(wire))
    pin_in[:] = wire
    del wire
    one = ca.Codec(0)
    res = {"workload": "%d x %d B masked frames, pinned host buffers" % (n, size)}
    try:
        for name, fn in (("one_gpu", lambda: ca.decode_batch_host_multi([one], pin_in, fs, out=pin_out)),
                         ("all_gpus", lambda: g.decode_batch_host(pin_in, fs, out=pin_out))):
            rc, _, _ = fn()
            assert rc == 0, rc
            t0 = time.perf_counter()
            for _ in range(reps):
                fn()
            res[name + "_GiBps"] = round(n * size * reps / (time.perf_counter() - t0) / 2**30, 2)
        ok = True
        for i in (0, n // 2, n - 1):
            a, b = int(fs[i]), int(fs[i]) + size + 14
            rc, ref, _ = oracle.decode_batch(np.array(pin_in[a:b]), np.zeros(1, np.uint64))
            ok &= rc == 0 and bool(np.array_equal(pin_out[a:b], ref))
        res["check"] = bool(ok)
    finally:
        one.close()
    return res


def main():
    ngpu = int(sys.argv[1])
    n_total = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    size = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    chunk = int(sys.argv[4]) if len(sys.argv) > 4 else 1024
    one_device = os.environ.get("WSG_MGPU_ONE_DEVICE") == "1"
    devs = [0] * ngpu if one_device else list(range(ngpu))
    g = ca.MultiGPU(devs)
    try:
        fsz = ca.frame_size(0x82, True, size)
        payloads, descs, wires, woffs = [], [], [], []
        for r in range(ngpu):
            ids = shard.rank_frames(r, ngpu, n_total, chunk)
            dev = torch.device("cuda", devs[r])
            payloads.append(wl.c5_payload_torch(ids, size, device=dev))
            descs.append(ca.desc_to_tensor(wl.c5_desc(ids, size), dev))
            wires.append(torch.empty(len(ids) * fsz, dtype=torch.uint8, device=dev))
            woffs.append(torch.empty(len(ids) + 1, dtype=torch.int64, device=dev))
        out = torch.empty(n_total * fsz, dtype=torch.uint8, device="cuda:0")
        out_off = torch.empty(n_total + 1, dtype=torch.int64, device="cuda:0")
        for d in sorted(set(devs)):
            torch.cuda.synchronize(d)
        g.encode_gather(n_total, chunk, payloads, descs, wires, woffs, root=0, out=out, out_off=out_off)   # warm
        t0 = time.perf_counter()
        enc_ms, gat_ms = g.encode_gather(n_total, chunk, payloads, descs, wires, woffs, root=0, out=out,
                                         out_off=out_off)
        wall = time.perf_counter() - t0
        ok = int(out_off[-1].item()) == n_total * fsz
        for gi in sorted({0, 1, chunk, n_total // 2 + 3, n_total - 1}):
            ids = np.array([gi])
            ref, _ = oracle.encode_batch(wl.c5_payload_np(ids, size), wl.c5_desc(ids, size))
            ok &= bool(np.array_equal(out[gi * fsz: (gi + 1) * fsz].cpu().numpy(), ref))
        moved = n_total * fsz - int(wires[0].numel())
        del payloads, wires, out
        torch.cuda.empty_cache()
        try:
            host = host_leg(g, len(set(devs)))
        except Exception as e:   # noqa: BLE001  (reported, the C5 result stands)
            host = {"error": repr(e)[:300]}
        print(json.dumps({"workload": "C5: %d x %d B frames over %d ranks on %d GPU(s) of one process "
                                      "(wsg_mgpu_create), gather to device 0 by device/xGMI peer copies"
                                      % (n_total, size, ngpu, len(set(devs))),
                          "encode_ms": round(enc_ms, 3), "gather_ms": round(gat_ms, 3),
                          "wall_ms": round(wall * 1e3, 3), "bytes_into_root": moved,
                          "GBps_into_root": round(moved / (gat_ms * 1e-3) / 1e9, 1) if gat_ms > 0 else None,
                          "root_check": bool(ok), "host_decode": host}))
    finally:
        g.close()


if __name__ == "__main__":
    main()
