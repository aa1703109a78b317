"""C5 footprint sweep (round 3): k_encode_mask on 1/8, 1/4, 1/2 and the whole
1 Mi x 16 KiB job (payload made in HBM, as bench.py does), per encode grid
cap, interleaved in one process.  Diagnostic only.

usage: python tools/c5_sweep.py [cap1,cap2,...]   (WSG_ENC_BLOCKS_PER_CU values; default 1024,65536)
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
    caps = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "1024,65536").split(",")]
    codecs = []
    for cap in caps:
        os.environ["WSG_ENC_BLOCKS_PER_CU"] = str(cap)
        codecs.append(ca.Codec(0))
    os.environ.pop("WSG_ENC_BLOCKS_PER_CU", None)
    size = 16384
    fsz = ca.frame_size(0x82, True, size)
    for frac in (8, 4, 2, 1):
        n = (1 << 20) // frac
        ids = np.arange(n, dtype=np.int64)
        payload = wl.c5_payload_torch(ids, size, device="cuda")
        desc = ca.desc_to_tensor(wl.c5_desc(ids, size), "cuda")
        wire = torch.empty(n * fsz, dtype=torch.uint8, device="cuda")
        woff = torch.empty(n + 1, dtype=torch.int64, device="cuda")
        alg = n * size + n * fsz
        res = [[] for _ in caps]
        for rep in range(3):
            for ci, c in enumerate(codecs):
                for _ in range(2):
                    c.encode_batch(payload, desc, wire=wire, wire_cap=wire.numel(), wire_off=woff)
                c.timing(True, 1)
                c.timing_read()
                for _ in range(6):
                    c.encode_batch(payload, desc, wire=wire, wire_cap=wire.numel(), wire_off=woff)
                ms, k = c.timing_read()
                c.timing(False)
                res[ci].append(ms / k)
        for cap, r in zip(caps, res):
            m = statistics.median(r)
            print("frames=%7d (1/%d) enc_blocks_per_cu=%6d  k_encode_mask %.4f ms  %.0f GB/s  frac %.3f" % (
                n, frac, cap, m, alg / m / 1e6, alg / m / 1e6 / 8000), flush=True)
        del payload, desc, wire, woff
        torch.cuda.empty_cache()
    for c in codecs:
        c.close()


if __name__ == "__main__":
    main()
