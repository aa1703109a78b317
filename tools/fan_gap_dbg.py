"""Debug of test_fuzz_fanout_many_vs_oracle: which bytes outside the messages'
frames a wsg_fanout_encode_many call writes (seed from argv, library from
$WSG_LIB_PATH)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
import oracle  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402

seed = int(sys.argv[1])
rng = np.random.default_rng(9000 + seed)
m = int(rng.integers(1, 41))
pool = [int(rng.choice([int(rng.integers(0, 126)), int(rng.integers(126, 9000)), 4096, 4092, 4088]))
        for _ in range(int(rng.integers(1, 4)))]
lens = np.array([pool[int(rng.integers(0, len(pool)))] for _ in range(m)])
ops = np.array([int(rng.choice([0x82, 0x81, 0x89])) for _ in range(m)])
k = int(rng.integers(1, 3000))
mask = bool(rng.random() < 0.8)
keys = rng.integers(0, 2**32, k, dtype=np.uint64).astype(np.uint32)
src = np.zeros(m, np.uint64)
src[1:] = np.cumsum(lens[:-1] + rng.integers(0, 17, m - 1))
arena = wl.random_bytes(rng, int(src[-1] + lens[-1] + 16))
total = 0
for i in range(m):
    total = (total + 127) // 128 * 128 + k * int(ca.frame_size(int(ops[i]), mask, int(lens[i])))
c = ca.Codec(0)
wire = torch.full((total + 256,), 0xA5, dtype=torch.uint8, device="cuda")
_, off = c.fanout_many(torch.from_numpy(arena).cuda(), src, lens, ops, torch.from_numpy(keys.view(np.int32)).cuda(),
                       mask=mask, wire=wire)
c.sync()
got = wire.cpu().numpy()
covered = np.zeros(len(got), bool)
for i in range(m):
    ref = oracle.fanout_encode(arena[int(src[i]): int(src[i]) + int(lens[i])], keys, int(ops[i]), mask)
    a = int(off[i])
    covered[a: a + len(ref)] = True
    print("msg", i, "len", int(lens[i]), "op", hex(int(ops[i])), "off", a, "end", a + len(ref),
          "ok", bool(np.array_equal(got[a: a + len(ref)], ref)))
bad = np.nonzero((got != 0xA5) & ~covered)[0]
print("bytes written outside frames:", bad.size)
if bad.size:
    runs = np.split(bad, np.nonzero(np.diff(bad) != 1)[0] + 1)
    for r in runs[:20]:
        print("  [%d, %d) values %s" % (r[0], r[-1] + 1, got[r[0]: min(r[-1] + 1, r[0] + 16)].tolist()))
