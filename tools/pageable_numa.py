"""The host-inclusive C2 decode from pageable buffers (wsg_decode_batch_host:
the caller's bytes copied into page-locked staging by the library's copy
workers and back) with this process bound to a NUMA node before any GPU or
torch call: `gpu` (the GPU's node), `other`, or `none`.  One JSON line.

usage: python tools/pageable_numa.py gpu|other|none"""
import json
import os
import sys
import time


def node_cpus(node):
    with open("/sys/devices/system/node/node%d/cpulist" % node) as f:
        spec = f.read().strip()
    cpus = set()
    for part in spec.split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return cpus & os.sched_getaffinity(0)


def gpu_node():
    # the first GPU's PCI function, from sysfs (no GPU call yet)
    import glob
    for d in sorted(glob.glob("/sys/bus/pci/devices/*")):
        try:
            if open(os.path.join(d, "vendor")).read().strip() == "0x1002" and \
               open(os.path.join(d, "class")).read().strip()[:4] in ("0x03", "0x12"):
                return int(open(os.path.join(d, "numa_node")).read().strip())
        except OSError:
            continue
    return -1


mode = sys.argv[1]
g = gpu_node()
nodes = sorted(int(p[len("/sys/devices/system/node/node"):]) for p in
               __import__("glob").glob("/sys/devices/system/node/node[0-9]*"))
target = None
if mode == "gpu" and g >= 0:
    target = g
elif mode == "other" and g >= 0:
    target = next((n for n in nodes if n != g), None)
if target is not None:
    cpus = node_cpus(target)
    if cpus:
        os.sched_setaffinity(0, cpus)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402
import oracle  # noqa: E402

rng = np.random.default_rng(5)
n, size = 4096, 65536
desc, total = wl.ragged_desc(rng, np.full(n, size))
desc["mask"] = True
payload = wl.random_bytes(rng, total)
wire, off = oracle.encode_batch(payload, desc)
fs = off[:-1].copy()
out = np.empty_like(wire)
c = ca.Codec(0)
rc, _, _ = c.decode_batch_host(wire, fs, out=out)
assert rc == 0
reps = 5
t0 = time.perf_counter()
for _ in range(reps):
    c.decode_batch_host(wire, fs, out=out)
dt = (time.perf_counter() - t0) / reps
ok = bool(np.array_equal(out[int(fs[0]) + 14: int(fs[0]) + 14 + 64],
                         oracle.decode_batch(wire[: int(fs[1])], np.zeros(1, np.uint64))[1][14:78]))
print(json.dumps({"mode": mode, "gpu_node": g, "bound_node": target, "pageable_GiBps": round(n * size / dt / 2**30, 2),
                  "check": ok}))
