import json, os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
import cppserver_amd as ca
from cppserver_amd import workloads as wl
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from lane_timeout_job import xor_ref
c = ca.Codec(0)
rng = np.random.default_rng(11)
t0 = time.perf_counter()
for i in range(3000):
    ln = int(rng.integers(1, 41)) if i % 5 else int(rng.integers(41, 300))
    data = bytes(wl.random_bytes(rng, ln))
    key, phase = int(rng.integers(0, 2**32)), int(rng.integers(0, 4))
    got = np.frombuffer(c.xor_host(data, key, phase), np.uint8)
    ok = np.array_equal(got, xor_ref(data, key, phase))
    if i % 250 == 0 or not ok:
        print(i, ok, c.lane_stats(), round(time.perf_counter() - t0, 4), flush=True)
print("end", c.lane_stats(), round(time.perf_counter() - t0, 4))
