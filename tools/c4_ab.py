"""C4 fan-out variants timed as bench.py times its c4 leg: one prepared
wsg_fanout_encode per step, HIP events around a region of K back-to-back
launches (no events between launches), interleaved over variants; by default the K
launches are one captured graph, replayed ($GRAPH=0: launched from Python,
where the host's ~6-7 us per call can bound a short kernel).

usage: python tools/c4_ab.py [NAME=VALUE@]path/to/libwsg.so ...   ($K, $REPS)
(NAME=VALUE is set in the environment before that library's context is made;
an empty spec is the in-tree library)
"""
import os
import statistics
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import cppserver_amd as ca  # noqa: E402
from cppserver_amd import workloads as wl  # noqa: E402


def make_codec(spec):
    env = None
    if spec and "@" in spec:
        env, _, spec = spec.partition("@")
        name, _, value = env.partition("=")
        os.environ[name] = value
    c = ca.Codec(0, lib_path=spec or None)
    if env:
        del os.environ[env.partition("=")[0]]
    return c


def main():
    specs = sys.argv[1:] or [""]
    k = int(os.environ.get("K", 200))
    payload, keys = wl.c4_fanout(4096, 10000)
    fsz = ca.frame_size(0x82, True, len(payload))
    p = torch.from_numpy(payload).cuda()
    kt = torch.from_numpy(keys.view(np.int32)).cuda()
    ref = None
    launches, wires = [], []
    graph = os.environ.get("GRAPH", "1") == "1"
    for s in specs:
        c = make_codec(s)
        w = torch.empty(fsz * len(keys), dtype=torch.uint8, device="cuda")
        launch = c.prepare_fanout(p, kt, 0x82, True, w)
        if graph:
            # K launches captured once and replayed: the host's cost per
            # launch (a ctypes call, ~6-7 us) no longer bounds the region
            launch()
            torch.cuda.synchronize()
            st = torch.cuda.Stream()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(st):
                launch()   # warm on the capture stream
                st.synchronize()
                with torch.cuda.graph(g, stream=st):
                    for _ in range(k):
                        launch()
            launch = g.replay
        launches.append(launch)
        wires.append(w)
    alg = len(payload) + 4 * len(keys) + fsz * len(keys)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = [[] for _ in specs]
    for _ in range(int(os.environ.get("REPS", 7))):
        for i, launch in enumerate(launches):
            for _ in range(1 if graph else 50):
                launch()
            torch.cuda.synchronize()
            e0.record()
            for _ in range(1 if graph else k):
                launch()
            e1.record()
            e1.synchronize()
            res[i].append(e0.elapsed_time(e1) * 1e3 / k)
    for i, s in enumerate(specs):
        ok = ""
        if "DIAG" not in s:
            got = wires[i].cpu().numpy()
            if ref is None:
                ref = got
            ok = "same bytes as the first" if np.array_equal(got, ref) else "BYTES DIFFER"
        m = statistics.median(res[i])
        print("%-60s %.3f us  frac %.4f  [%s]  %s" % (s or "(in-tree)", m, alg / (m * 1e-6) / 1e9 / 8000,
                                                    " ".join("%.2f" % x for x in res[i]), ok), flush=True)


if __name__ == "__main__":
    main()
