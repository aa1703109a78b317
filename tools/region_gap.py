"""bench.py's own C2 timed region (bench.timed_region on bench.Workload),
repeated in one process: wall - events per region with the roctx range on
and off, right after the oracle spot check and after a plain host pause.
Diagnostic only.  usage: python tools/region_gap.py [trials]
"""
import contextlib
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.argv = [sys.argv[0], "--steps", "20", "--warmup", "5", "--no-configs", "--no-extras", "--no-cpu"] + sys.argv[2:]
import bench  # noqa: E402


class _GcStub:
    """bench.py's gc calls in the region, each kept or made a no-op."""

    def __init__(self, collect, disable):
        import gc

        self._gc, self._c, self._d = gc, collect, disable

    def collect(self):
        if self._c:
            self._gc.collect()

    def disable(self):
        if self._d:
            self._gc.disable()

    def enable(self):
        self._gc.enable()


def main(trials):
    import torch

    import cppserver_amd as ca

    args = bench.parse()
    rank, world, local = bench.dist_setup(args)
    device = torch.device("cuda", local)
    codec = ca.Codec(local)
    w = bench.Workload(args, codec, rank, device)
    real_marker = bench.marker
    rows = {}
    def inline_region():
        # the bare region on the same workload: no barrier, gc or marker
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        e1.record()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record()
        for _ in range(args.steps):
            w.step()
        e1.record()
        t_sub = time.perf_counter()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        return {"elapsed": el, "region_event_ms": e0.elapsed_time(e1), "submit_ms": (t_sub - t0) * 1e3}

    for t in range(trials):
        for variant in ("inline", "pause", "pause-nogc", "pause-disable", "inline-after"):
            if variant.startswith("inline"):
                time.sleep(1.0)
                for _ in range(args.warmup):
                    w.step()
                codec.sync()
                r = inline_region()
                gap = r["elapsed"] * 1e6 - r["region_event_ms"] * 1e3
                rows.setdefault(variant, []).append((gap, r["submit_ms"] * 1e3))
                continue
            if variant.startswith("spot"):
                w.spot_check()
            else:
                time.sleep(1.0)
            bench.marker = real_marker if variant.endswith("marker") else (lambda name: contextlib.nullcontext())
            bench.gc = _GcStub(collect=variant == "pause", disable=variant in ("pause", "pause-disable"))
            for _ in range(args.warmup):
                w.step()
            codec.sync()
            r = bench.timed_region(w, args.steps, world, device)
            gap = r["elapsed"] * 1e6 - r["region_event_ms"] * 1e3
            rows.setdefault(variant, []).append((gap, r["submit_ms"] * 1e3))
    bench.marker = real_marker
    for v, xs in rows.items():
        gaps = [g for g, _ in xs]
        subs = [s for _, s in xs]
        print("%-13s wall-events median %6.1f us  max %6.1f us  min %6.1f us  submit median %6.1f us"
              % (v, statistics.median(gaps), max(gaps), min(gaps), statistics.median(subs)), flush=True)
    codec.close()


if __name__ == "__main__":
    main(int(os.environ.get("GAP_TRIALS", "6")))
