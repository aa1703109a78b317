"""Split a rocprofv3 kernel trace of `python bench.py` by bench leg (round 3):
bench.py wraps every leg's timed region in a roctx range
("bench.<cfg>.timed"); run under `rocprofv3 --kernel-trace --marker-trace`,
every kernel that starts inside a range belongs to that leg.  Writes, per
leg and kernel, the launch count and average / min / max / stdev duration
(JSON), and compares them with the bench line's own event timings.

usage: python tools/trace_split.py TRACE_DIR BENCH_JSON OUT_JSON
"""
import csv
import glob
import json
import os
import statistics
import sys


def rows(d, suffix):
    out = []
    for path in glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True):
        with open(path) as f:
            out.extend(csv.DictReader(f))
    return out


def short(name):
    return name.split("(")[0].replace("void ", "").replace("wsg::", "")


def main():
    tdir, bench_json, out_json = sys.argv[1:4]
    kernels = rows(tdir, "kernel_trace.csv")
    markers = rows(tdir, "marker_api_trace.csv")
    ranges = []
    for m in markers:
        name = m.get("Function") or m.get("Message") or m.get("Name") or ""
        if name.startswith("bench.") and name.endswith(".timed"):
            ranges.append((name.split(".")[1], int(m["Start_Timestamp"]), int(m["End_Timestamp"])))
    legs = {}
    for k in kernels:
        s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
        for cfg, a, b in ranges:
            if a <= s <= b:
                legs.setdefault(cfg, {}).setdefault(short(k["Kernel_Name"]), []).append((e - s) / 1e6)   # ms
    with open(bench_json) as f:
        line = json.loads(f.read().strip().splitlines()[-1])
    doc = {"trace_dir": os.path.basename(tdir.rstrip("/")), "ranges": len(ranges), "legs": {}}
    for cfg, ks in sorted(legs.items()):
        leg = {}
        for name, ds in sorted(ks.items(), key=lambda kv: -sum(kv[1])):
            leg[name] = {"calls": len(ds), "avg_ms": round(statistics.mean(ds), 5), "min_ms": round(min(ds), 5),
                         "max_ms": round(max(ds), 5), "stdev_ms": round(statistics.pstdev(ds), 5)}
        obj = line if cfg == "c2" else line.get(cfg, {})   # the headline leg is C2
        rf = obj.get("roofline", {})
        checks = []
        for h in (rf.get("halves") or [rf]):
            k = h.get("kernel")
            match = [n for n in leg if k and n.startswith(k)]
            if match:
                tr = leg[match[0]]["avg_ms"]
                checks.append({"kernel": k, "bench_avg_ms": h.get("avg_kernel_ms"), "trace_avg_ms": tr,
                               "ratio": round(h["avg_kernel_ms"] / tr, 4) if tr else None})
        doc["legs"][cfg] = {"kernels": leg, "bench_vs_trace": checks}
    with open(out_json, "w") as f:
        json.dump(doc, f, indent=1)
    for cfg, d in doc["legs"].items():
        for c in d["bench_vs_trace"]:
            print("%-4s %-18s bench %.5f ms  trace %.5f ms  ratio %.4f" % (cfg, c["kernel"], c["bench_avg_ms"],
                                                                       c["trace_avg_ms"], c["ratio"]))


if __name__ == "__main__":
    main()
