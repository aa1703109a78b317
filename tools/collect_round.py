"""Copy one tools/round_artifacts.sh run into profiles/<round>/: the bench line
as the driver runs it, the rocprofv3 kernel stats of the same command and
its per-leg split (tools/trace_split.py), the PMC counter CSVs (codec
kernels only) and the HBM traffic per launch they give
(profiles/pmc_traffic.json via tools/pmc_summary.py, calibrated on the
membench known-byte kernels of the same run).

usage: python tools/collect_round.py gpurun_out/art_r4 r4
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "profiles", sys.argv[2] if len(sys.argv) > 2 else "r4")
# pmc_traffic.json key -> (config run, kernel)
KEYS = {"c2": ("c2", "k_decode"), "c3": ("c3", "k_encode_mask"), "c3_dec": ("c3", "k_decode"),
        "c4": ("c4", "k_fanout"), "c5": ("c5", "k_encode_mask")}


def main():
    src = sys.argv[1]
    os.makedirs(DST, exist_ok=True)
    py = sys.executable
    tools = os.path.join(ROOT, "tools")
    if os.path.exists(os.path.join(src, "bench.out")):
        line = open(os.path.join(src, "bench.out")).read().strip().splitlines()[-1]
        with open(os.path.join(DST, "bench.json"), "w") as f:
            f.write(line + "\n")
        for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(DST, "kernel_stats.csv"))
        for f in glob.glob(os.path.join(src, "trace", "**", "*marker_api_stats.csv"), recursive=True):
            shutil.copy(f, os.path.join(DST, "marker_stats.csv"))
        subprocess.run([py, os.path.join(tools, "trace_split.py"), os.path.join(src, "trace"),
                        os.path.join(DST, "bench.json"), os.path.join(DST, "trace_by_leg.json")], check=True)
    for k in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(os.path.join(src, "pmc_calib_%s" % k, "**", "*counter_collection.csv"), recursive=True):
            shutil.copy(f, os.path.join(DST, "pmc_membench_calib_%s.csv" % k))
    pmc_json = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    for key, (cfg, kernel) in KEYS.items():
        fd, wd = os.path.join(src, "pmc_%s_FETCH_SIZE" % cfg), os.path.join(src, "pmc_%s_WRITE_SIZE" % cfg)
        if not os.path.isdir(fd):
            continue
        for k, d in (("FETCH_SIZE", fd), ("WRITE_SIZE", wd)):
            for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
                rows = list(csv.reader(open(f)))
                ki = rows[0].index("Kernel_Name")
                with open(os.path.join(DST, "pmc_%s_%s.csv" % (cfg, k)), "w", newline="") as fh:
                    csv.writer(fh).writerows([rows[0]] + [r for r in rows[1:] if "wsg::" in r[ki]])
        bench = json.loads(open(os.path.join(src, "pmc_%s_FETCH_SIZE.out" % cfg)).read().strip().splitlines()[-1])
        rf = bench["roofline"]
        alg = [h for h in (rf.get("halves") or [rf]) if h["kernel"].startswith(kernel)][0]["alg_bytes_per_launch"]
        subprocess.run([py, os.path.join(tools, "pmc_summary.py"), fd, wd,
                        "--calib-fetch", os.path.join(src, "pmc_calib_FETCH_SIZE"),
                        "--calib-write", os.path.join(src, "pmc_calib_WRITE_SIZE"),
                        "--out", pmc_json, "--config", key, "--kernel", kernel, "--alg-bytes", str(alg)],
                       check=True, stdout=subprocess.DEVNULL)
        t = json.load(open(pmc_json))[key]
        print("%-7s %-16s HBM bytes/launch %.4g  / algorithmic %.4f" % (key, t["kernel"], t["hbm_bytes_per_launch"],
                                                                          t["hbm_over_alg"]))
    shutil.copy(pmc_json, os.path.join(DST, "pmc_traffic.json"))


if __name__ == "__main__":
    main()
