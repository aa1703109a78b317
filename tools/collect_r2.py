"""Copy one round_artifacts_r2.sh run (one or more gpurun_out/ directories)
into profiles/r2/: bench lines, rocprofv3 kernel stats, PMC counter CSVs,
and the derived HBM traffic per launch (profiles/pmc_traffic.json via
tools/pmc_summary.py, calibrated on the membench known-byte kernels of the
same run).

usage: python tools/collect_r2.py gpurun_out/art_a [gpurun_out/art_b ...]
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(ROOT, "profiles", "r2")
KERNEL = {"c2": "k_decode", "c3": "k_encode_mask", "c4": "k_fanout", "c4x16": "k_fanout", "c5": "k_encode_mask"}


def main():
    srcs = sys.argv[1:]
    calib = [s for s in srcs if os.path.isdir(os.path.join(s, "pmc_calib_FETCH_SIZE"))][0]
    for k in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(os.path.join(calib, "pmc_calib_%s" % k, "**", "*counter_collection.csv"), recursive=True):
            shutil.copy(f, os.path.join(DST, "pmc_membench_calib_%s.csv" % k))
    pmc_json = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    for src in srcs:
        for out in sorted(glob.glob(os.path.join(src, "bench_*.out"))):
            cfg = os.path.basename(out)[len("bench_"):-len(".out")]
            line = open(out).read().strip().splitlines()[-1]
            doc = json.loads(line)
            for f in glob.glob(os.path.join(src, "trace_%s" % cfg, "*kernel_stats.csv")):
                shutil.copy(f, os.path.join(DST, "%s_kernel_stats.csv" % cfg))
            for k in ("FETCH_SIZE", "WRITE_SIZE"):
                for f in glob.glob(os.path.join(src, "pmc_%s_%s" % (cfg, k), "**", "*counter_collection.csv"),
                                   recursive=True):
                    # the codec's kernels only (C5's run also profiles the
                    # torch kernels that make its 16 GiB of payload)
                    rows = list(csv.reader(open(f)))
                    ki = rows[0].index("Kernel_Name")
                    with open(os.path.join(DST, "pmc_%s_%s.csv" % (cfg, k)), "w", newline="") as fh:
                        csv.writer(fh).writerows([rows[0]] + [r for r in rows[1:] if "wsg::" in r[ki]])
            subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"),
                            os.path.join(src, "pmc_%s_FETCH_SIZE" % cfg), os.path.join(src, "pmc_%s_WRITE_SIZE" % cfg),
                            "--calib-fetch", os.path.join(calib, "pmc_calib_FETCH_SIZE"),
                            "--calib-write", os.path.join(calib, "pmc_calib_WRITE_SIZE"),
                            "--out", pmc_json, "--config", cfg, "--kernel", KERNEL[cfg],
                            "--alg-bytes", str(doc["roofline"]["alg_bytes_per_launch"])], check=True,
                           stdout=subprocess.DEVNULL)
            # the bench line as run, with roofline.traffic from this run's PMC passes
            traffic = json.load(open(pmc_json))[cfg]["hbm_bytes_per_launch"]
            doc["roofline"]["traffic"] = traffic
            with open(os.path.join(DST, "bench_%s.json" % cfg), "w") as f:
                f.write(json.dumps(doc) + "\n")
            print(cfg, doc["value"], doc["roofline"]["avg_kernel_ms"], doc["roofline"]["frac"],
                  "traffic/alg %.4f" % (traffic / doc["roofline"]["alg_bytes_per_launch"]))
    shutil.copy(pmc_json, os.path.join(DST, "pmc_traffic.json"))


if __name__ == "__main__":
    main()
