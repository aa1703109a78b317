"""Average HBM traffic per launch from rocprofv3 --pmc counter_collection CSVs.

FETCH_SIZE / WRITE_SIZE are kilobytes (x1024).  On gfx950 FETCH_SIZE reads
low for wide streaming reads (MI355X_MICROARCH.md §HBM: exactly half); the
correction for OUR access patterns is calibrated from membench's known-byte
kernels (`membench 1024 calib`: each launch reads and writes exactly 1 GiB,
plain and nontemporal) profiled in the same kind of pass, and applied to the
codec kernels: the nontemporal factor to k_decode (nontemporal loads), the
plain one to the encode / fan-out kernels (plain loads).

usage:
  python tools/pmc_summary.py FETCH_DIR WRITE_DIR [--calib-fetch DIR --calib-write DIR]
                              [--out JSON --config NAME --kernel K --alg-bytes N]
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(d, counter):
    per = defaultdict(list)
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row.get("Kernel_Name", "")
                per[name].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in per.items()}, {k: len(v) for k, v in per.items()}


def short(name):
    return name.split("(")[0].replace("wsg::", "").replace("void ", "")


def calibration(fetch, write, calib_bytes):
    calib = {}
    for name, v in fetch.items():
        if "k_stream" in name:
            nt = "Li3E" in name or ", 3>" in name
            calib["nt" if nt else "plain"] = (calib_bytes / v if v else None,
                                              calib_bytes / write[name] if write.get(name) else None)
    return calib


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--calib-fetch")
    ap.add_argument("--calib-write")
    ap.add_argument("--calib-bytes", type=float, default=float(1 << 30))
    ap.add_argument("--out")
    ap.add_argument("--config", default="c2")
    ap.add_argument("--kernel", default="k_decode")
    ap.add_argument("--alg-bytes", type=float, default=None)
    a = ap.parse_args()
    fetch, nf = load(a.fetch_dir, "FETCH_SIZE")
    write, nw = load(a.write_dir, "WRITE_SIZE")
    if a.calib_fetch:
        cf, _ = load(a.calib_fetch, "FETCH_SIZE")
        cw, _ = load(a.calib_write, "WRITE_SIZE")
        calib = calibration(cf, cw, a.calib_bytes)
    else:
        calib = calibration(fetch, write, a.calib_bytes)
    print("calibration (true/measured) read, write:", calib)
    rows = {}
    for name in sorted(set(fetch) | set(write)):
        f, w = fetch.get(name), write.get(name)
        print("%-40s launches=%-4s FETCH=%14.0f B  WRITE=%14.0f B" % (short(name)[:40], nf.get(name), f or 0,
                                                                      w or 0))
        rows[short(name)] = (f, w)
    k = [n for n in rows if a.kernel in n]
    if a.out and k:
        # the dominant kernel: the one with the most traffic among the matches
        name = max(k, key=lambda n: (rows[n][0] or 0) + (rows[n][1] or 0))
        f, w = rows[name]
        kind = "nt" if "k_decode" in name else "plain"
        rf, rw = calib.get(kind, (2.0, 1.0))
        hbm = (f or 0) * (rf or 2.0) + (w or 0) * (rw or 1.0)
        doc = {}
        if os.path.exists(a.out):
            with open(a.out) as fh:
                doc = json.load(fh)
        doc[a.config] = {
            "kernel": name,
            "fetch_bytes_raw": f, "write_bytes_raw": w,
            "read_correction": rf, "write_correction": rw, "correction_from": "membench k_stream " + kind,
            "hbm_bytes_per_launch": hbm,
            "alg_bytes_per_launch": a.alg_bytes,
            "hbm_over_alg": (hbm / a.alg_bytes) if a.alg_bytes else None,
            "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; KB x1024; "
                      "read/write corrections calibrated on membench kernels of known bytes",
        }
        with open(a.out, "w") as fh:
            json.dump(doc, fh, indent=1)
        print("wrote", a.out, doc[a.config])


if __name__ == "__main__":
    main()
