"""Symbolize tools/sampler.cpp output: per-function sample shares.

usage: python tools/sampler_report.py sampler.txt [--lines] [--top N]
Measurement tool only (addr2line from binutils or the ROCm llvm tree).
"""
import collections
import shutil
import subprocess
import sys


def addr2line():
    for c in ("addr2line", "/opt/rocm/lib/llvm/bin/llvm-addr2line"):
        if shutil.which(c) or c.startswith("/"):
            return c
    raise SystemExit("no addr2line")


def main():
    path = sys.argv[1]
    lines = "--lines" in sys.argv
    top = 40
    if "--top" in sys.argv:
        top = int(sys.argv[sys.argv.index("--top") + 1])
    by_mod = collections.defaultdict(list)
    total = 0
    for ln in open(path):
        mod, off, cnt = ln.rsplit(" ", 2)
        by_mod[mod].append((int(off, 16), int(cnt)))
        total += int(cnt)
    tool = addr2line()
    fn = collections.Counter()
    for mod, rows in by_mod.items():
        if mod == "?" or not rows:
            for _, c in rows:
                fn[("?", mod)] += c
            continue
        # shared objects: dladdr offsets are file offsets for PIE/.so alike
        out = subprocess.run([tool, "-f", "-C", "-e", mod] + [hex(o) for o, _ in rows],
                             capture_output=True, text=True).stdout.splitlines()
        short = mod.rsplit("/", 1)[-1]
        for i, (_, c) in enumerate(rows):
            name = out[2 * i] if 2 * i < len(out) else "?"
            loc = out[2 * i + 1] if 2 * i + 1 < len(out) else "?"
            key = f"{name}  [{loc.rsplit('/', 1)[-1]}]" if lines else name
            fn[(short, key[:150])] += c
    print(f"total samples {total}")
    for (mod, name), c in fn.most_common(top):
        print(f"{100.0 * c / total:6.2f}%  {mod:<18} {name}")


if __name__ == "__main__":
    main()
