"""Symbolize tools/sampler.cpp output: per-function sample shares.

usage: python tools/sampler_report.py sampler.txt [--lines] [--top N]
       python tools/sampler_report.py sampler.txt.stacks --callers SUBSTRING
         (the call stacks of the samples whose function name contains it)
Measurement tool only (addr2line from binutils or the ROCm llvm tree).
"""
import collections
import os
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
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def local(mod):
        # a run on the GPU box names its copy of the tree: map it back here
        if os.path.exists(mod):
            return mod
        for part in ("cppserver_amd/", "tools/", "tests/"):
            if part in mod:
                cand = os.path.join(root, part + mod.split(part, 1)[1])
                if os.path.exists(cand):
                    return cand
        return mod

    for mod, rows in by_mod.items():
        mod_path = local(mod)
        if mod == "?" or not rows:
            for _, c in rows:
                fn[("?", mod)] += c
            continue
        # shared objects: dladdr offsets are file offsets for PIE/.so alike
        out = subprocess.run([tool, "-f", "-C", "-e", mod_path] + [hex(o) for o, _ in rows],
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


def callers(path, needle, top=25):
    """Stacks whose leaf function contains `needle`, symbolized, by count."""
    tool = addr2line()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    rows = []
    want = collections.defaultdict(set)
    for ln in open(path):
        cnt, st = ln.rstrip("\n").split(" ", 1)
        frames = [f.rsplit("@", 1) for f in st.split(";")]
        rows.append((int(cnt), frames))
        for mod, off in frames:
            want[mod].add(int(off, 16))
    names = {}
    for mod, offs in want.items():
        mp = mod
        if not os.path.exists(mp):
            for part in ("cppserver_amd/", "tools/", "tests/"):
                if part in mod and os.path.exists(os.path.join(root, part + mod.split(part, 1)[1])):
                    mp = os.path.join(root, part + mod.split(part, 1)[1])
        offs = sorted(offs)
        out = subprocess.run([tool, "-f", "-C", "-e", mp] + [hex(o) for o in offs], capture_output=True,
                             text=True).stdout.splitlines() if mod != "?" else []
        for i, o in enumerate(offs):
            nm = out[2 * i] if 2 * i < len(out) else "?"
            names[(mod, o)] = (nm if nm != "??" else mod.rsplit("/", 1)[-1] + "+" + hex(o))[:70]
    agg = collections.Counter()
    total = sum(c for c, _ in rows)
    for c, frames in rows:
        sym = [names[(m, int(o, 16))] for m, o in frames]
        if needle in sym[0]:
            agg[" < ".join(sym[:6])] += c
    print(f"stack samples {total}; leaf ~ {needle!r}: {sum(agg.values())}")
    for st, c in agg.most_common(top):
        print(f"{100.0 * c / total:6.2f}%  {st}")


if __name__ == "__main__":
    if "--callers" in sys.argv:
        callers(sys.argv[1], sys.argv[sys.argv.index("--callers") + 1])
    else:
        main()
