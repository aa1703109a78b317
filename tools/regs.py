"""Register/occupancy report for k_decode and source variants with paths cut
out (which path sets the kernel's VGPR count).  Compiles for gfx950 only
(no GPU needed).

usage: python tools/regs.py
"""
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "cppserver_amd", "csrc", "wsg_kernels.hip")


def report(text, tag, kernel="_ZN3wsg8k_decode"):
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "k.hip")
        with open(path, "w") as f:
            f.write(text)
        r = subprocess.run(
            ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I" + os.path.join(ROOT, "include"),
             "-I" + os.path.join(ROOT, "cppserver_amd", "csrc"), "--cuda-device-only", "-S", "-o",
             os.path.join(d, "k.s"), path, "-Rpass-analysis=kernel-resource-usage"],
            capture_output=True, text=True)
    out = r.stderr
    i = out.find("Function Name: " + kernel)
    block = out[i:i + 2500] if i >= 0 else ""

    def g(k):
        m = re.search(k + r": (\d+)", block)
        return m.group(1) if m else "?"
    print("%-28s VGPR %s SGPR %s sspill %s vspill %s occ %s" % (
        tag, g(" VGPRs"), g("TotalSGPRs"), g("SGPRs Spill"), g("VGPRs Spill"), g(r"Occupancy \[waves/SIMD\]")))


def cut(text, marker):
    assert marker in text, marker
    return text.replace(marker, "return;\n" + marker, 1)   # inside process_tile


if __name__ == "__main__":
    src = open(SRC).read()
    staged = "    // staged: payload segments in LDS"
    boundary = "        // boundary: per chunk"
    report(src, "full")
    report(cut(src, staged), "no-staged")
    report(cut(src, boundary), "no-boundary")
    report(cut(cut(src, staged), boundary), "no-staged-no-boundary")
