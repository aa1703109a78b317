"""Builds the pre-0b854e9 copy pattern for the one-off check of
tests/test_gpu_c5.py::test_mgpu_rank_form_copy_ordering:
the gather's host->device rounds as plain hipMemcpy (null stream) in the
product, and the loopback double's copies as plain hipMemcpy, both from the
CURRENT sources (so the $WSG_TEST_NULL_SPIN_US hook is in them).  Outputs:
cppserver_amd/_build/var/oldcopy/libwsg.so and
tests/cpp/_build/var/libloopback_oldcopy.so (CPU-side build, in-tree).

On the box:  WSG_LIB_PATH=<oldcopy libwsg.so> WSG_RCCL_LIB=<old double>
WSG_RANK_JOB=ordering [WSG_TEST_NULL_SPIN_US=50000] python tests/mgpu_rank_job.py
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TMP = os.path.join(ROOT, "cppserver_amd", "_build", "var", "oldcopy", "src")


def revert_mgpu(src):
    # hipMemcpyAsync(dst, src, n, H2D, stream_of(x)) + hipStreamSynchronize -> hipMemcpy(dst, src, n, H2D)
    pat = re.compile(r"hipMemcpyAsync\(([^;]*?),\s*hipMemcpyHostToDevice,\s*stream_of\([^)]*\)\)\);\s*"
                     r"WSG_HIP\(hipStreamSynchronize\(stream_of\([^)]*\)\)\);", re.S)
    out, n1 = pat.subn(r"hipMemcpy(\1, hipMemcpyHostToDevice));", src)
    pat2 = re.compile(r"hipMemcpyAsync\((root_l->d_goff[^;]*?),\s*hipMemcpyHostToDevice,\s*stream_of\(\*root_l\)\) "
                      r"!= hipSuccess \|\|\s*hipStreamSynchronize\(stream_of\(\*root_l\)\) != hipSuccess\)", re.S)
    out, n2 = pat2.subn(r"hipMemcpy(\1, hipMemcpyHostToDevice) != hipSuccess)", out)
    assert (n1, n2) == (2, 1), (n1, n2)
    return out


def revert_loopback(src):
    a = ("hipMemcpyAsync(op.dst, s->src, op.bytes, hipMemcpyDefault, op.stream) == hipSuccess &&\n"
         "                            hipStreamSynchronize(op.stream) == hipSuccess;")
    assert a in src
    src = src.replace(a, "hipMemcpy(op.dst, s->src, op.bytes, hipMemcpyDefault) == hipSuccess;")
    b = "hipMemcpyDefault, op.stream) != hipSuccess)"
    assert src.count(b) == 1
    return src.replace(b, "hipMemcpyDefault) != hipSuccess)")


def main():
    os.makedirs(TMP, exist_ok=True)
    csrc = os.path.join(ROOT, "cppserver_amd", "csrc")
    with open(os.path.join(csrc, "wsg_mgpu.cpp")) as f:
        m = revert_mgpu(f.read())
    with open(os.path.join(TMP, "wsg_mgpu.cpp"), "w") as f:
        f.write(m)
    with open(os.path.join(ROOT, "tests", "cpp", "loopback_rccl.cpp")) as f:
        lb = revert_loopback(f.read())
    with open(os.path.join(TMP, "loopback_rccl.cpp"), "w") as f:
        f.write(lb)
    out = os.path.dirname(TMP)
    h = "/opt/rocm/bin/hipcc"
    inc = ["-I" + os.path.join(ROOT, "include"), "-I" + csrc]
    objs = []
    for name in ("wsg_kernels.hip", "wsg_capi.hip", "ws.cpp", "ws_api.cpp", "ws_batch.cpp", "http.cpp", "tls.cpp",
                 "wss.cpp", "wsg_mgpu.cpp"):
        src = os.path.join(TMP if name == "wsg_mgpu.cpp" else csrc, name)
        o = os.path.join(out, name + ".o")
        arch = ["--offload-arch=gfx950"] if name.endswith(".hip") else []
        subprocess.run([h, "-O3", "-std=c++17", "-fPIC"] + arch + inc + ["-c", src, "-o", o], check=True)
        objs.append(o)
    subprocess.run([h, "--offload-arch=gfx950", "-shared", "-o", os.path.join(out, "libwsg.so")] + objs +
                   ["-lssl", "-lcrypto", "-ldl", "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx"], check=True)
    lbo = os.path.join(ROOT, "tests", "cpp", "_build", "var")
    os.makedirs(lbo, exist_ok=True)
    subprocess.run([h, "-O2", "-std=c++17", "-fPIC", "-shared", "-o", os.path.join(lbo, "libloopback_oldcopy.so"),
                    os.path.join(TMP, "loopback_rccl.cpp"), "-pthread"], check=True)
    print(os.path.join(out, "libwsg.so"))
    print(os.path.join(lbo, "libloopback_oldcopy.so"))


if __name__ == "__main__":
    sys.exit(main())
