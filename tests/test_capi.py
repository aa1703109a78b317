"""C-ABI library checks that need no GPU: it loads, exports every function
include/*.h declares, its host-side header helpers agree with the oracle, and
device entry points fail loudly (no CPU fallback) when no GPU is present."""
import ctypes
import glob
import os
import re

import numpy as np
import pytest

import cppserver_amd as ca
import oracle
from cppserver_amd.layout import frame_size

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"\b(wsg_\w+)\s*\(", text):
            if not re.search(r"typedef[^;]*\(\s*\*\s*" + m.group(1), text):
                names.add(m.group(1))
    return sorted(names)


def test_header_declares_entry_points():
    names = declared_functions()
    for must in ["wsg_create", "wsg_decode_batch", "wsg_encode_batch", "wsg_fanout_encode",
                 "wsg_header_pack", "wsg_header_unpack", "wsg_session_prepare_send",
                 "wsg_session_prepare_receive"]:
        assert must in names


@pytest.mark.parametrize("name", declared_functions())
def test_library_exports(name):
    lib = ctypes.CDLL(ca.LIB_PATH)
    assert hasattr(lib, name), name


def test_abi_version():
    assert ca.lib().wsg_abi_version() == 3


@pytest.mark.parametrize("opcode,mask,length,status", [
    (0x81, True, 0, 0), (0x82, False, 125, 0), (0x82, True, 126, 0), (0x82, True, 65535, 0),
    (0x82, True, 65536, 0), (0x88, True, 0, 1000), (0x88, False, 123, 1001), (0x88, True, 124, 5),
    (0x89, True, 3, 0), (0x8A, False, 65534, 0), (0x80, True, 1 << 33, 0), (0x02, False, 7, -3),
])
def test_header_pack_matches_oracle(opcode, mask, length, status):
    key = 0xA1B2C3D4
    hdr = ca.header_pack(opcode, mask, length, status, key)
    assert ca.abi_frame_size(opcode, mask, length, status) == frame_size(opcode, mask, length, status)
    if length <= 70000:
        s = oracle.Session(key)
        frame = s.prepare_send(opcode, mask, bytes(length), status)
        assert frame[: len(hdr)] == hdr
        assert len(frame) == ca.abi_frame_size(opcode, mask, length, status)
    rc, info = ca.header_unpack(hdr + bytes(4))
    assert rc == 0
    assert info["hdr_len"] == len(hdr)
    assert info["masked"] == int(mask)
    assert info["key"] == (key if mask else 0)
    assert info["b0"] == opcode and info["opcode"] == opcode & 0x0F and info["fin"] == opcode >> 7


def test_header_unpack_truncated():
    assert ca.header_unpack(b"\x82")[0] == ca.WSG_ETRUNC
    assert ca.header_unpack(b"\x82\xfe\x00")[0] == ca.WSG_ETRUNC
    assert ca.header_unpack(b"\x82\xff" + bytes(11))[0] == ca.WSG_ETRUNC
    assert ca.header_unpack(b"\x82\x85\x01\x02\x03")[0] == ca.WSG_ETRUNC


def test_no_cpu_fallback_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    ctx = ctypes.c_void_p()
    assert ca.lib().wsg_create(0, ctypes.byref(ctx)) == ca.WSG_EHIP
    with pytest.raises(ca.WSGError):
        ca.Codec(0)


def test_strerror_names_codes():
    for code in (ca.WSG_OK, ca.WSG_EINVAL, ca.WSG_ETRUNC, ca.WSG_ENOMEM, ca.WSG_EHIP):
        assert ca.lib().wsg_strerror(code)


def test_loopback_rccl_double_exports():
    """The RCCL test double (tests/cpp/loopback_rccl.cpp) the rank-form GPU
    test loads through $WSG_RCCL_LIB has every entry point wsg_mgpu.cpp's
    rccl() looks up; without one of them the product would refuse it."""
    path = os.path.join(ROOT, "tests", "cpp", "_build", "libloopback_rccl.so")
    if not os.path.exists(path):
        pytest.skip("tests/cpp not built")
    src = open(os.path.join(ROOT, "cppserver_amd", "csrc", "wsg_mgpu.cpp")).read()
    wanted = re.findall(r'sym\(r\.\w+, "(nccl\w+)"\)', src)
    assert len(wanted) == 9
    lib = ctypes.CDLL(path)
    for name in wanted + ["loopback_rccl_errors"]:
        assert hasattr(lib, name), name
