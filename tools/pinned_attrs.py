"""What hipPointerGetAttributes reports for the host buffers the host batch
paths see (the direct small-batch path takes a host pointer as a device
pointer only when the device address equals it): hipHostMalloc memory,
torch's pinned memory, and hipHostRegister'd memory, at the base and inside.
Prints one JSON line."""
import ctypes
import json

import numpy as np
import torch


class Attr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("device", ctypes.c_int), ("devicePointer", ctypes.c_void_p),
                ("hostPointer", ctypes.c_void_p), ("isManaged", ctypes.c_int), ("allocationFlags", ctypes.c_uint)]


def main():
    torch.cuda.init()
    hip = ctypes.CDLL("libamdhip64.so")
    out = {}

    def probe(name, p):
        a = Attr()
        rc = hip.hipPointerGetAttributes(ctypes.byref(a), ctypes.c_void_p(p))
        out[name] = dict(rc=rc, type=a.type, dev_eq_p=(a.devicePointer == p), host_eq_p=(a.hostPointer == p),
                         dev_off=(a.devicePointer or 0) - p)

    hm = ctypes.c_void_p()
    assert hip.hipHostMalloc(ctypes.byref(hm), ctypes.c_size_t(1 << 20), 0) == 0
    probe("hipHostMalloc_base", hm.value)
    probe("hipHostMalloc_inner", hm.value + 4096 + 16)
    t = torch.empty(1 << 20, dtype=torch.uint8).pin_memory()
    probe("torch_pinned_base", t.data_ptr())
    probe("torch_pinned_inner", t.data_ptr() + 4096 + 16)
    buf = np.zeros(1 << 22, dtype=np.uint8)
    base = buf.ctypes.data + (-buf.ctypes.data) % 4096
    assert hip.hipHostRegister(ctypes.c_void_p(base), ctypes.c_size_t(1 << 21), 0) == 0
    probe("hipHostRegister_base", base)
    probe("hipHostRegister_inner", base + 4096 + 16)
    hip.hipHostUnregister(ctypes.c_void_p(base))
    hip.hipHostFree(hm)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
