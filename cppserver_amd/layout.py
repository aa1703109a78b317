"""Record layouts shared by the C-ABI (include/wsg_capi.h) and its callers.

numpy structured dtypes whose byte layout is exactly ``wsg_send_desc`` and
``wsg_recv_info``; importing this module loads no native code.
"""
import numpy as np

# wsg_send_desc: one PrepareSendFrame call (reference ws.cpp:212).
SEND_DESC = np.dtype(
    [
        ("src_off", "<u8"),
        ("len", "<u8"),
        ("key", "<u4"),
        ("status", "<i4"),
        ("opcode", "u1"),
        ("mask", "u1"),
        ("_pad", "u1", (6,)),
    ]
)

# wsg_recv_info: the per-frame header arithmetic of PrepareReceiveFrame
# (reference ws.cpp:320-386).
RECV_INFO = np.dtype(
    [
        ("payload_off", "<u8"),
        ("len", "<u8"),
        ("key", "<u4"),
        ("opcode", "u1"),
        ("fin", "u1"),
        ("masked", "u1"),
        ("hdr_len", "u1"),
        ("b0", "u1"),
        ("error", "i1"),
        ("_pad", "u1", (6,)),
    ]
)

assert SEND_DESC.itemsize == 32 and RECV_INFO.itemsize == 32

# Opcode byte values (reference include/server/ws/ws.h:33-43).
WS_FIN, WS_TEXT, WS_BINARY, WS_CLOSE, WS_PING, WS_PONG = 0x80, 0x01, 0x02, 0x08, 0x09, 0x0A

# Status codes (include/wsg_capi.h).
WSG_OK, WSG_EINVAL, WSG_ETRUNC, WSG_ENOMEM, WSG_EHIP = 0, -22, -61, -12, -5

# Callback kinds (include/wsg_capi.h WSG_CB_*).
CB_RECEIVED, CB_CLOSE, CB_PING, CB_PONG = 1, 2, 3, 4


def key_from_bytes(b):
    """_ws_send_mask[0..3] -> the little-endian uint32 the ABI carries."""
    b = bytes(b)
    return b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24


def frame_size(opcode, mask, length, status=0):
    """Bytes PrepareSendFrame emits (reference ws.cpp:215-252)."""
    prefix = (opcode & WS_CLOSE) == WS_CLOSE and (length > 0 or status != 0)
    body = length + (2 if prefix else 0)
    hdr = 2 if body < 126 else 4 if body < 65536 else 10
    return hdr + (4 if mask else 0) + body


def frame_sizes(desc):
    """frame_size over a SEND_DESC array, vectorized (uint64 per frame)."""
    op = desc["opcode"].astype(np.uint64)
    length = desc["len"].astype(np.uint64)
    prefix = ((op & WS_CLOSE) == WS_CLOSE) & ((length > 0) | (desc["status"] != 0))
    body = length + np.where(prefix, 2, 0).astype(np.uint64)
    hdr = np.where(body < 126, 2, np.where(body < 65536, 4, 10)).astype(np.uint64)
    return hdr + np.where(desc["mask"] != 0, 4, 0).astype(np.uint64) + body
