"""cppserver_amd — MI355X-native WebSocket frame codec (CppServer's WS hot path).

The product is the C-ABI library ``_build/libwsg.so`` (include/wsg_capi.h):
gfx950 HIP kernels for batched header pack/unpack and payload mask/unmask.
This module is a thin ctypes binding over that ABI for Python callers and the
test-suite; torch is used only to own device memory and streams.

There is no CPU fallback: if the library or a GPU is missing, ``Codec``
raises instead of computing anything.
"""
import ctypes
import os

import numpy as np

from .layout import (  # noqa: F401  (re-exported)
    CB_CLOSE, CB_PING, CB_PONG, CB_RECEIVED, RECV_INFO, SEND_DESC, WS_BINARY, WS_CLOSE, WS_FIN, WS_PING,
    WS_PONG, WS_TEXT, WSG_EHIP, WSG_EINVAL, WSG_ENOMEM, WSG_ETRUNC, WSG_OK, frame_size, frame_sizes, key_from_bytes,
)

_HERE = os.path.dirname(os.path.abspath(__file__))
# $WSG_LIB_PATH: another build of the same ABI for a one-off A/B check (tools/);
# unset, the in-tree library
LIB_PATH = os.environ.get("WSG_LIB_PATH") or os.path.join(_HERE, "_build", "libwsg.so")
ROOT = os.path.dirname(_HERE)
HEADERS = [os.path.join(ROOT, "include", "wsg_capi.h")]

_lib = None


class WSGError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        msg = lib().wsg_strerror(code).decode() if _lib is not None else str(code)
        super().__init__("%s failed: %s (%d)" % (what or "wsg", msg, code))


def lib(path=None):
    """Load the HIP codec library; raise loudly if it was not built.

    `path` loads another build of the same ABI (A/B tuning); default is the
    in-tree library."""
    global _lib
    if path is None and _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise ImportError(
            "cppserver_amd: native library %s is missing; run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(or `make -C cppserver_amd`). There is no CPU fallback." % p
        )
    L = ctypes.CDLL(p)
    vp, u32, u64, i32, sz, ci = (ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32,
                                 ctypes.c_size_t, ctypes.c_int)
    sig = {
        "wsg_abi_version": (ci, []),
        "wsg_strerror": (ctypes.c_char_p, [ci]),
        "wsg_create": (ci, [ci, ctypes.POINTER(vp)]),
        "wsg_destroy": (ci, [vp]),
        "wsg_sync": (ci, [vp, vp]),
        "wsg_stream": (vp, [vp]),
        "wsg_decode_batch": (ci, [vp, vp, u64, vp, u32, vp, vp, vp]),
        "wsg_encode_batch": (ci, [vp, vp, vp, u32, vp, u64, vp, vp]),
        "wsg_fanout_encode": (ci, [vp, vp, u64, vp, u32, ctypes.c_uint8, ci, vp, u64, vp]),
        "wsg_fanout_encode_many": (ci, [vp, vp, vp, vp, vp, u32, vp, u32, ci, vp, u64, vp, vp]),
        "wsg_xor_host": (ci, [vp, vp, vp, sz, u32, u32]),
        "wsg_decode_batch_host": (ci, [vp, vp, u64, vp, u32, vp, vp]),
        "wsg_encode_batch_host": (ci, [vp, vp, u64, vp, u32, vp, u64, vp]),
        "wsg_host_alloc": (ci, [sz, ctypes.POINTER(vp)]),
        "wsg_host_free": (ci, [vp]),
        "wsg_frame_size": (u64, [ctypes.c_uint8, ci, u64, i32]),
        "wsg_header_pack": (ci, [ctypes.c_uint8, ci, u64, i32, u32, vp]),
        "wsg_header_unpack": (ci, [vp, u64, vp]),
        "wsg_ws_accept": (ci, [ctypes.c_char_p, sz, ctypes.c_char_p, sz]),
        "wsg_session_create": (ci, [vp, ctypes.POINTER(vp)]),
        "wsg_session_destroy": (ci, [vp]),
        "wsg_session_set_send_key": (ci, [vp, u32]),
        "wsg_session_prepare_send": (ci, [vp, ctypes.c_uint8, ci, vp, sz, i32, vp, sz, ctypes.POINTER(sz)]),
        "wsg_session_prepare_receive": (ci, [vp, vp, sz, vp, vp]),
        "wsg_session_required": (sz, [vp]),
        "wsg_session_clear": (ci, [vp]),
        "wsg_rx_create": (ci, [vp, ctypes.POINTER(vp)]),
        "wsg_rx_destroy": (ci, [vp]),
        "wsg_rx_feed": (ci, [vp, vp, vp, sz]),
        "wsg_rx_clear": (ci, [vp, vp]),
        "wsg_rx_forget": (ci, [vp, vp]),
        "wsg_rx_pending": (ci, [vp, ctypes.POINTER(u32), ctypes.POINTER(u64)]),
        "wsg_rx_set_devices": (ci, [vp, vp, ci]),
        "wsg_rx_flush": (ci, [vp, vp, vp, ctypes.POINTER(u32)]),
        "wsg_tx_create": (ci, [vp, ctypes.POINTER(vp)]),
        "wsg_tx_destroy": (ci, [vp]),
        "wsg_tx_queue": (ci, [vp, vp, ctypes.c_uint8, ci, vp, sz, i32]),
        "wsg_tx_forget": (ci, [vp, vp]),
        "wsg_tx_pending": (ci, [vp, ctypes.POINTER(u32), ctypes.POINTER(u64)]),
        "wsg_tx_set_devices": (ci, [vp, vp, ci]),
        "wsg_tx_flush": (ci, [vp, vp, vp, ctypes.POINTER(u32)]),
        "wsg_mgpu_create": (ci, [vp, ci, ctypes.POINTER(vp)]),
        "wsg_mgpu_unique_id": (ci, [vp]),
        "wsg_mgpu_create_rank": (ci, [ci, vp, ci, ci, ctypes.POINTER(vp)]),
        "wsg_mgpu_destroy": (ci, [vp]),
        "wsg_mgpu_info": (ci, [vp, ctypes.POINTER(ci), ctypes.POINTER(ci), ctypes.POINTER(ci)]),
        "wsg_mgpu_ctx": (vp, [vp, ci]),
        "wsg_mgpu_shard_count": (u64, [u64, u32, ci, ci]),
        "wsg_mgpu_encode_gather": (ci, [vp, u64, u32, vp, vp, vp, vp, vp, vp, ci, vp, u64, vp, vp]),
        "wsg_decode_batch_host_multi": (ci, [vp, ci, vp, u64, vp, u32, vp, vp]),
        "wsg_encode_batch_host_multi": (ci, [vp, ci, vp, u64, vp, u32, vp, u64, vp]),
        "wsg_mgpu_decode_batch_host": (ci, [vp, vp, u64, vp, u32, vp, vp]),
        "wsg_mgpu_encode_batch_host": (ci, [vp, vp, u64, vp, u32, vp, u64, vp]),
        "wsg_timing_enable": (ci, [vp, ci]),
        "wsg_timing_read": (ci, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(u64), ci]),
        "wsg_timing_minmax": (ci, [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
        "wsg_lane_stats": (ci, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64), ctypes.POINTER(ci)]),
        "wsg_lane_events": (ci, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
    }
    for name, (res, args) in sig.items():
        if path is not None and not hasattr(L, name):
            continue   # an older A/B build of the library (tools/): bind what it has
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = L
    return L


def _np_ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc, what):
    if rc != 0:
        raise WSGError(rc, what)


# ---- host helpers (pure host functions of the ABI; no device needed) ------
def header_pack(opcode, mask, length, status=0, key=0):
    buf = (ctypes.c_uint8 * 16)()
    n = lib().wsg_header_pack(opcode, 1 if mask else 0, length, status, key, buf)
    if n < 0:
        raise WSGError(n, "wsg_header_pack")
    return bytes(buf[:n])


def header_unpack(data):
    data = bytes(data)
    info = np.zeros(1, dtype=RECV_INFO)
    rc = lib().wsg_header_unpack(data, len(data), _np_ptr(info))
    return rc, info[0]


class _Pinned:
    """Owner of a wsg_host_alloc block; freed when the last view dies."""

    def __init__(self, nbytes):
        self.ptr = ctypes.c_void_p()
        _check(lib().wsg_host_alloc(nbytes, ctypes.byref(self.ptr)), "wsg_host_alloc")

    def __del__(self):
        if self.ptr:
            lib().wsg_host_free(self.ptr)
            self.ptr = None


def pinned_empty(nbytes, dtype=np.uint8):
    """numpy array in page-locked host memory (DMA without staging)."""
    owner = _Pinned(max(int(nbytes), 1))
    buf = (ctypes.c_uint8 * max(int(nbytes), 1)).from_address(owner.ptr.value)
    buf._owner = owner   # the numpy view keeps buf alive, buf keeps the block alive
    return np.frombuffer(buf, dtype=np.uint8)[: int(nbytes)].view(dtype)


def abi_frame_size(opcode, mask, length, status=0):
    return int(lib().wsg_frame_size(opcode, 1 if mask else 0, length, status))


class Codec:
    """A wsg_ctx bound to one HIP device.

    Batch methods take torch CUDA (HIP) tensors resident in HBM and run
    asynchronously on ``stream`` (default: torch's current stream); call
    :meth:`sync` before reading results on the host.
    """

    def __init__(self, device=0, lib_path=None):
        import torch

        self._torch = torch
        self._L = lib(lib_path)
        if not torch.cuda.is_available():
            raise WSGError(WSG_EHIP, "Codec: no HIP device visible")
        self.device = torch.device("cuda", device)
        ctx = ctypes.c_void_p()
        _check(self._L.wsg_create(device, ctypes.byref(ctx)), "wsg_create")
        self._ctx = ctx

    def close(self):
        if getattr(self, "_ctx", None):
            self._L.wsg_destroy(self._ctx)
            self._ctx = None

    __del__ = close

    # -- streams / sync ----------------------------------------------------
    def _stream(self, stream):
        if stream is None:
            stream = self._torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))

    def sync(self, stream=None):
        """Synchronize and raise WSGError on a latched data-dependent error."""
        _check(self._L.wsg_sync(self._ctx, self._stream(stream)), "wsg_sync")

    def sync_status(self, stream=None):
        return self._L.wsg_sync(self._ctx, self._stream(stream))

    # -- batch decode (unmask) ----------------------------------------------
    def decode_batch(self, wire, frame_start, out=None, info=None, stream=None):
        """Unmask every frame of ``wire`` (uint8 CUDA tensor) whose starts are
        ``frame_start`` (int64 CUDA tensor).  Returns (out, info_bytes)."""
        t = self._torch
        n = int(frame_start.numel())
        if out is None:
            out = t.empty_like(wire)
        if info is None:
            info = t.empty(max(n, 1) * RECV_INFO.itemsize, dtype=t.uint8, device=wire.device)
        rc = self._L.wsg_decode_batch(self._ctx, ctypes.c_void_p(wire.data_ptr()), wire.numel(),
                                      ctypes.c_void_p(frame_start.data_ptr()), n,
                                      ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(info.data_ptr()),
                                      self._stream(stream))
        _check(rc, "wsg_decode_batch")
        return out, info

    def prepare_decode(self, wire, frame_start, out, info, stream=None):
        """wsg_decode_batch on fixed buffers (a server's batch arena), with
        the ctypes arguments bound once: returns a callable that launches one
        decode per call (asynchronous, like decode_batch)."""
        n = int(frame_start.numel())
        if int(out.numel()) < int(wire.numel()) or int(info.numel()) < n * RECV_INFO.itemsize:
            raise WSGError(WSG_EINVAL, "prepare_decode: out or info smaller than the batch needs")
        fn = self._L.wsg_decode_batch
        args = (self._ctx, ctypes.c_void_p(wire.data_ptr()), ctypes.c_uint64(wire.numel()),
                ctypes.c_void_p(frame_start.data_ptr()), ctypes.c_uint32(n), ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(info.data_ptr()))
        keep = (wire, frame_start, out, info)   # the buffers live as long as the callable
        fixed = None if stream is None else self._stream(stream)

        def launch():
            # stream=None: torch's current stream at each launch, as decode_batch
            rc = fn(*args, fixed if fixed is not None else self._stream(None))
            if rc != 0:
                raise WSGError(rc, "wsg_decode_batch")
            return keep

        return launch

    def prepare_fanout(self, payload, keys, opcode, mask, wire, length=None, stream=None):
        """wsg_fanout_encode on fixed buffers with the ctypes arguments bound
        once (the multicast loop of a server); returns a launch callable."""
        k = int(keys.numel())
        length = int(payload.numel()) if length is None else int(length)
        if frame_size(opcode, mask, length) * k > int(wire.numel()):
            raise WSGError(WSG_ENOMEM, "prepare_fanout: wire smaller than %d frames" % k)
        fn = self._L.wsg_fanout_encode
        args = (self._ctx, ctypes.c_void_p(payload.data_ptr()), ctypes.c_uint64(length),
                ctypes.c_void_p(keys.data_ptr()), ctypes.c_uint32(k), ctypes.c_uint8(opcode), 1 if mask else 0,
                ctypes.c_void_p(wire.data_ptr()), ctypes.c_uint64(wire.numel()))
        keep = (payload, keys, wire)
        fixed = None if stream is None else self._stream(stream)

        def launch():
            # stream=None: torch's current stream at each launch, as fanout
            rc = fn(*args, fixed if fixed is not None else self._stream(None))
            if rc != 0:
                raise WSGError(rc, "wsg_fanout_encode")
            return keep

        return launch

    # -- batch encode (mask) --------------------------------------------------
    def encode_batch(self, payload, desc, wire=None, wire_cap=None, wire_off=None, stream=None):
        """Encode frames ``desc`` (uint8 CUDA tensor of n*32 bytes) whose data
        live in ``payload``.  Returns (wire, wire_off int64[n+1])."""
        t = self._torch
        n = int(desc.numel() // SEND_DESC.itemsize)
        if wire is None:
            wire = t.empty(max(int(wire_cap), 16), dtype=t.uint8, device=desc.device)
        cap = int(wire.numel()) if wire_cap is None else int(wire_cap)
        if cap > int(wire.numel()):
            raise WSGError(WSG_EINVAL, "encode_batch: wire_cap %d exceeds the wire tensor (%d bytes)"
                           % (cap, int(wire.numel())))
        if wire_off is None:
            wire_off = t.empty(n + 1, dtype=t.int64, device=desc.device)
        rc = self._L.wsg_encode_batch(self._ctx, ctypes.c_void_p(payload.data_ptr()),
                                      ctypes.c_void_p(desc.data_ptr()), n, ctypes.c_void_p(wire.data_ptr()),
                                      cap, ctypes.c_void_p(wire_off.data_ptr()), self._stream(stream))
        _check(rc, "wsg_encode_batch")
        return wire, wire_off

    def fanout(self, payload, keys, opcode, mask=True, wire=None, length=None, stream=None):
        t = self._torch
        k = int(keys.numel())
        length = int(payload.numel()) if length is None else int(length)
        fsz = frame_size(opcode, mask, length)
        if wire is None:
            wire = t.empty(max(fsz * k, 16), dtype=t.uint8, device=payload.device)
        rc = self._L.wsg_fanout_encode(self._ctx, ctypes.c_void_p(payload.data_ptr()), length,
                                       ctypes.c_void_p(keys.data_ptr()), k, opcode, 1 if mask else 0,
                                       ctypes.c_void_p(wire.data_ptr()), wire.numel(), self._stream(stream))
        _check(rc, "wsg_fanout_encode")
        return wire

    def fanout_many(self, payload, src_off, lens, opcodes, keys, mask=True, wire=None, stream=None):
        """m messages (payload[src_off[i]:][:lens[i]], opcode opcodes[i]) x k
        keys in one call (wsg_fanout_encode_many).  Returns (wire, wire_off):
        message i's k frames start at wire_off[i] (host numpy, m + 1)."""
        t = self._torch
        src_off = np.ascontiguousarray(src_off, dtype=np.uint64)
        lens = np.ascontiguousarray(lens, dtype=np.uint64)
        opcodes = np.ascontiguousarray(opcodes, dtype=np.uint8)
        m, k = len(lens), int(keys.numel())
        need = 0
        for i in range(m):
            need = (need + 127) // 128 * 128 + frame_size(int(opcodes[i]), mask, int(lens[i])) * k
        if wire is None:
            wire = t.empty(max(need, 16), dtype=t.uint8, device=keys.device)
        off = np.zeros(m + 1, dtype=np.uint64)
        rc = self._L.wsg_fanout_encode_many(self._ctx, ctypes.c_void_p(payload.data_ptr()), _np_ptr(src_off),
                                            _np_ptr(lens), _np_ptr(opcodes), m, ctypes.c_void_p(keys.data_ptr()), k,
                                            1 if mask else 0, ctypes.c_void_p(wire.data_ptr()), wire.numel(),
                                            _np_ptr(off), self._stream(stream))
        _check(rc, "wsg_fanout_encode_many")
        return wire, off

    # -- host-staged paths ----------------------------------------------------
    def xor_host(self, data, key, phase=0):
        src = bytes(data)
        dst = ctypes.create_string_buffer(max(len(src), 1))
        _check(self._L.wsg_xor_host(self._ctx, src, dst, len(src), key, phase), "wsg_xor_host")
        return dst.raw[: len(src)]

    def decode_batch_host(self, wire, frame_start, out=None):
        wire = np.ascontiguousarray(wire, dtype=np.uint8)
        fs = np.ascontiguousarray(frame_start, dtype=np.uint64)
        if out is None:
            out = np.empty(max(len(wire), 1), dtype=np.uint8)
        info = np.zeros(max(len(fs), 1), dtype=RECV_INFO)
        rc = self._L.wsg_decode_batch_host(self._ctx, _np_ptr(wire), len(wire), _np_ptr(fs), len(fs),
                                           _np_ptr(out), _np_ptr(info))
        return rc, out[: len(wire)], info[: len(fs)]

    def encode_batch_host(self, payload, desc, wire=None):
        """Host-staged batch encode: returns (rc, wire bytes, wire_off)."""
        payload = np.ascontiguousarray(payload, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=SEND_DESC)
        n = len(desc)
        total = int(frame_sizes(desc).sum()) if n else 0
        if wire is None:
            wire = np.empty(max(total, 1), dtype=np.uint8)
        off = np.zeros(n + 1, dtype=np.uint64)
        rc = self._L.wsg_encode_batch_host(self._ctx, _np_ptr(payload) if len(payload) else None, len(payload),
                                           _np_ptr(desc) if n else None, n, _np_ptr(wire), len(wire), _np_ptr(off))
        return rc, wire[:total], off

    # -- measurement hooks ----------------------------------------------------
    def timing(self, on=True, every=1):
        """Time the dominant kernel of every `every`-th batch call (HIP events)."""
        _check(self._L.wsg_timing_enable(self._ctx, int(every) if on else 0), "wsg_timing_enable")

    def timing_minmax(self):
        """(shortest, longest) timed launch in ms since the last reset."""
        lo, hi = ctypes.c_double(), ctypes.c_double()
        _check(self._L.wsg_timing_minmax(self._ctx, ctypes.byref(lo), ctypes.byref(hi)), "wsg_timing_minmax")
        return lo.value, hi.value

    def lane_stats(self):
        """(requests this context put on the lane, launches of the device's
        lane, running: 1 / 0 / -1 given up) — wsg_lane_stats."""
        r, l, on = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_int()
        _check(self._L.wsg_lane_stats(self._ctx, ctypes.byref(r), ctypes.byref(l), ctypes.byref(on)),
               "wsg_lane_stats")
        return r.value, l.value, on.value

    def lane_events(self):
        """(give-ups, re-arms) of the device's lane — wsg_lane_events."""
        g, r = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._L.wsg_lane_events(self._ctx, ctypes.byref(g), ctypes.byref(r)), "wsg_lane_events")
        return g.value, r.value

    def timing_read(self, reset=True):
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        _check(self._L.wsg_timing_read(self._ctx, ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0),
               "wsg_timing_read")
        return ms.value, n.value


RECEIVE_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t,
                              ctypes.c_int)
RX_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8),
                         ctypes.c_size_t, ctypes.c_int)


class Session:
    """One connection's codec state through the C-ABI (wsg_session_*): the
    reference WebSocket mix-in with its payload XOR on the GPU."""

    def __init__(self, codec, send_key=0):
        self._L = lib()
        self._codec = codec          # keeps the ctx alive
        s = ctypes.c_void_p()
        _check(self._L.wsg_session_create(codec._ctx, ctypes.byref(s)), "wsg_session_create")
        self._s = s
        self.set_send_key(send_key)
        self._events = []

        def _cb(user, kind, data, size, status):
            self._events.append((kind, ctypes.string_at(data, size) if size else b"", status))

        self._cb = RECEIVE_CB(_cb)

    def close(self):
        if getattr(self, "_s", None):
            self._L.wsg_session_destroy(self._s)
            self._s = None

    __del__ = close

    def set_send_key(self, key):
        _check(self._L.wsg_session_set_send_key(self._s, key), "wsg_session_set_send_key")

    def prepare_send(self, opcode, mask, payload=b"", status=0):
        buf = bytes(payload)
        cap = frame_size(opcode, mask, len(buf), status)
        out = ctypes.create_string_buffer(max(cap, 1))
        n = ctypes.c_size_t()
        _check(self._L.wsg_session_prepare_send(self._s, opcode, 1 if mask else 0, buf, len(buf), status, out, cap,
                                                ctypes.byref(n)), "wsg_session_prepare_send")
        return out.raw[: n.value]

    def prepare_receive(self, data):
        buf = bytes(data)
        _check(self._L.wsg_session_prepare_receive(self._s, buf if buf else None, len(buf), self._cb, None),
               "wsg_session_prepare_receive")

    def events(self, clear=True):
        ev = list(self._events)
        if clear:
            self._events.clear()
        return ev

    def required(self):
        return self._L.wsg_session_required(self._s)

    def clear(self):
        _check(self._L.wsg_session_clear(self._s), "wsg_session_clear")


class RxBatch:
    """Batched receive over many sessions through the C-ABI (wsg_rx_*): feed()
    frames each session's stream on the host, flush() unmasks the batch in one
    GPU pass and fires every session's callbacks in arrival order.  Events are
    (session, kind, payload bytes, status)."""

    def __init__(self, codec):
        self._L = lib()
        self._codec = codec
        rx = ctypes.c_void_p()
        _check(self._L.wsg_rx_create(codec._ctx, ctypes.byref(rx)), "wsg_rx_create")
        self._rx = rx
        self._events = []
        self._by_ptr = {}

        def _cb(user, sess, kind, data, size, status):
            self._events.append((self._by_ptr.get(sess), kind, ctypes.string_at(data, size) if size else b"",
                                 status))

        self._cb = RX_CB(_cb)

    def close(self):
        if getattr(self, "_rx", None):
            self._L.wsg_rx_destroy(self._rx)
            self._rx = None

    __del__ = close

    def _reg(self, session):
        self._by_ptr[session._s.value] = session
        return session._s

    def feed(self, session, data):
        buf = bytes(data)
        _check(self._L.wsg_rx_feed(self._rx, self._reg(session), buf if buf else None, len(buf)), "wsg_rx_feed")

    def clear(self, session):
        _check(self._L.wsg_rx_clear(self._rx, self._reg(session)), "wsg_rx_clear")

    def forget(self, session):
        _check(self._L.wsg_rx_forget(self._rx, self._reg(session)), "wsg_rx_forget")

    def pending(self):
        f, b = ctypes.c_uint32(), ctypes.c_uint64()
        _check(self._L.wsg_rx_pending(self._rx, ctypes.byref(f), ctypes.byref(b)), "wsg_rx_pending")
        return f.value, b.value

    def set_devices(self, devices):
        """Spread every flush over these GPUs (wsg_rx_set_devices)."""
        d = (ctypes.c_int * max(len(devices), 1))(*devices)
        _check(self._L.wsg_rx_set_devices(self._rx, d, len(devices)), "wsg_rx_set_devices")

    def flush(self):
        n = ctypes.c_uint32()
        _check(self._L.wsg_rx_flush(self._rx, self._cb, None, ctypes.byref(n)), "wsg_rx_flush")
        return n.value

    def events(self, clear=True):
        ev = list(self._events)
        if clear:
            self._events.clear()
        return ev


TX_SINK = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint8), ctypes.c_size_t)


class TxBatch:
    """Batched send over many sessions through the C-ABI (wsg_tx_*): queue()
    records a PrepareSendFrame call, flush() encodes all of them in one GPU
    pass and returns [(session, frame bytes)] in queue order."""

    def __init__(self, codec):
        self._L = lib()
        self._codec = codec
        tx = ctypes.c_void_p()
        _check(self._L.wsg_tx_create(codec._ctx, ctypes.byref(tx)), "wsg_tx_create")
        self._tx = tx
        self._out = []
        self._by_ptr = {}

        def _sink(user, sess, frame, size):
            self._out.append((self._by_ptr.get(sess), ctypes.string_at(frame, size)))

        self._sink = TX_SINK(_sink)

    def close(self):
        if getattr(self, "_tx", None):
            self._L.wsg_tx_destroy(self._tx)
            self._tx = None

    __del__ = close

    def queue(self, session, opcode, mask, payload=b"", status=0):
        self._by_ptr[session._s.value] = session
        buf = bytes(payload)
        _check(self._L.wsg_tx_queue(self._tx, session._s, opcode, 1 if mask else 0, buf if buf else None, len(buf),
                                    status), "wsg_tx_queue")

    def forget(self, session):
        _check(self._L.wsg_tx_forget(self._tx, session._s), "wsg_tx_forget")

    def pending(self):
        f, b = ctypes.c_uint32(), ctypes.c_uint64()
        _check(self._L.wsg_tx_pending(self._tx, ctypes.byref(f), ctypes.byref(b)), "wsg_tx_pending")
        return f.value, b.value

    def set_devices(self, devices):
        """Spread every flush over these GPUs (wsg_tx_set_devices)."""
        d = (ctypes.c_int * max(len(devices), 1))(*devices)
        _check(self._L.wsg_tx_set_devices(self._tx, d, len(devices)), "wsg_tx_set_devices")

    def flush(self):
        n = ctypes.c_uint32()
        self._out = []
        _check(self._L.wsg_tx_flush(self._tx, self._sink, None, ctypes.byref(n)), "wsg_tx_flush")
        out, self._out = self._out, []
        if len(out) != n.value:
            raise WSGError(WSG_EINVAL, "wsg_tx_flush: %d frames handed out, %d reported" % (len(out), n.value))
        return out


def info_to_numpy(info_tensor, n):
    """Device info bytes -> numpy RECV_INFO records."""
    return info_tensor[: n * RECV_INFO.itemsize].cpu().numpy().view(RECV_INFO)


def desc_to_tensor(desc, device):
    import torch

    desc = np.ascontiguousarray(desc, dtype=SEND_DESC)
    return torch.from_numpy(desc.view(np.uint8).copy()).to(device)


def _ptr_array(ptrs):
    return (ctypes.c_void_p * len(ptrs))(*[ctypes.c_void_p(p) for p in ptrs])


def _host_decode_args(wire, frame_start, out):
    wire = np.ascontiguousarray(wire, dtype=np.uint8)
    fs = np.ascontiguousarray(frame_start, dtype=np.uint64)
    if out is None:
        out = np.empty(max(len(wire), 1), dtype=np.uint8)
    info = np.zeros(max(len(fs), 1), dtype=RECV_INFO)
    return wire, fs, out, info


def _host_encode_args(payload, desc, wire):
    payload = np.ascontiguousarray(payload, dtype=np.uint8)
    desc = np.ascontiguousarray(desc, dtype=SEND_DESC)
    total = int(frame_sizes(desc).sum()) if len(desc) else 0
    if wire is None:
        wire = np.empty(max(total, 1), dtype=np.uint8)
    off = np.zeros(len(desc) + 1, dtype=np.uint64)
    return payload, desc, wire, off, total


def decode_batch_host_multi(codecs, wire, frame_start, out=None):
    """wsg_decode_batch_host_multi: one host batch over several contexts
    (their GPUs' PCIe links at once).  Returns (rc, out, info) like
    Codec.decode_batch_host."""
    wire, fs, out, info = _host_decode_args(wire, frame_start, out)
    ctxs = _ptr_array([c._ctx.value for c in codecs])
    rc = lib().wsg_decode_batch_host_multi(ctxs, len(codecs), _np_ptr(wire), len(wire), _np_ptr(fs), len(fs),
                                           _np_ptr(out), _np_ptr(info))
    return rc, out[: len(wire)], info[: len(fs)]


def encode_batch_host_multi(codecs, payload, desc, wire=None):
    """wsg_encode_batch_host_multi: returns (rc, wire bytes, wire_off)."""
    payload, desc, wire, off, total = _host_encode_args(payload, desc, wire)
    ctxs = _ptr_array([c._ctx.value for c in codecs])
    n = len(desc)
    rc = lib().wsg_encode_batch_host_multi(ctxs, len(codecs), _np_ptr(payload) if len(payload) else None,
                                           len(payload), _np_ptr(desc) if n else None, n, _np_ptr(wire), len(wire),
                                           _np_ptr(off))
    return rc, wire[:total], off


class MultiGPU:
    """The multi-GPU entry of the C-ABI (wsg_mgpu_*): round-robin shards of a
    frame batch encoded on their GPUs and gathered to one rank.

    MultiGPU(devices=[0, 1, ...]) drives every rank from this process, one
    rank per listed device (a device may be listed more than once): chunks
    move to the root by device copies (xGMI peer copies between GPUs);
    MultiGPU.rank(device, uid, rank, world) is one rank of a multi-process
    group over RCCL (uid from MultiGPU.unique_id() on rank 0, handed to
    every rank)."""

    ID_BYTES = 128

    def __init__(self, devices=None, _handle=None):
        self._L = lib()
        if _handle is not None:
            self._g = _handle
        else:
            devs = (ctypes.c_int * len(devices))(*devices)
            g = ctypes.c_void_p()
            _check(self._L.wsg_mgpu_create(devs, len(devices), ctypes.byref(g)), "wsg_mgpu_create")
            self._g = g
        w, nl, fr = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(self._L.wsg_mgpu_info(self._g, ctypes.byref(w), ctypes.byref(nl), ctypes.byref(fr)), "wsg_mgpu_info")
        self.world, self.nlocal, self.first_rank = w.value, nl.value, fr.value

    @staticmethod
    def unique_id():
        buf = (ctypes.c_uint8 * MultiGPU.ID_BYTES)()
        _check(lib().wsg_mgpu_unique_id(buf), "wsg_mgpu_unique_id")
        return bytes(buf)

    @classmethod
    def rank(cls, device, uid, rank, world):
        g = ctypes.c_void_p()
        buf = (ctypes.c_uint8 * cls.ID_BYTES).from_buffer_copy(bytes(uid))
        _check(lib().wsg_mgpu_create_rank(device, buf, rank, world, ctypes.byref(g)), "wsg_mgpu_create_rank")
        return cls(_handle=g)

    @staticmethod
    def shard_count(n_total, chunk, world, rank):
        return int(lib().wsg_mgpu_shard_count(n_total, chunk, world, rank))

    def close(self):
        if getattr(self, "_g", None):
            self._L.wsg_mgpu_destroy(self._g)
            self._g = None

    __del__ = close

    def _ctx(self, i):
        ctx = self._L.wsg_mgpu_ctx(self._g, int(i))
        if not ctx:
            raise WSGError(WSG_EINVAL, "wsg_mgpu_ctx(%d)" % i)
        return ctypes.c_void_p(ctx)

    def timing(self, on=True, every=1, i=0):
        """Time the dominant kernel of local rank i's encodes (its context's
        HIP events, as Codec.timing): k_encode_mask inside encode_gather."""
        _check(self._L.wsg_timing_enable(self._ctx(i), int(every) if on else 0), "wsg_timing_enable")

    def timing_read(self, reset=True, i=0):
        ms, n = ctypes.c_double(), ctypes.c_uint64()
        _check(self._L.wsg_timing_read(self._ctx(i), ctypes.byref(ms), ctypes.byref(n), 1 if reset else 0),
               "wsg_timing_read")
        return ms.value, n.value

    def encode_gather(self, n_total, chunk, payloads, descs, wires, wire_offs, root=0, out=None, out_off=None):
        """Per local rank (lists of CUDA tensors): payload arena, descriptor
        bytes (n_local * 32), wire buffer, wire_off (n_local + 1 int64).  On
        the root: `out` (uint8) and `out_off` (int64, n_total + 1, or None).
        Returns (encode_ms, gather_ms)."""
        k = self.nlocal
        n_local = (ctypes.c_uint32 * k)(*[int(d.numel()) // SEND_DESC.itemsize for d in descs])
        caps = (ctypes.c_uint64 * k)(*[int(w.numel()) for w in wires])
        times = (ctypes.c_double * 2)()
        rc = self._L.wsg_mgpu_encode_gather(
            self._g, int(n_total), int(chunk), _ptr_array([p.data_ptr() for p in payloads]),
            _ptr_array([d.data_ptr() for d in descs]), n_local, _ptr_array([w.data_ptr() for w in wires]), caps,
            _ptr_array([o.data_ptr() for o in wire_offs]), int(root),
            ctypes.c_void_p(out.data_ptr() if out is not None else 0), int(out.numel()) if out is not None else 0,
            ctypes.c_void_p(out_off.data_ptr() if out_off is not None else 0), times)
        _check(rc, "wsg_mgpu_encode_gather")
        return times[0], times[1]

    def decode_batch_host(self, wire, frame_start, out=None):
        """wsg_mgpu_decode_batch_host: a host batch over this process's GPUs."""
        wire, fs, out, info = _host_decode_args(wire, frame_start, out)
        rc = self._L.wsg_mgpu_decode_batch_host(self._g, _np_ptr(wire), len(wire), _np_ptr(fs), len(fs),
                                                _np_ptr(out), _np_ptr(info))
        return rc, out[: len(wire)], info[: len(fs)]

    def encode_batch_host(self, payload, desc, wire=None):
        payload, desc, wire, off, total = _host_encode_args(payload, desc, wire)
        n = len(desc)
        rc = self._L.wsg_mgpu_encode_batch_host(self._g, _np_ptr(payload) if len(payload) else None, len(payload),
                                                _np_ptr(desc) if n else None, n, _np_ptr(wire), len(wire),
                                                _np_ptr(off))
        return rc, wire[:total], off

