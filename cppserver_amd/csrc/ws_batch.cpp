// ws_batch.cpp — batched receive and send for many connections
// (include/server/ws/ws_batch.h) and their C-ABI (wsg_rx_*, wsg_tx_*).
//
// Feed() is the framing half of the reference's PrepareReceiveFrame
// (source/server/ws/ws.cpp:292-397) run on the connection's own state; the
// payload half (ws.cpp:399-406) becomes one GPU decode per Flush(), and the
// message half (ws.cpp:407-452) WebSocket::DeliverFrame, called in arrival
// order.
#include "server/ws/ws_batch.h"
#include "server/ws/ws_transport.h"
#include "ws_session_impl.h"

#include <algorithm>
#include <cstring>
#include <new>
#include <stdexcept>
#include <string>

namespace CppServer {
namespace WS {

namespace {

void check(int rc, const char* what)
{
    if (rc != WSG_OK)
        throw std::runtime_error(std::string(what) + ": " + wsg_strerror(rc));
}

} // namespace

WSReceiveBatch::WSReceiveBatch(wsg_ctx* codec) : _ctx(codec) {}

WSReceiveBatch::~WSReceiveBatch()
{
    for (Batch* b : {&_cur, &_spare}) {
        Release(b->wire);
        Release(b->out);
    }
}

void WSReceiveBatch::Grow(Pinned& b, uint64_t need)
{
    if (need <= b.cap)
        return;
    const uint64_t cap = std::max<uint64_t>(need, std::max<uint64_t>(2 * b.cap, uint64_t(1) << 20));
    void* p = nullptr;
    check(wsg_host_alloc(cap, &p), "wsg_host_alloc");
    if (b.len)
        std::memcpy(p, b.p, b.len);
    Release(b);
    b.p = static_cast<uint8_t*>(p);
    b.cap = cap;
}

void WSReceiveBatch::Release(Pinned& b)
{
    if (b.p)
        wsg_host_free(b.p);
    b.p = nullptr;
    b.cap = 0;
}

void WSReceiveBatch::Emit(WebSocket& ws, const uint8_t* frame, uint64_t total, uint32_t hdr, const uint8_t* key)
{
    Batch& b = _cur;
    Grow(b.wire, b.wire.len + total);
    uint8_t* dst = b.wire.p + b.wire.len;
    std::memcpy(dst, frame, total);
    // The reference takes the key from the bytes it pulled for the mask field
    // (ws.cpp:374-386); after a split inside an earlier header field those are
    // not the bytes at hdr-4 of its frame buffer.  The decode
    // kernel reads the key from the frame, so give it the reference's key.
    if (key)
        std::memcpy(dst + hdr - 4, key, 4);
    b.recs.push_back(Rec{&ws, int64_t(b.fs.size()), ws._ws_opcode, (frame[0] & 0x80) != 0});
    b.fs.push_back(b.wire.len);
    b.wire.len += total;
}

void WSReceiveBatch::Feed(WebSocket& ws, const void* buffer, size_t size)
{
    const uint8_t* data = static_cast<const uint8_t*>(buffer);
    auto& fb = ws._ws_receive_frame_buffer;
    do {
        if (ws._ws_frame_received)
            ws.ResetFrame();
        if (size == 0)
            return;

        // Whole frame in the input and nothing buffered: copy it straight into
        // the batch.  With every header byte present the byte-at-a-time pulls
        // below read exactly these fields, so the result is the same.
        if (fb.empty() && size >= 2) {
            const uint8_t b0 = data[0], b1 = data[1];
            const size_t len7 = b1 & 0x7F;
            const size_t ext = len7 == 126 ? 2 : len7 == 127 ? 8 : 0;
            const size_t hdr = 2 + ext + ((b1 & 0x80) ? 4 : 0);
            if (size >= hdr) {
                uint64_t len = len7;
                if (ext) {
                    len = 0;
                    for (size_t k = 0; k < ext; ++k)
                        len = (len << 8) | data[2 + k];
                }
                if (len <= size - hdr) {
                    if ((b0 & 0x0F) != 0)
                        ws._ws_opcode = b0 & 0x0F;
                    ws._ws_header_size = hdr;
                    ws._ws_payload_size = size_t(len);
                    Emit(ws, data, hdr + len, uint32_t(hdr), nullptr);
                    ws._ws_frame_received = true;
                    data += hdr + len;
                    size -= hdr + len;
                    continue;
                }
            }
        }

        // The reference's byte-at-a-time header (split headers included, Q7).
        if (fb.size() < 2 && !ws.PullHeaderField(data, size, 2))
            return;
        const uint8_t b0 = fb[0];
        const uint8_t b1 = fb[1];
        const bool masked = (b1 & 0x80) != 0;
        if ((b0 & 0x0F) != 0)
            ws._ws_opcode = b0 & 0x0F;
        const size_t len7 = b1 & 0x7F;
        const size_t ext = len7 == 126 ? 2 : len7 == 127 ? 8 : 0;
        size_t len = len7;
        if (ext) {
            if (fb.size() < 2 + ext && !ws.PullHeaderField(data, size, ext))
                return;
            len = 0;
            for (size_t k = 0; k < ext; ++k)
                len = (len << 8) | fb[2 + k];
        }
        ws._ws_header_size = 2 + ext + (masked ? 4 : 0);
        ws._ws_payload_size = len;
        if (masked && fb.size() < ws._ws_header_size && !ws.PullHeaderField(data, size, 4, ws._ws_receive_mask))
            return;

        const size_t total = ws._ws_header_size + ws._ws_payload_size;
        const size_t take = std::min(total - fb.size(), size);
        fb.insert(fb.end(), data, data + take);
        data += take;
        size -= take;
        if (fb.size() != total)
            continue;
        Emit(ws, fb.data(), total, uint32_t(ws._ws_header_size), masked ? ws._ws_receive_mask : nullptr);
        ws._ws_frame_received = true;
    } while (size > 0);
}

void WSReceiveBatch::Clear(WebSocket& ws)
{
    ws.ClearWSBuffers();
    _cur.recs.push_back(Rec{&ws, -1, 0, false});
}

void WSReceiveBatch::Forget(WebSocket& ws)
{
    for (Batch* b : {&_cur, &_spare})
        for (Rec& r : b->recs)
            if (r.ws == &ws)
                r.ws = nullptr;
}

size_t WSReceiveBatch::Flush()
{
    if (_flushing || _cur.recs.empty())
        return 0;
    std::swap(_cur, _spare);
    _cur.reset();
    Batch& b = _spare;
    _flushing = true;
    struct Done {
        WSReceiveBatch* t;
        ~Done()
        {
            t->_flushing = false;
            t->_spare.reset();
        }
    } done{this};

    const size_t n = b.fs.size();
    if (n) {
        if (n > UINT32_MAX)
            throw std::length_error("WSReceiveBatch: more than 2^32-1 frames in one flush");
        Grow(b.out, b.wire.len);
        b.info.resize(n);
        check(wsg_decode_batch_host(_ctx ? _ctx : ThreadCodec(), b.wire.p, b.wire.len, b.fs.data(), uint32_t(n),
                                    b.out.p, b.info.data()),
              "wsg_decode_batch_host");
    }
    size_t delivered = 0;
    for (size_t r = 0; r < b.recs.size(); ++r) {
        const Rec rec = b.recs[r];   // a callback may Forget() a connection: re-read each record
        if (!rec.ws)
            continue;
        if (rec.frame < 0) {
            rec.ws->ResetMessage();
            continue;
        }
        const wsg_recv_info& in = b.info[size_t(rec.frame)];
        if (in.error)
            throw std::runtime_error("WSReceiveBatch: decode rejected a framed frame");
        rec.ws->DeliverFrame(rec.opcode, rec.fin, b.out.p + in.payload_off, size_t(in.len));
        ++delivered;
    }
    return delivered;
}

// ---------------------------------------------------------------- send batch

namespace {

void grow_pinned(uint8_t*& p, uint64_t& cap, uint64_t len, uint64_t need)
{
    if (need <= cap)
        return;
    const uint64_t ncap = std::max<uint64_t>(need, std::max<uint64_t>(2 * cap, uint64_t(1) << 20));
    void* q = nullptr;
    check(wsg_host_alloc(ncap, &q), "wsg_host_alloc");
    if (len)
        std::memcpy(q, p, len);
    if (p)
        wsg_host_free(p);
    p = static_cast<uint8_t*>(q);
    cap = ncap;
}

} // namespace

WSSendBatch::WSSendBatch(wsg_ctx* codec) : _ctx(codec) {}

WSSendBatch::~WSSendBatch()
{
    if (_payload.p)
        wsg_host_free(_payload.p);
    if (_wire.p)
        wsg_host_free(_wire.p);
}

void WSSendBatch::Push(Transport* t, void* tag, uint32_t key, uint8_t opcode, bool mask, const void* buffer,
                       size_t size, int status)
{
    if (size && !buffer)
        throw std::invalid_argument("WSSendBatch: null payload");
    grow_pinned(_payload.p, _payload.cap, _payload.len, _payload.len + size);
    wsg_send_desc d{};
    d.src_off = _payload.len;
    d.len = size;
    d.key = key;
    d.status = status;
    d.opcode = opcode;
    d.mask = mask ? 1 : 0;
    if (size)
        std::memcpy(_payload.p + _payload.len, buffer, size);
    _payload.len += size;
    _desc.push_back(d);
    _recs.push_back(Rec{t, tag});
}

void WSSendBatch::Queue(Transport& transport, uint32_t key, uint8_t opcode, bool mask, const void* buffer,
                        size_t size, int status)
{
    Push(&transport, nullptr, key, opcode, mask, buffer, size, status);
}

void WSSendBatch::Queue(void* tag, uint32_t key, uint8_t opcode, bool mask, const void* buffer, size_t size,
                        int status)
{
    Push(nullptr, tag, key, opcode, mask, buffer, size, status);
}

void WSSendBatch::Forget(Transport& transport)
{
    for (Rec& r : _recs)
        if (r.transport == &transport)
            r = Rec{nullptr, nullptr};
}

void WSSendBatch::Forget(void* tag)
{
    for (Rec& r : _recs)
        if (r.tag == tag && !r.transport)
            r = Rec{nullptr, nullptr};
}

size_t WSSendBatch::Flush(Sink sink, void* user)
{
    if (_flushing || _desc.empty())
        return 0;
    if (_desc.size() > UINT32_MAX)
        throw std::length_error("WSSendBatch: more than 2^32-1 frames in one flush");
    _flushing = true;
    struct Done {
        WSSendBatch* t;
        ~Done() { t->_flushing = false; }
    } done{this};
    const uint32_t n = uint32_t(_desc.size());
    uint64_t total = 0;
    for (const wsg_send_desc& d : _desc)
        total += wsg_frame_size(d.opcode, d.mask, d.len, d.status);
    grow_pinned(_wire.p, _wire.cap, 0, std::max<uint64_t>(total, 1));
    _wire_off.resize(size_t(n) + 1);
    check(wsg_encode_batch_host(_ctx ? _ctx : ThreadCodec(), _payload.p, _payload.len, _desc.data(), n, _wire.p,
                                _wire.cap, _wire_off.data()),
          "wsg_encode_batch_host");
    // encoded: the queue is empty again before any frame is handed out, so a
    // transport's SendAsync may queue more frames (they go with the next
    // flush); if the encode failed above, everything stays queued
    std::vector<Rec> recs;
    recs.swap(_recs);
    _desc.clear();
    _payload.len = 0;
    size_t sent = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t* f = _wire.p + _wire_off[i];
        const size_t len = size_t(_wire_off[i + 1] - _wire_off[i]);
        if (recs[i].transport) {
            recs[i].transport->SendAsync(f, len);
            ++sent;
        } else if (recs[i].tag && sink) {
            sink(user, recs[i].tag, f, len);
            ++sent;
        }
    }
    return sent;
}

} // namespace WS
} // namespace CppServer

// ===========================================================================
// C-ABI (include/wsg_capi.h)
// ===========================================================================

struct wsg_rx {
    explicit wsg_rx(wsg_ctx* c) : batch(c) {}
    CppServer::WS::WSReceiveBatch batch;
};

extern "C" {

int wsg_rx_create(wsg_ctx* ctx, wsg_rx** out)
{
    if (!ctx || !out)
        return WSG_EINVAL;
    *out = new (std::nothrow) wsg_rx(ctx);
    return *out ? WSG_OK : WSG_ENOMEM;
}

int wsg_rx_destroy(wsg_rx* rx)
{
    if (!rx)
        return WSG_EINVAL;
    delete rx;
    return WSG_OK;
}

int wsg_rx_feed(wsg_rx* rx, wsg_session* s, const void* buf, size_t size)
{
    if (!rx || !s || (size && !buf))
        return WSG_EINVAL;
    try {
        rx->batch.Feed(*s, buf, size);
        return WSG_OK;
    } catch (const std::bad_alloc&) {
        return WSG_ENOMEM;
    } catch (...) {
        return WSG_ENOMEM;   // pinned batch growth failed
    }
}

int wsg_rx_clear(wsg_rx* rx, wsg_session* s)
{
    if (!rx || !s)
        return WSG_EINVAL;
    try {
        rx->batch.Clear(*s);
        return WSG_OK;
    } catch (...) {
        return WSG_ENOMEM;
    }
}

int wsg_rx_forget(wsg_rx* rx, wsg_session* s)
{
    if (!rx || !s)
        return WSG_EINVAL;
    rx->batch.Forget(*s);
    return WSG_OK;
}

int wsg_rx_pending(wsg_rx* rx, uint32_t* frames, uint64_t* bytes)
{
    if (!rx)
        return WSG_EINVAL;
    if (frames)
        *frames = uint32_t(rx->batch.frames());
    if (bytes)
        *bytes = rx->batch.bytes();
    return WSG_OK;
}

int wsg_rx_flush(wsg_rx* rx, wsg_rx_cb cb, void* user, uint32_t* delivered)
{
    if (!rx)
        return WSG_EINVAL;
    const wsg_rx_dispatch saved = g_rx_dispatch;
    g_rx_dispatch = wsg_rx_dispatch{cb, user};
    int rc = WSG_OK;
    size_t n = 0;
    try {
        n = rx->batch.Flush();
    } catch (const std::bad_alloc&) {
        rc = WSG_ENOMEM;
    } catch (...) {
        rc = WSG_EHIP;
    }
    g_rx_dispatch = saved;
    if (delivered)
        *delivered = uint32_t(n);
    return rc;
}

// ---- batched send ---------------------------------------------------------

struct wsg_tx {
    explicit wsg_tx(wsg_ctx* c) : batch(c) {}
    CppServer::WS::WSSendBatch batch;
};

int wsg_tx_create(wsg_ctx* ctx, wsg_tx** out)
{
    if (!ctx || !out)
        return WSG_EINVAL;
    *out = new (std::nothrow) wsg_tx(ctx);
    return *out ? WSG_OK : WSG_ENOMEM;
}

int wsg_tx_destroy(wsg_tx* tx)
{
    if (!tx)
        return WSG_EINVAL;
    delete tx;
    return WSG_OK;
}

int wsg_tx_queue(wsg_tx* tx, wsg_session* s, uint8_t opcode, int mask, const void* buf, size_t size, int32_t status)
{
    if (!tx || !s || (size && !buf))
        return WSG_EINVAL;
    try {
        std::scoped_lock locker(s->send_lock());   // the key is read under the send lock, as Send* does
        tx->batch.Queue(static_cast<void*>(s), s->send_key(), opcode, mask != 0, buf, size, status);
        return WSG_OK;
    } catch (...) {
        return WSG_ENOMEM;
    }
}

int wsg_tx_forget(wsg_tx* tx, wsg_session* s)
{
    if (!tx || !s)
        return WSG_EINVAL;
    tx->batch.Forget(static_cast<void*>(s));
    return WSG_OK;
}

int wsg_tx_pending(wsg_tx* tx, uint32_t* frames, uint64_t* payload_bytes)
{
    if (!tx)
        return WSG_EINVAL;
    if (frames)
        *frames = uint32_t(tx->batch.frames());
    if (payload_bytes)
        *payload_bytes = tx->batch.payload_bytes();
    return WSG_OK;
}

namespace {
struct TxSink {
    wsg_tx_sink sink;
    void* user;
};
void tx_sink(void* user, void* tag, const uint8_t* frame, size_t size)
{
    const TxSink* t = static_cast<const TxSink*>(user);
    t->sink(t->user, static_cast<wsg_session*>(tag), frame, size);
}
} // namespace

int wsg_tx_flush(wsg_tx* tx, wsg_tx_sink sink, void* user, uint32_t* sent)
{
    if (!tx || !sink)
        return WSG_EINVAL;
    TxSink t{sink, user};
    size_t n = 0;
    int rc = WSG_OK;
    try {
        n = tx->batch.Flush(tx_sink, &t);
    } catch (const std::bad_alloc&) {
        rc = WSG_ENOMEM;
    } catch (...) {
        rc = WSG_EHIP;
    }
    if (sent)
        *sent = uint32_t(n);
    return rc;
}

} // extern "C"
