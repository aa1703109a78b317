// ws_batch.cpp — batched receive and send for many connections
// (include/server/ws/ws_batch.h) and their C-ABI (wsg_rx_*, wsg_tx_*).
//
// Feed() is the framing half of the reference's PrepareReceiveFrame
// (source/server/ws/ws.cpp:292-397) run on the connection's own state; the
// payload half (ws.cpp:399-406) becomes one GPU decode per Flush(), and the
// message half (ws.cpp:407-452) WebSocket::DeliverFrame, called in arrival
// order.
#include "server/ws/ws_batch.h"
#include "wsg_env.h"
#include "server/ws/ws_transport.h"
#include "ws_session_impl.h"
#include "wsg_frame.h"

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <stdexcept>
#include <thread>
#include <string>

namespace CppServer {
namespace WS {

namespace {

void check(int rc, const char* what)
{
    if (rc != WSG_OK)
        throw std::runtime_error(std::string(what) + ": " + wsg_strerror(rc));
}

// One owned context per device (replacing `ctxs`); contexts of devices
// already held are kept.
void set_devices(std::vector<wsg_ctx*>& ctxs, const std::vector<int>& devices)
{
    std::vector<wsg_ctx*> next;
    try {
        for (int d : devices) {
            wsg_ctx* c = nullptr;
            check(wsg_create(d, &c), "wsg_create");
            next.push_back(c);
        }
    } catch (...) {
        for (wsg_ctx* c : next)
            wsg_destroy(c);
        throw;
    }
    for (wsg_ctx* c : ctxs)
        wsg_destroy(c);
    ctxs.swap(next);
}

} // namespace

WSReceiveBatch::WSReceiveBatch(wsg_ctx* codec) : _ctx(codec) {}

WSReceiveBatch::~WSReceiveBatch()
{
    for (Batch* b : {&_cur, &_spare}) {
        Release(b->wire);
        Release(b->out);
    }
    for (wsg_ctx* c : _devs)
        wsg_destroy(c);
}

void WSReceiveBatch::SetDevices(const std::vector<int>& devices)
{
    std::scoped_lock l(_lock);
    if (_flushing)
        throw std::logic_error("WSReceiveBatch::SetDevices during a flush");
    set_devices(_devs, devices);
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
    // masked frames (MASK bit) with a nonzero key need the unmask pass
    if ((frame[1] & 0x80) && (dst[hdr - 4] | dst[hdr - 3] | dst[hdr - 2] | dst[hdr - 1]))
        b.keyed = true;
    b.recs.push_back(Rec{&ws, int64_t(b.fs.size()), ws._ws_opcode, (frame[0] & 0x80) != 0, hdr});
    b.fs.push_back(b.wire.len);
    b.wire.len += total;
    _n_frames.store(b.fs.size(), std::memory_order_relaxed);
    _n_bytes.store(b.wire.len, std::memory_order_relaxed);
}

void WSReceiveBatch::Feed(WebSocket& ws, const void* buffer, size_t size)
{
    std::scoped_lock locker(_lock);
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
    std::scoped_lock locker(_lock);
    ws.ClearWSBuffers();
    _cur.recs.push_back(Rec{&ws, -1, 0, false, 0});
}

void WSReceiveBatch::Forget(WebSocket& ws)
{
    if (std::vector<Rec>* d = DrainRecs())   // from a callback of a Drain's delivery on this thread
        for (Rec& r : *d)
            if (r.ws == &ws)
                r.ws = nullptr;
    std::unique_lock<QueueLock> locker(_lock);
    for (Rec& r : _cur.recs)
        if (r.ws == &ws)
            r.ws = nullptr;
    if (!_flushing)
        return;
    if (_flusher == std::this_thread::get_id()) {
        // from a callback of this thread's flush: its records are this thread's
        for (Rec& r : _spare.recs)
            if (r.ws == &ws)
                r.ws = nullptr;
        return;
    }
    // Another thread is delivering.  It drops ws's frames before its next
    // record: the flush announces each record's connection in _busy and
    // then looks for pending Forgets (both sequentially consistent, as here
    // the flag is raised before _busy is read), so either it sees this
    // Forget before it calls into ws again, or ws is what it announced.
    // Only then is there anything to wait for: the callback it is running
    // for ws itself.  A flush busy with other connections is not waited for
    // (two threads' callbacks destroying each other's connections must not
    // block on each other's whole flush).
    _pending.push_back(&ws);
    _has_pending.store(true, std::memory_order_seq_cst);
    if (_busy.load(std::memory_order_seq_cst) != &ws)
        return;
    _waiters.fetch_add(1, std::memory_order_seq_cst);
    _busy_cv.wait(locker, [&] { return !_flushing || _busy.load(std::memory_order_seq_cst) != &ws; });
    _waiters.fetch_sub(1, std::memory_order_relaxed);
}

namespace {
template <class Recs>
bool holds(const Recs& recs, size_t from, const WebSocket* ws)
{
    for (size_t r = from; r < recs.size(); ++r)
        if (recs[r].ws == ws)
            return true;
    return false;
}
} // namespace

std::vector<WSReceiveBatch::Rec>*& WSReceiveBatch::DrainRecs()
{
    static thread_local std::vector<Rec>* recs = nullptr;
    return recs;
}

void WSReceiveBatch::Drain(WebSocket& ws)
{
    // Only ws's own frames are waited for, never the rest of another
    // thread's flush: two threads whose callbacks each move a connection off
    // the batch the other is flushing must not block on each other.
    Batch mine;   // ws's queued frames, taken out while another thread flushes
    for (;;) {
        std::unique_lock<QueueLock> locker(_lock);
        if (_flushing && _flusher == std::this_thread::get_id())
            return;   // (a callback of this thread's flush: the rest goes with a later flush)
        if (_flushing) {
            // ws's frames still ahead of (or at) the record the other flush
            // delivers: wait for it to move past them (it announces every
            // change of connection, _pos before _waiters, as for Forget)
            _waiters.fetch_add(1, std::memory_order_seq_cst);
            _busy_cv.wait(locker, [&] {
                return !_flushing || !holds(_spare.recs, _pos.load(std::memory_order_seq_cst), &ws);
            });
            _waiters.fetch_sub(1, std::memory_order_relaxed);
        }
        if (!holds(_cur.recs, 0, &ws))
            return;
        if (!_flushing) {
            locker.unlock();
            Flush();   // (0 when another thread started one meanwhile: again)
            continue;
        }
        // Another flush runs: ws's queued frames leave the queue and are
        // unmasked and delivered here, in their order; ws's earlier frames
        // have all been delivered (above) and no later one is queued while
        // its connection drains (RouteFrames waits).
        for (Rec& r : _cur.recs) {
            if (r.ws != &ws)
                continue;
            Rec m = r;
            r.ws = nullptr;
            if (r.frame >= 0) {
                const size_t f = size_t(r.frame);
                const uint64_t at = _cur.fs[f];
                const uint64_t end = f + 1 < _cur.fs.size() ? _cur.fs[f + 1] : _cur.wire.len;
                const uint8_t* frame = _cur.wire.p + at;
                Grow(mine.wire, mine.wire.len + (end - at));
                std::memcpy(mine.wire.p + mine.wire.len, frame, end - at);
                if ((frame[1] & 0x80) && (frame[r.hdr - 4] | frame[r.hdr - 3] | frame[r.hdr - 2] | frame[r.hdr - 1]))
                    mine.keyed = true;
                m.frame = int64_t(mine.fs.size());
                mine.fs.push_back(mine.wire.len);
                mine.wire.len += end - at;
            }
            mine.recs.push_back(m);
        }
        break;
    }
    struct Free {
        Batch& b;
        std::vector<Rec>* outer;   // (a Drain from a callback of another Drain's delivery)
        ~Free()
        {
            DrainRecs() = outer;
            Release(b.wire);
            Release(b.out);
        }
    } free_mine{mine, DrainRecs()};
    // (on this thread's own codec: the batch's contexts — its codec, or one per
    // device after SetDevices — are the running flush's, and a context is
    // one thread's at a time)
    const uint8_t* base = Unmask(mine, true);
    DrainRecs() = &mine.recs;   // (a Forget(ws) from one of these callbacks drops the rest)
    for (size_t r = 0; r < mine.recs.size(); ++r) {
        const Rec rec = mine.recs[r];
        if (!rec.ws)
            continue;
        if (rec.frame < 0) {
            rec.ws->ResetMessage();
            continue;
        }
        const size_t f = size_t(rec.frame);
        const uint64_t at = mine.fs[f] + rec.hdr;
        const uint64_t end = f + 1 < mine.fs.size() ? mine.fs[f + 1] : mine.wire.len;
        rec.ws->DeliverFrame(rec.opcode, rec.fin, base + at, size_t(end - at));
    }
}

const uint8_t* WSReceiveBatch::Unmask(Batch& b, bool thread_codec)
{
    // No frame with a key to apply (unmasked frames, or key 0: the
    // server-to-client direction of every reference session, ws.cpp:206):
    // unmasking is the identity, exactly as the per-call path skips it, so
    // the payloads are handed out where they lie in the batch, at the header
    // sizes the framer recorded (b.info is not used).
    const size_t n = b.fs.size();
    if (!n || !b.keyed)
        return b.wire.p;
    if (n > UINT32_MAX)
        throw std::length_error("WSReceiveBatch: more than 2^32-1 frames in one flush");
    b.info.resize(n);
    Grow(b.out, b.wire.len);
    if (thread_codec)
        check(wsg_decode_batch_host(ThreadCodec(), b.wire.p, b.wire.len, b.fs.data(), uint32_t(n), b.out.p,
                                    b.info.data()),
              "wsg_decode_batch_host");
    else if (_devs.size() > 1)
        check(wsg_decode_batch_host_multi(_devs.data(), int(_devs.size()), b.wire.p, b.wire.len, b.fs.data(),
                                          uint32_t(n), b.out.p, b.info.data()),
              "wsg_decode_batch_host_multi");
    else
        check(wsg_decode_batch_host(_devs.size() == 1 ? _devs[0] : _ctx ? _ctx : ThreadCodec(), b.wire.p, b.wire.len,
                                    b.fs.data(), uint32_t(n), b.out.p, b.info.data()),
              "wsg_decode_batch_host");
    return b.out.p;
}

void WSReceiveBatch::ApplyPending(size_t from)
{
    // the flushing thread, _lock held
    for (WebSocket* ws : _pending)
        for (size_t r = from; r < _spare.recs.size(); ++r)
            if (_spare.recs[r].ws == ws)
                _spare.recs[r].ws = nullptr;
    _pending.clear();
    _has_pending.store(false, std::memory_order_relaxed);
}

size_t WSReceiveBatch::Flush()
{
    {
        std::scoped_lock locker(_lock);
        if (_flushing || _cur.recs.empty())
            return 0;
        std::swap(_cur, _spare);
        _cur.reset();
        _n_frames.store(0, std::memory_order_relaxed);
        _n_bytes.store(0, std::memory_order_relaxed);
        _flushing = true;
        _flusher = std::this_thread::get_id();
        _pos.store(0, std::memory_order_relaxed);
    }
    Batch& b = _spare;   // this thread's until _flushing drops: Feed only touches _cur
    struct Done {
        WSReceiveBatch* t;
        ~Done()
        {
            std::scoped_lock locker(t->_lock);
            t->_flushing = false;
            t->_busy.store(nullptr, std::memory_order_seq_cst);
            t->_spare.reset();
            t->ApplyPending(0);
            t->_busy_cv.notify_all();   // nothing left to deliver: release any waiting Forget
        }
    } done{this};

    const size_t n = b.fs.size();
    const uint8_t* payload_base = Unmask(b);
    size_t delivered = 0;
    const void* announced = nullptr;
    // b.recs is written only by this thread (its callbacks' Forget); other
    // threads' Forget()s are applied here, between two records
    for (size_t r = 0; r < b.recs.size(); ++r) {
        // announce the connection, then look for Forgets (see Forget).  Only
        // this thread writes _busy, so while the records stay on one
        // connection it already holds that connection: no store, no wake-up
        if (b.recs[r].ws != announced) {
            announced = b.recs[r].ws;
            _pos.store(r, std::memory_order_seq_cst);   // (a Drain waits for the records from here on)
            _busy.store(announced, std::memory_order_seq_cst);
            if (_waiters.load(std::memory_order_seq_cst)) {
                std::scoped_lock locker(_lock);   // a Forget waiting for the previous connection may go
                _busy_cv.notify_all();
            }
        }
        if (_has_pending.load(std::memory_order_seq_cst)) {
            std::scoped_lock locker(_lock);
            ApplyPending(r);
        }
        const Rec rec = b.recs[r];
        if (!rec.ws)
            continue;
        if (rec.frame < 0) {
            rec.ws->ResetMessage();
            continue;
        }
        // the payload where the framer put it (its header size; the frames
        // lie back to back), in the unmasked copy when a pass ran: the pass
        // returned WSG_OK, so every frame parsed as framed and its record
        // says the same (the records the GPU wrote are not read back)
        const size_t f = size_t(rec.frame);
        const uint64_t at = b.fs[f] + rec.hdr;
        const uint64_t end = f + 1 < n ? b.fs[f + 1] : b.wire.len;
        rec.ws->DeliverFrame(rec.opcode, rec.fin, payload_base + at, size_t(end - at));
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
    for (Pinned* p : {&_q.payload, &_inflight.payload, &_wire})
        if (p->p)
            wsg_host_free(p->p);
    for (wsg_ctx* c : _devs)
        wsg_destroy(c);
}

void WSSendBatch::SetDevices(const std::vector<int>& devices)
{
    std::scoped_lock l(_lock);
    if (_flushing)
        throw std::logic_error("WSSendBatch::SetDevices during a flush");
    set_devices(_devs, devices);
}

void WSSendBatch::Push(Rec rec, uint32_t key, uint8_t opcode, bool mask, const void* buffer, size_t size,
                       int status)
{
    if (size && !buffer)
        throw std::invalid_argument("WSSendBatch: null payload");
    std::scoped_lock locker(_lock);
    Pinned& pl = _q.payload;
    grow_pinned(pl.p, pl.cap, pl.len, pl.len + size);
    wsg_send_desc d{};
    d.src_off = pl.len;
    d.len = size;
    d.key = key;
    d.status = status;
    d.opcode = opcode;
    d.mask = mask ? 1 : 0;
    if (size)
        std::memcpy(pl.p + pl.len, buffer, size);
    pl.len += size;
    _q.desc.push_back(d);
    _q.recs.push_back(std::move(rec));
    Counted();
}

void WSSendBatch::Queue(Transport& transport, uint32_t key, uint8_t opcode, bool mask, const void* buffer,
                        size_t size, int status)
{
    Push(Rec{&transport, nullptr, nullptr}, key, opcode, mask, buffer, size, status);
}

void WSSendBatch::Queue(void* tag, uint32_t key, uint8_t opcode, bool mask, const void* buffer, size_t size,
                        int status)
{
    Push(Rec{nullptr, tag, nullptr}, key, opcode, mask, buffer, size, status);
}

void WSSendBatch::QueueFanout(std::function<void(const uint8_t*, size_t)> deliver, uint32_t key, uint8_t opcode,
                              bool mask, const void* buffer, size_t size, int status)
{
    Push(Rec{nullptr, nullptr, std::make_shared<std::function<void(const uint8_t*, size_t)>>(std::move(deliver))},
         key, opcode, mask, buffer, size, status);
}

void WSSendBatch::Forget(Transport& transport) { ForgetIf(&transport, nullptr); }

void WSSendBatch::Forget(void* tag) { ForgetIf(nullptr, tag); }

namespace {
bool rec_matches(Transport* rt, void* rtag, Transport* transport, void* tag)
{
    return transport ? rt == transport : (rtag == tag && !rt);
}
} // namespace

void WSSendBatch::ForgetIf(Transport* transport, void* tag)
{
    std::unique_lock<QueueLock> locker(_lock);
    for (Rec& r : _q.recs)
        if (rec_matches(r.transport, r.tag, transport, tag))
            r = Rec{nullptr, nullptr, nullptr};
    if (!_flushing)
        return;
    if (_flusher == std::this_thread::get_id()) {   // from a callback of this thread's flush
        for (Rec& r : _inflight.recs)
            if (rec_matches(r.transport, r.tag, transport, tag))
                r = Rec{nullptr, nullptr, nullptr};
        return;
    }
    // applied by the flush before its next frame; waited for only while the
    // flush is handing a frame to this very transport / tag (as
    // WSReceiveBatch::Forget)
    _pending.emplace_back(transport, tag);
    _has_pending.store(true, std::memory_order_seq_cst);
    const void* mine = transport ? static_cast<const void*>(transport) : tag;
    if (_busy.load(std::memory_order_seq_cst) != mine)
        return;
    _waiters.fetch_add(1, std::memory_order_seq_cst);
    _busy_cv.wait(locker, [&] { return !_flushing || _busy.load(std::memory_order_seq_cst) != mine; });
    _waiters.fetch_sub(1, std::memory_order_relaxed);
}

void WSSendBatch::ApplyPending(size_t from)
{
    // the flushing thread, _lock held
    for (const auto& p : _pending)
        for (size_t i = from; i < _inflight.recs.size(); ++i) {
            Rec& r = _inflight.recs[i];
            if (rec_matches(r.transport, r.tag, p.first, p.second))
                r = Rec{nullptr, nullptr, nullptr};
        }
    _pending.clear();
    _has_pending.store(false, std::memory_order_relaxed);
}

size_t WSSendBatch::Flush(Sink sink, void* user)
{
    {
        std::scoped_lock locker(_lock);
        if (_flushing || _q.desc.empty())
            return 0;
        std::swap(_q, _inflight);   // the queue is empty again: callers may queue while this encodes
        _q.payload.len = 0;
        _q.desc.clear();
        _q.recs.clear();
        Counted();
        _flushing = true;
        _flusher = std::this_thread::get_id();
    }
    struct Done {
        WSSendBatch* t;
        ~Done()
        {
            std::scoped_lock locker(t->_lock);
            t->_flushing = false;
            t->_busy.store(nullptr, std::memory_order_seq_cst);
            t->_inflight.payload.len = 0;
            t->_inflight.desc.clear();
            t->_inflight.recs.clear();
            t->ApplyPending(0);
            t->_busy_cv.notify_all();   // nothing left to hand out: release any waiting Forget
        }
    } done{this};
    Queue_& b = _inflight;
    if (b.desc.size() > UINT32_MAX)
        throw std::length_error("WSSendBatch: more than 2^32-1 frames in one flush");
    const uint32_t n = uint32_t(b.desc.size());
    // frame offsets (the host path's sizes; a keyed pass recomputes them
    // on the device) and whether any frame has a key to apply
    _wire_off.resize(size_t(n) + 1);
    uint64_t total = 0;
    bool keyed = false;
    for (uint32_t i = 0; i < n; ++i) {
        const wsg_send_desc& d = b.desc[i];
        _wire_off[i] = total;
        const wsg::SendGeom g = wsg::send_geom(d.opcode, d.mask != 0, d.len, d.status);   // = wsg_frame_size
        total += g.hdr + g.body;
        keyed = keyed || d.key != 0;
    }
    _wire_off[n] = total;
    grow_pinned(_wire.p, _wire.cap, 0, std::max<uint64_t>(total, 1));
    int rc = WSG_OK;
    if (keyed) {
        if (_devs.size() > 1)
            rc = wsg_encode_batch_host_multi(_devs.data(), int(_devs.size()), b.payload.p, b.payload.len,
                                             b.desc.data(), n, _wire.p, _wire.cap, _wire_off.data());
        else
            rc = wsg_encode_batch_host(_devs.size() == 1 ? _devs[0] : _ctx ? _ctx : ThreadCodec(), b.payload.p,
                                       b.payload.len, b.desc.data(), n, _wire.p, _wire.cap, _wire_off.data());
    } else {
        // every frame has key 0 (server sessions, ws.cpp:206): the XOR is the
        // identity, as on the per-call path; header + status + payload copy
        for (uint32_t i = 0; i < n; ++i) {
            const wsg_send_desc& d = b.desc[i];
            uint8_t* f = _wire.p + _wire_off[i];
            const wsg::SendGeom g = wsg::send_geom(d.opcode, d.mask != 0, d.len, d.status);
            for (uint32_t r = 0; r < g.hdr; ++r)   // = wsg_header_pack with key 0
                f[r] = wsg::header_byte(d.opcode, d.mask != 0, g.body, 0, r);
            if (g.prefix) {
                f[g.hdr] = uint8_t((d.status >> 8) & 0xFF);
                f[g.hdr + 1] = uint8_t(d.status & 0xFF);
            }
            if (d.len)
                std::memcpy(f + g.hdr + g.prefix, b.payload.p + d.src_off, d.len);
        }
    }
    if (rc != WSG_OK) {
        // nothing was handed out: the frames go back in front of anything
        // queued meanwhile, so a later flush still sends them in order
        std::scoped_lock locker(_lock);
        ApplyPending(0);   // forgotten frames are not requeued
        const uint64_t shift = b.payload.len;
        grow_pinned(b.payload.p, b.payload.cap, b.payload.len, b.payload.len + _q.payload.len);
        if (_q.payload.len)
            std::memcpy(b.payload.p + b.payload.len, _q.payload.p, _q.payload.len);
        b.payload.len += _q.payload.len;
        for (wsg_send_desc d : _q.desc) {
            d.src_off += shift;
            b.desc.push_back(d);
        }
        for (Rec& r : _q.recs)
            b.recs.push_back(std::move(r));
        std::swap(_q, b);
        b.payload.len = 0;
        b.desc.clear();
        b.recs.clear();
        Counted();
        check(rc, "wsg_encode_batch_host");
    }
    size_t sent = 0;
    const void* announced = nullptr;
    // b.recs is written only by this thread (its callbacks' Forget); other
    // threads' Forget()s are applied here, between two hand-outs
    for (uint32_t i = 0; i < n;) {
        const uint8_t* f = _wire.p + _wire_off[i];
        {
            // announced only when the target changes (see WSReceiveBatch::Flush)
            const Rec& next = b.recs[i];
            const void* target = next.transport ? static_cast<const void*>(next.transport) : next.tag;
            if (target != announced) {
                announced = target;
                _busy.store(target, std::memory_order_seq_cst);
                if (_waiters.load(std::memory_order_seq_cst)) {
                    std::scoped_lock locker(_lock);
                    _busy_cv.notify_all();
                }
            }
        }
        if (_has_pending.load(std::memory_order_seq_cst)) {
            std::scoped_lock locker(_lock);
            ApplyPending(i);
        }
        const Rec& rec = b.recs[i];   // written by this thread only (ApplyPending above)
        if (rec.transport) {
            // a run of frames for one transport lies contiguous in _wire: one
            // SendAsync hands the transport the same bytes in the same order
            uint32_t j = i + 1;
            while (j < n && b.recs[j].transport == rec.transport)
                ++j;
            rec.transport->SendAsync(f, size_t(_wire_off[j] - _wire_off[i]));
            sent += j - i;
            i = j;
            continue;
        }
        const size_t len = size_t(_wire_off[i + 1] - _wire_off[i]);
        if (rec.deliver) {
            (*rec.deliver)(f, len);
            ++sent;
        } else if (rec.tag && sink) {
            sink(user, rec.tag, f, len);
            ++sent;
        }
        ++i;
    }
    return sent;
}

// ---------------------------------------------------------------- batch scope

namespace {

// Every thread's automatic batches, so that a connection being destroyed can
// drop what it queued into another thread's scope (ForgetEverywhere).  The
// batches are shared: one outlives its thread while a ForgetEverywhere uses it.
struct AutoEntry {
    std::weak_ptr<WSReceiveBatch> rx;
    std::weak_ptr<WSSendBatch> tx;
};
std::mutex& auto_registry_lock()
{
    static std::mutex* m = new std::mutex;   // leaked: used from thread exits after static destruction
    return *m;
}
std::vector<AutoEntry>& auto_registry()
{
    static auto* v = new std::vector<AutoEntry>;
    return *v;
}

struct AutoState {
    int depth = 0;
    bool draining = false;
    int enabled = -1;   // -1: from $WSG_AUTO_BATCH on first use
    size_t max_frames = size_t(1) << 20;
    uint64_t max_bytes = uint64_t(64) << 20;
    std::shared_ptr<WSReceiveBatch> rx_ = std::make_shared<WSReceiveBatch>(nullptr);
    std::shared_ptr<WSSendBatch> tx_ = std::make_shared<WSSendBatch>(nullptr);
    WSReceiveBatch& rx = *rx_;
    WSSendBatch& tx = *tx_;
    AutoState()
    {
        std::lock_guard<std::mutex> g(auto_registry_lock());
        auto& reg = auto_registry();
        reg.erase(std::remove_if(reg.begin(), reg.end(), [](const AutoEntry& e) { return e.rx.expired(); }),
                  reg.end());
        reg.push_back(AutoEntry{rx_, tx_});
    }
    // The thread is ending: its entry goes under the registry lock, so that a
    // ForgetEverywhere on another thread either still finds the batches (and
    // synchronizes with their last flush through their lock) or comes after
    // this point (and after every delivery this thread made).  An expired
    // weak_ptr alone orders nothing.
    ~AutoState()
    {
        std::lock_guard<std::mutex> g(auto_registry_lock());
        auto& reg = auto_registry();
        const WSReceiveBatch* mine = rx_.get();
        reg.erase(std::remove_if(reg.begin(), reg.end(),
                                 [&](const AutoEntry& e) {
                                     const auto p = e.rx.lock();
                                     return !p || p.get() == mine;
                                 }),
                  reg.end());
    }
};

AutoState& auto_state()
{
    thread_local AutoState st __attribute__((tls_model("initial-exec")));   // (see ThreadCodec, ws.cpp)
    if (st.enabled < 0) {
        const char* e = wsg::envp("WSG_AUTO_BATCH");
        st.enabled = (e && std::strcmp(e, "0") == 0) ? 0 : 1;
    }
    return st;
}

// AtEnd registrations: (thread, key, fn), process-wide so that Cancel works
// from any thread.  A hook being run is listed in g_end_running until it
// returns, and Cancel from another thread waits for it: the object can be
// destroyed only after its hook is done with it.
struct EndHook {
    std::thread::id thread;
    void* key;
    void (*fn)(void*);
};
std::mutex g_end_lock;
std::condition_variable g_end_done;
std::vector<EndHook> g_end_hooks;
std::vector<EndHook> g_end_running;

void run_end_hooks()
{
    const auto me = std::this_thread::get_id();
    for (;;) {
        EndHook h;
        {
            std::lock_guard<std::mutex> g(g_end_lock);
            auto it = std::find_if(g_end_hooks.begin(), g_end_hooks.end(),
                                   [&](const EndHook& e) { return e.thread == me; });
            if (it == g_end_hooks.end())
                return;
            h = *it;
            g_end_hooks.erase(it);
            g_end_running.push_back(h);
        }
        struct Finish {
            const EndHook& h;
            ~Finish()
            {
                std::lock_guard<std::mutex> g(g_end_lock);
                for (size_t i = 0; i < g_end_running.size(); ++i)
                    if (g_end_running[i].key == h.key && g_end_running[i].thread == h.thread) {
                        g_end_running.erase(g_end_running.begin() + std::ptrdiff_t(i));
                        break;
                    }
                g_end_done.notify_all();
            }
        } finish{h};
        h.fn(h.key);
    }
}

} // namespace

BatchScope::BatchScope() noexcept { ++auto_state().depth; }

BatchScope::~BatchScope()
{
    AutoState& st = auto_state();
    if (st.depth == 1 && !st.draining) {
        try {
            Flush();
            run_end_hooks();
        } catch (...) {
            // a destructor must not throw; the frames stay queued for the next flush
        }
    }
    --st.depth;
}

void BatchScope::ForgetEverywhere(WebSocket& ws, Transport& transport)
{
    std::vector<std::pair<std::shared_ptr<WSReceiveBatch>, std::shared_ptr<WSSendBatch>>> live;
    {
        std::lock_guard<std::mutex> g(auto_registry_lock());
        for (const AutoEntry& e : auto_registry())
            live.emplace_back(e.rx.lock(), e.tx.lock());
    }
    // outside the registry lock: a Forget may wait for a flush on another thread
    for (auto& [rx, tx] : live) {
        if (rx)
            rx->Forget(ws);
        if (tx)
            tx->Forget(transport);
    }
}

void BatchScope::AtEnd(void* key, void (*fn)(void*))
{
    std::lock_guard<std::mutex> g(g_end_lock);
    const auto me = std::this_thread::get_id();
    for (const EndHook& h : g_end_hooks)
        if (h.key == key && h.thread == me)
            return;
    g_end_hooks.push_back(EndHook{me, key, fn});
}

void BatchScope::Cancel(void* key)
{
    std::unique_lock<std::mutex> g(g_end_lock);
    for (size_t i = 0; i < g_end_hooks.size();) {
        if (g_end_hooks[i].key == key) {
            g_end_hooks[i] = g_end_hooks.back();
            g_end_hooks.pop_back();
        } else {
            ++i;
        }
    }
    // a hook of `key` running on another thread finishes first (on this
    // thread it is the caller itself: nothing to wait for)
    const auto me = std::this_thread::get_id();
    g_end_done.wait(g, [&] {
        return std::none_of(g_end_running.begin(), g_end_running.end(),
                            [&](const EndHook& e) { return e.key == key && e.thread != me; });
    });
}

size_t BatchScope::Flush()
{
    AutoState& st = auto_state();
    if (st.draining)
        return 0;
    st.draining = true;
    ++st.depth;   // callbacks' Send*Async queue into this thread's batch
    struct Done {
        AutoState& s;
        ~Done()
        {
            --s.depth;
            s.draining = false;
        }
    } done{st};
    size_t n = 0;
    // received frames first (their callbacks queue replies), then the sends;
    // again while the callbacks keep queueing
    for (int round = 0; round < 64 && (st.rx.frames() || st.tx.frames()); ++round) {
        n += st.rx.Flush();
        n += st.tx.Flush();
    }
    return n;
}

bool BatchScope::Enabled() { return auto_state().enabled != 0; }

void BatchScope::SetEnabled(bool on) { auto_state().enabled = on ? 1 : 0; }

bool BatchScope::Active()
{
    AutoState& st = auto_state();
    return st.enabled != 0 && st.depth > 0;
}

void BatchScope::SetLimits(size_t frames, uint64_t bytes)
{
    AutoState& st = auto_state();
    st.max_frames = std::max<size_t>(frames, 1);
    st.max_bytes = std::max<uint64_t>(bytes, 1);
}

WSReceiveBatch& BatchScope::Receive() { return auto_state().rx; }

WSSendBatch& BatchScope::Send() { return auto_state().tx; }

void BatchScope::CheckLimits()
{
    AutoState& st = auto_state();
    if (st.draining)
        return;
    if (st.rx.frames() >= st.max_frames || st.rx.bytes() >= st.max_bytes || st.tx.frames() >= st.max_frames ||
        st.tx.payload_bytes() >= st.max_bytes)
        Flush();
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

int wsg_rx_set_devices(wsg_rx* rx, const int* devices, int n)
{
    if (!rx || n < 0 || (n && !devices))
        return WSG_EINVAL;
    try {
        rx->batch.SetDevices(std::vector<int>(devices, devices + n));
        return WSG_OK;
    } catch (const std::logic_error&) {
        return WSG_EINVAL;
    } catch (...) {
        return WSG_EHIP;
    }
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

int wsg_tx_set_devices(wsg_tx* tx, const int* devices, int n)
{
    if (!tx || n < 0 || (n && !devices))
        return WSG_EINVAL;
    try {
        tx->batch.SetDevices(std::vector<int>(devices, devices + n));
        return WSG_OK;
    } catch (const std::logic_error&) {
        return WSG_EINVAL;
    } catch (...) {
        return WSG_EHIP;
    }
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
