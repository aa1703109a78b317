/*
 * server/ws/ws_batch.h — batched receive for many connections (SURVEY.md §8f
 * item 1): the host framer + session batcher that connects the batch decode
 * kernels to WSSession::onReceived.
 *
 * The reference unmasks each frame on the IO thread that read it, inside
 * PrepareReceiveFrame (source/server/ws/ws.cpp:273-456), one connection at a
 * time.  Here Feed() runs the same per-connection framing state machine
 * (ws.cpp:292-397, RequiredReceiveFrameSize semantics, ws.cpp:458-482,
 * including the split-header behaviour of SURVEY Q7) but, instead of
 * unmasking, appends every completed frame to one page-locked batch; Flush()
 * unmasks the whole batch in one GPU pass (wsg_decode_batch_host) and then
 * delivers the frames in arrival order through each connection's message
 * logic (continuations, ws.cpp:326/406/411; dispatch, ws.cpp:413-452), so
 * every connection sees exactly the onWS* calls PrepareReceiveFrame would
 * have made, only later.
 *
 * Callback buffers are valid until the next Flush() (those of a Drain's own
 * delivery until it returns).  Feed / Clear / Forget
 * may come from any thread (a mutex guards the queue, as the reference's
 * per-session strands and locks let any IO thread call in); a Flush runs on
 * the calling thread with that thread's GPU codec context unless the batch
 * was given one, and fires the callbacks on that thread.  Forget(ws) drops
 * ws's frames at once and never waits for the rest of a flush: from another
 * thread it waits only while that flush is inside a callback FOR ws itself
 * (ws must outlive a call into it), so ws can be destroyed as soon as Forget
 * returns; from inside a callback of the flush it takes effect at once.  Two
 * threads whose callbacks each destroy a connection the other is delivering
 * to are therefore never blocked on each other, only a thread destroying the
 * very connection another thread is calling into is.
 */
#ifndef CPPSERVER_AMD_WS_BATCH_H
#define CPPSERVER_AMD_WS_BATCH_H

#include "server/ws/ws.h"

#include "wsg_capi.h"

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <new>
#include <type_traits>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace CppServer {
namespace WS {

//! The batches' queue lock.  Queueing a frame is a few stores, and an
//! uncontended std::mutex — two locked instructions behind two libc calls per
//! frame — was a fifth of a batched echo's host work (tools/sampler.cpp);
//! this one is an inline exchange and a release store.  Contended (an
//! explicit batch fed by several threads) it spins briefly, then yields.
class QueueLock
{
public:
    void lock() noexcept
    {
        for (unsigned i = 0; _held.exchange(true, std::memory_order_acquire); ++i) {
            while (_held.load(std::memory_order_relaxed)) {
                if (++i > 64)
                    std::this_thread::yield();
#if defined(__x86_64__)
                else
                    __builtin_ia32_pause();
#endif
            }
        }
    }
    bool try_lock() noexcept
    {
        return !_held.load(std::memory_order_relaxed) && !_held.exchange(true, std::memory_order_acquire);
    }
    void unlock() noexcept { _held.store(false, std::memory_order_release); }

private:
    std::atomic<bool> _held{false};
};

//! A growable array of trivially copyable records in page-locked memory
//! (wsg_host_alloc): a batch's frame table, records and descriptors, which
//! the GPU pass then reads and writes where they are instead of through a
//! staging copy.  Growing keeps the old block until the array is destroyed:
//! a grow happens under the batch's queue lock, and freeing page-locked memory
//! waits for the device to drain (a resident lane hands over every few ms), so
//! no free runs there.  The kept blocks total less than the live one.
template <class T>
class PinnedArray
{
    static_assert(std::is_trivially_copyable<T>::value, "PinnedArray holds plain records");

public:
    PinnedArray() = default;
    PinnedArray(const PinnedArray&) = delete;
    PinnedArray& operator=(const PinnedArray&) = delete;
    PinnedArray(PinnedArray&& o) noexcept
        : _p(o._p), _n(o._n), _cap(o._cap), _retired(std::move(o._retired))
    {
        o._p = nullptr, o._n = o._cap = 0;
    }
    PinnedArray& operator=(PinnedArray&& o) noexcept
    {
        std::swap(_p, o._p);
        std::swap(_n, o._n);
        std::swap(_cap, o._cap);
        std::swap(_retired, o._retired);
        return *this;
    }
    ~PinnedArray()
    {
        if (_p)
            wsg_host_free(_p);
        for (void* q : _retired)
            wsg_host_free(q);
    }
    T* data() noexcept { return _p; }
    const T* data() const noexcept { return _p; }
    size_t size() const noexcept { return _n; }
    bool empty() const noexcept { return _n == 0; }
    void clear() noexcept { _n = 0; }
    T& operator[](size_t i) noexcept { return _p[i]; }
    const T& operator[](size_t i) const noexcept { return _p[i]; }
    T* begin() noexcept { return _p; }
    T* end() noexcept { return _p + _n; }
    void push_back(const T& v)
    {
        if (_n == _cap)
            grow(_n + 1);
        _p[_n++] = v;
    }
    //! new elements are not initialized
    void resize(size_t n)
    {
        if (n > _cap)
            grow(n);
        _n = n;
    }

private:
    void grow(size_t need)
    {
        size_t cap = 2 * _cap > need ? 2 * _cap : need;
        if (cap < 4096 / sizeof(T))
            cap = 4096 / sizeof(T);
        void* q = nullptr;
        _retired.reserve(_retired.size() + 1);   // (before the allocation: nothing leaks if this throws)
        if (wsg_host_alloc(cap * sizeof(T), &q) != WSG_OK)
            throw std::bad_alloc();
        if (_n)
            std::memcpy(q, _p, _n * sizeof(T));
        if (_p)
            _retired.push_back(_p);
        _p = static_cast<T*>(q);
        _cap = cap;
    }
    T* _p = nullptr;
    size_t _n = 0, _cap = 0;
    std::vector<void*> _retired;   // earlier blocks, freed with the array
};

class WSReceiveBatch
{
public:
    //! codec: context the flushes decode on (nullptr: the calling thread's)
    explicit WSReceiveBatch(wsg_ctx* codec = nullptr);
    ~WSReceiveBatch();
    WSReceiveBatch(const WSReceiveBatch&) = delete;
    WSReceiveBatch& operator=(const WSReceiveBatch&) = delete;

    //! Frame `size` bytes of `ws`'s receive stream into the batch
    //! (the framing half of PrepareReceiveFrame, ws.cpp:292-397)
    void Feed(WebSocket& ws, const void* buffer, size_t size);
    //! ClearWSBuffers for a batched connection: its framing state is reset
    //! now, its message state at this point of the delivery order
    void Clear(WebSocket& ws);
    //! Drop every queued frame of `ws` (call before destroying it)
    void Forget(WebSocket& ws);
    //! Deliver every queued frame of `ws` (a connection leaving the batch),
    //! in order, on the calling thread.  It waits only while another
    //! thread's flush still has frames of ws to deliver (never for the rest
    //! of that flush); ws's frames still queued then are unmasked and
    //! delivered here without the others, and with no flush running the
    //! whole queue is flushed.  From inside a callback of this thread's own
    //! flush it returns at once.  No frame of ws may be fed meanwhile (the
    //! connection's reads wait while it switches batches: SetReceiveBatch).
    void Drain(WebSocket& ws);
    //! Unmask every queued frame on the GPU and deliver them in arrival
    //! order; returns the number of frames delivered.  A Flush() called from
    //! inside a callback returns 0 (its frames go with the next one).
    size_t Flush();
    //! Spread every flush's GPU pass over these devices' PCIe links
    //! (wsg_decode_batch_host_multi: one context per device, owned by the
    //! batch); empty: the batch's own context.  Not during a flush.
    void SetDevices(const std::vector<int>& devices);

    // queued frames / wire bytes (exact for the queueing thread; a snapshot
    // for others): read on every queued frame (BatchScope::CheckLimits), so
    // counters kept beside the queue instead of taking its lock
    size_t frames() const { return _n_frames.load(std::memory_order_relaxed); }
    uint64_t bytes() const { return _n_bytes.load(std::memory_order_relaxed); }

private:
    struct Pinned {
        uint8_t* p = nullptr;
        uint64_t cap = 0, len = 0;
    };
    struct Rec {
        WebSocket* ws;
        int64_t frame;    // index into fs, or -1: message reset marker
        uint8_t opcode;   // _ws_opcode in force when the frame completed
        bool fin;
        uint32_t hdr;     // header bytes of the frame (its payload follows them)
    };
    struct Batch {
        Pinned wire, out;
        PinnedArray<uint64_t> fs;   // (page-locked: the decode pass reads the table and
        std::vector<Rec> recs;
        PinnedArray<wsg_recv_info> info;   //  writes the records in place)
        bool keyed = false;   // some frame carries a nonzero mask key: the GPU pass has bytes to change
        void reset()
        {
            wire.len = out.len = 0;
            fs.clear();
            recs.clear();
            keyed = false;
        }
    };

    void Emit(WebSocket& ws, const uint8_t* frame, uint64_t total, uint32_t hdr, const uint8_t* key);
    void ApplyPending(size_t from);
    //! the batch's GPU pass (when a frame has a key); where the payloads lie.
    //! thread_codec: on the calling thread's codec instead of the batch's
    const uint8_t* Unmask(Batch& b, bool thread_codec = false);
    //! this thread's Drain delivery in progress (its records), or nullptr
    static std::vector<Rec>*& DrainRecs();
    static void Grow(Pinned& b, uint64_t need);
    static void Release(Pinned& b);

    wsg_ctx* _ctx;
    std::vector<wsg_ctx*> _devs;   // SetDevices: owned, one per device
    Batch _cur, _spare;   // queueing | the flush's (its records: written by the flushing thread only)
    bool _flushing = false;
    std::thread::id _flusher;
    std::vector<WebSocket*> _pending;    // other threads' Forget()s the flush has not applied yet
    std::atomic<bool> _has_pending{false};
    std::atomic<const void*> _busy{nullptr};   // the connection the flush is at (announced before its Forget check)
    std::atomic<size_t> _pos{0};               // the first record of that connection's run (a Drain waits past ws's)
    std::atomic<int> _waiters{0};              // Forget()s / Drain()s waiting for _busy / _pos to move on
    std::condition_variable_any _busy_cv;
    std::atomic<size_t> _n_frames{0};          // _cur.fs.size(), written under _lock
    std::atomic<uint64_t> _n_bytes{0};         // _cur.wire.len, written under _lock
    mutable QueueLock _lock;   // _cur, _flushing, _pending
};

class Transport;

/*
 * Batched send for many connections.  The reference
 * encodes every Send*Async on the caller's thread (PrepareSendFrame,
 * ws.cpp:212-271) and hands the frame to the transport right away
 * (tcp_session.cpp:257-307).  Queue() records the same call — the
 * connection's key, opcode, mask flag, close status and a copy of the
 * payload — and Flush() encodes every queued frame in one pipelined GPU pass
 * (wsg_encode_batch_host) and hands each frame to its transport in queue
 * order: the same bytes the per-call path sends, in the same order per
 * connection.
 */
class WSSendBatch
{
public:
    //! Sink for frames queued without a transport (the C-ABI's wsg_tx_flush)
    using Sink = void (*)(void* user, void* tag, const uint8_t* frame, size_t size);

    explicit WSSendBatch(wsg_ctx* codec = nullptr);
    ~WSSendBatch();
    WSSendBatch(const WSSendBatch&) = delete;
    WSSendBatch& operator=(const WSSendBatch&) = delete;

    //! PrepareSendFrame(opcode, mask, buffer, size, status) with send key
    //! `key`, deferred: the frame goes to transport.SendAsync at Flush()
    void Queue(Transport& transport, uint32_t key, uint8_t opcode, bool mask, const void* buffer, size_t size,
               int status = 0);
    //! The same, for a frame the flush sink receives with `tag`
    void Queue(void* tag, uint32_t key, uint8_t opcode, bool mask, const void* buffer, size_t size, int status = 0);
    //! The same, for a frame handed to `deliver` at Flush() (a multicast:
    //! encoded once, then copied to every session, ws_server.cpp:36-64)
    void QueueFanout(std::function<void(const uint8_t* frame, size_t size)> deliver, uint32_t key, uint8_t opcode,
                     bool mask, const void* buffer, size_t size, int status = 0);
    //! Drop every queued frame of `transport` (call before destroying it)
    void Forget(Transport& transport);
    //! Drop every queued frame queued with `tag`
    void Forget(void* tag);
    //! Encode everything queued and hand the frames out in queue order;
    //! returns the number of frames handed out
    size_t Flush(Sink sink = nullptr, void* user = nullptr);
    //! Spread every flush's GPU pass over these devices' PCIe links
    //! (wsg_encode_batch_host_multi; contexts owned by the batch); empty:
    //! the batch's own context.  Not during a flush.
    void SetDevices(const std::vector<int>& devices);

    // as WSReceiveBatch::frames()
    size_t frames() const { return _n_frames.load(std::memory_order_relaxed); }
    uint64_t payload_bytes() const { return _n_bytes.load(std::memory_order_relaxed); }

private:
    struct Pinned {
        uint8_t* p = nullptr;
        uint64_t cap = 0, len = 0;
    };
    struct Rec {
        Transport* transport;
        void* tag;
        std::shared_ptr<std::function<void(const uint8_t*, size_t)>> deliver;
    };
    void Push(Rec rec, uint32_t key, uint8_t opcode, bool mask, const void* buffer, size_t size, int status);
    void ForgetIf(Transport* transport, void* tag);
    void ApplyPending(size_t from);

    struct Queue_ {
        Pinned payload;
        PinnedArray<wsg_send_desc> desc;   // (page-locked: read by the encode pass in place)
        std::vector<Rec> recs;
    };

    wsg_ctx* _ctx;
    std::vector<wsg_ctx*> _devs;   // SetDevices: owned, one per device
    Queue_ _q, _inflight;   // frames being queued | the frames a flush is encoding (written by its thread only)
    Pinned _wire;
    PinnedArray<uint64_t> _wire_off;
    bool _flushing = false;
    std::thread::id _flusher;
    std::vector<std::pair<Transport*, void*>> _pending;   // other threads' Forget()s not applied yet
    std::atomic<bool> _has_pending{false};
    std::atomic<const void*> _busy{nullptr};   // transport / tag the flush is at (see WSReceiveBatch)
    std::atomic<int> _waiters{0};
    std::condition_variable_any _busy_cv;
    std::atomic<size_t> _n_frames{0};   // _q.desc.size(), written under _lock
    std::atomic<uint64_t> _n_bytes{0};  // _q.payload.len, written under _lock
    void Counted()
    {
        _n_frames.store(_q.desc.size(), std::memory_order_relaxed);
        _n_bytes.store(_q.payload.len, std::memory_order_relaxed);
    }
    mutable QueueLock _lock;   // _q, _flushing, _pending
};

/*
 * Automatic batching: what makes the drop-in API fast without code changes.
 *
 * The reference encodes every Send*Async and unmasks every received frame on
 * the spot, one connection at a time (ws.cpp:212-456).  Here
 * WSClient/WSSession::onReceived open a BatchScope on the calling thread:
 * the frames of the bytes read are framed on the host and unmasked in ONE
 * GPU pass when the outermost scope closes, and every Send*Async made
 * meanwhile — by the onWS* callbacks, e.g. an echo — is encoded in ONE GPU
 * pass after them.  Callbacks still fire before onReceived returns, in
 * arrival order, with the reference's arguments; each connection's frames
 * leave in call order (a sync Send* / Receive* flushes first).
 *
 * A transport that reads many connections per loop iteration (an epoll /
 * io_uring tick) opens one BatchScope around the iteration and every
 * connection's frames of that tick share the two GPU passes.  A batch that
 * reaches the limits (SetLimits) is flushed early.  Send*Async outside any
 * scope (a timer thread, the multicaster of ws_multicast) is encoded per
 * call.  $WSG_AUTO_BATCH=0 (or SetEnabled(false)) gives the per-call path.
 */
class BatchScope
{
public:
    BatchScope() noexcept;
    ~BatchScope();
    BatchScope(const BatchScope&) = delete;
    BatchScope& operator=(const BatchScope&) = delete;

    //! Decode and deliver what this thread received, then encode and send
    //! what it queued (repeated while the callbacks queue more); returns the
    //! frames handled.  No effect from inside a delivery on this thread.
    static size_t Flush();
    //! Automatic batching on this thread (default: on, unless $WSG_AUTO_BATCH=0)
    static bool Enabled();
    static void SetEnabled(bool on);
    //! Inside a scope on this thread
    static bool Active();
    //! Flush early when the receive batch holds `frames` frames or `bytes`
    //! wire bytes, or the send batch that many frames / payload bytes
    static void SetLimits(size_t frames, uint64_t bytes);

    //! This thread's automatic batches (used by the WS classes)
    static WSReceiveBatch& Receive();
    static WSSendBatch& Send();
    //! Early flush when a batch passed the limits (inside a scope)
    static void CheckLimits();

    //! Drop a connection's queued frames from the automatic batches of EVERY
    //! thread (a session queued into another thread's scope, e.g. a SendAsync
    //! from a worker thread), waiting for a flush in progress there to drop
    //! them; the connection's destructor calls it
    static void ForgetEverywhere(WebSocket& ws, Transport& transport);

    //! Call fn(key) once when the outermost scope on this thread ends, after
    //! its last flush (a transport that coalesces what one scope sends: the
    //! TLS records of a tick).  Registering a key twice is one call;
    //! Cancel(key) drops it (the object is going away).
    static void AtEnd(void* key, void (*fn)(void*));
    static void Cancel(void* key);
};

} // namespace WS
} // namespace CppServer

#endif // CPPSERVER_AMD_WS_BATCH_H
