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
 * Callback buffers are valid until the next Flush().  A batch is used from
 * one thread (the IO thread that owns the connections feeding it).
 */
#ifndef CPPSERVER_AMD_WS_BATCH_H
#define CPPSERVER_AMD_WS_BATCH_H

#include "server/ws/ws.h"

#include <cstdint>
#include <vector>

namespace CppServer {
namespace WS {

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
    //! Unmask every queued frame on the GPU and deliver them in arrival
    //! order; returns the number of frames delivered.  A Flush() called from
    //! inside a callback returns 0 (its frames go with the next one).
    size_t Flush();

    size_t frames() const { return _cur.fs.size(); }
    uint64_t bytes() const { return _cur.wire.len; }

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
    };
    struct Batch {
        Pinned wire, out;
        std::vector<uint64_t> fs;
        std::vector<Rec> recs;
        std::vector<wsg_recv_info> info;
        void reset()
        {
            wire.len = out.len = 0;
            fs.clear();
            recs.clear();
        }
    };

    void Emit(WebSocket& ws, const uint8_t* frame, uint64_t total, uint32_t hdr, const uint8_t* key);
    static void Grow(Pinned& b, uint64_t need);
    static void Release(Pinned& b);

    wsg_ctx* _ctx;
    Batch _cur, _spare;
    bool _flushing = false;
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
    //! Drop every queued frame of `transport` (call before destroying it)
    void Forget(Transport& transport);
    //! Drop every queued frame queued with `tag`
    void Forget(void* tag);
    //! Encode everything queued and hand the frames out in queue order;
    //! returns the number of frames handed out
    size_t Flush(Sink sink = nullptr, void* user = nullptr);

    size_t frames() const { return _desc.size(); }
    uint64_t payload_bytes() const { return _payload.len; }

private:
    struct Pinned {
        uint8_t* p = nullptr;
        uint64_t cap = 0, len = 0;
    };
    struct Rec {
        Transport* transport;
        void* tag;
    };
    void Push(Transport* t, void* tag, uint32_t key, uint8_t opcode, bool mask, const void* buffer, size_t size,
              int status);

    wsg_ctx* _ctx;
    Pinned _payload, _wire;
    std::vector<wsg_send_desc> _desc;
    std::vector<Rec> _recs;
    std::vector<uint64_t> _wire_off;
    bool _flushing = false;
};

} // namespace WS
} // namespace CppServer

#endif // CPPSERVER_AMD_WS_BATCH_H
