// ws_api.cpp — WSClient / WSSession / WSServer over a Transport.
//
// Send* = lock _ws_send_lock, PrepareSendFrame (payload masked on the GPU),
// hand the frame to the transport (reference ws_client.h:53-90,
// ws_session.h:46-83).  onReceived routes post-upgrade bytes to
// PrepareReceiveFrame (ws_client.cpp:76-87, ws_session.cpp:40-51).
// Multicast encodes once and queues the same bytes on every handshaked
// session (ws_server.cpp:36-64).
#include "server/ws/ws_client.h"
#include "server/ws/ws_server.h"
#include "server/ws/ws_session.h"

#include <algorithm>
#include <thread>
#include <unordered_set>

namespace CppServer {
namespace WS {

namespace {

// Synchronous framing loop shared by client and session Receive*
// (reference ws_client.cpp:139-157).  The reference then copies from
// final_buffer + header_size (ws_client.cpp:155), skipping the
// first header_size payload bytes; this build returns the whole message.
template <class Required, class Prepare, class Recv>
bool receive_message(std::vector<uint8_t>& out, Required required, Prepare prepare, Recv recv,
                     const std::vector<uint8_t>& final_buf, const bool& frame_received, const bool& final_received)
{
    std::vector<uint8_t> cache;
    while (!final_received) {
        while (!frame_received) {
            const size_t want = required();
            cache.resize(want);
            if (recv(cache.data(), want) != want)
                return false;
            prepare(cache.data(), want);
        }
        if (!final_received)
            prepare(nullptr, 0);
    }
    out.assign(final_buf.begin(), final_buf.end());
    prepare(nullptr, 0);
    return true;
}

} // namespace

// ---------------------------------------------------------------- WSClient

void WSClient::ResetBuffers()
{
    {
        std::scoped_lock<QueueLock> use(_rx_use);
        if (WSReceiveBatch* b = _rx_batch.load(std::memory_order_acquire)) {
            b->Clear(*this);   // message state resets in delivery order
            return;
        }
        if (_rx_draining) {
            _rx_prev->Clear(*this);   // after the frames still queued in the batch being left
            return;
        }
    }
    if (BatchScope::Active())
        BatchScope::Receive().Clear(*this);
    else
        ClearWSBuffers();
}

WSClient::~WSClient()
{
    // frames still queued on any thread's automatic batches
    BatchScope::ForgetEverywhere(*this, _transport);
}

void WSClient::SetReceiveBatch(WSReceiveBatch* batch)
{
    // swapped atomically (the IO thread reads it per read); the old batch
    // delivers this connection's queued frames before its next read is taken
    WSReceiveBatch* old;
    {
        std::scoped_lock<QueueLock> use(_rx_use);   // (a read still feeding the old batch finishes first)
        old = _rx_batch.exchange(batch, std::memory_order_acq_rel);
        if (old && old != batch) {
            _rx_prev = old;
            _rx_draining = true;
        }
    }
    if (old && old != batch) {
        // the frames this connection queued there are delivered before any
        // later read of it goes the new way (reads wait meanwhile)
        old->Drain(*this);
        std::scoped_lock<QueueLock> use(_rx_use);
        _rx_draining = false;
        _rx_prev = nullptr;
    }
}

bool WSClient::Connect()
{
    if (!_transport.IsConnected())
        return false;
    ResetBuffers();
    _http_buf.clear();
    HTTP::HTTPRequest request;
    onWSConnecting(request);
    request.SetBody();
    const std::string& req = request.cache();
    return _transport.Send(req.data(), req.size()) == req.size();
}

bool WSClient::ConnectAsync()
{
    if (!_transport.IsConnected())
        return false;
    ResetBuffers();
    _http_buf.clear();
    HTTP::HTTPRequest request;
    onWSConnecting(request);
    request.SetBody();
    const std::string& req = request.cache();
    return _transport.SendAsync(req.data(), req.size());
}

bool WSClient::Disconnect()
{
    const bool ok = _transport.Disconnect();
    onDisconnected();
    return ok;
}

void WSClient::onDisconnected()
{
    if (_ws_handshaked) {
        _ws_handshaked = false;
        onWSDisconnected();
    }
    ResetBuffers();
    InitWSNonce();
}

void WSClient::onReceived(const void* buffer, size_t size)
{
    // everything this read triggers (onWS* callbacks, their Send*Async) is
    // batched on this thread and flushed when the outermost scope closes
    BatchScope scope;
    if (!_ws_handshaked) {
        // the upgrade response (reference ws_client.cpp:76-116 via HTTPClient)
        _http_buf.append(static_cast<const char*>(buffer), size);
        HTTP::HTTPResponse response;
        const size_t used = response.Parse(_http_buf);
        if (used == 0)
            return;   // header block not complete yet
        const std::string rest = _http_buf.substr(used);
        _http_buf.clear();
        if (response.error()) {
            onWSError("Invalid HTTP response");
            return;
        }
        if (!PerformClientUpgrade(response) || rest.empty())
            return;
        RouteFrames(rest.data(), rest.size());   // frames that came with the response
        return;
    }
    RouteFrames(buffer, size);
}

void WSClient::RouteFrames(const void* buffer, size_t size)
{
    for (;;) {
        {
            std::scoped_lock<QueueLock> use(_rx_use);   // (SetReceiveBatch waits for this feed)
            if (!_rx_draining) {
                if (WSReceiveBatch* b = _rx_batch.load(std::memory_order_acquire)) {
                    b->Feed(*this, buffer, size);
                    return;
                }
                break;
            }
        }
        std::this_thread::yield();   // a batch switch delivers this connection's earlier frames first
    }
    if (BatchScope::Active()) {
        BatchScope::Receive().Feed(*this, buffer, size);
        BatchScope::CheckLimits();
    } else {
        PrepareReceiveFrame(buffer, size);
    }
}

void WSClient::SetSendBatch(WSSendBatch* batch)
{
    WSSendBatch* old;
    {
        std::scoped_lock locker(_ws_send_lock, _tx_use);
        old = _tx_batch.exchange(batch, std::memory_order_acq_rel);
    }
    // not under the send lock: Forget may wait for a flush on another thread
    // whose deliveries take session send locks (a multicast)
    if (old && old != batch)
        old->Forget(_transport);
}

size_t WSClient::SendFrame(uint8_t opcode, const void* buffer, size_t size, int status,
                           const CppCommon::Timespan* timeout)
{
    bool batched = false;
    {
        std::scoped_lock<QueueLock> use(_tx_use);   // (SetSendBatch waits for this flush)
        if (WSSendBatch* b = _tx_batch.load(std::memory_order_acquire)) {
            b->Flush();   // earlier async frames go first
            batched = true;
        }
    }
    if (!batched && BatchScope::Active())
        BatchScope::Send().Flush();
    std::scoped_lock locker(_ws_send_lock);
    PrepareSendFrame(opcode, true, buffer, size, status);
    return timeout ? _transport.Send(_ws_send_buffer.data(), _ws_send_buffer.size(), *timeout)
                   : _transport.Send(_ws_send_buffer.data(), _ws_send_buffer.size());
}

bool WSClient::SendFrameAsync(uint8_t opcode, const void* buffer, size_t size, int status)
{
    if (!_tx_batch.load(std::memory_order_acquire) && BatchScope::Active()) {
        // the thread's own scope: nothing of this connection but its key is
        // touched, and the scope's queue has its own lock
        BatchScope::Send().Queue(_transport, send_key(), opcode, true, buffer, size, status);
        BatchScope::CheckLimits();
        return true;
    }
    {
        std::scoped_lock locker(_ws_send_lock);
        if (WSSendBatch* b = _tx_batch.load(std::memory_order_relaxed)) {
            // an explicit batch: queued under the send lock, so that once
            // SetSendBatch has swapped it out no thread is still queueing into it
            b->Queue(_transport, send_key(), opcode, true, buffer, size, status);
            return true;
        }
        if (!BatchScope::Active()) {
            PrepareSendFrame(opcode, true, buffer, size, status);
            return _transport.SendAsync(_ws_send_buffer.data(), _ws_send_buffer.size());
        }
        BatchScope::Send().Queue(_transport, send_key(), opcode, true, buffer, size, status);
    }
    BatchScope::CheckLimits();   // not under the send lock: a flush may fire callbacks
    return true;
}

bool WSClient::ReceiveMessage(std::vector<uint8_t>& out, const CppCommon::Timespan* timeout)
{
    if (!_ws_handshaked)
        return false;
    if (BatchScope::Active())
        BatchScope::Send().Flush();   // what this thread queued goes out before it waits
    return receive_message(
        out, [this]() { return RequiredReceiveFrameSize(); },
        [this](const void* b, size_t n) { PrepareReceiveFrame(b, n); },
        [this, timeout](void* b, size_t n) {
            return timeout ? _transport.Receive(b, n, *timeout) : _transport.Receive(b, n);
        },
        _ws_receive_final_buffer, _ws_frame_received, _ws_final_received);
}

std::string WSClient::ReceiveText()
{
    std::vector<uint8_t> msg;
    if (!ReceiveMessage(msg))
        return std::string();
    return std::string(msg.begin(), msg.end());
}

std::string WSClient::ReceiveText(const CppCommon::Timespan& timeout)
{
    std::vector<uint8_t> msg;
    if (!ReceiveMessage(msg, &timeout))
        return std::string();
    return std::string(msg.begin(), msg.end());
}

std::vector<uint8_t> WSClient::ReceiveBinary()
{
    std::vector<uint8_t> msg;
    ReceiveMessage(msg);
    return msg;
}

std::vector<uint8_t> WSClient::ReceiveBinary(const CppCommon::Timespan& timeout)
{
    std::vector<uint8_t> msg;
    ReceiveMessage(msg, &timeout);
    return msg;
}

// ---------------------------------------------------------------- WSSession

void WSSession::ResetBuffers()
{
    {
        std::scoped_lock<QueueLock> use(_rx_use);
        if (WSReceiveBatch* b = _rx_batch.load(std::memory_order_acquire)) {
            b->Clear(*this);   // message state resets in delivery order
            return;
        }
        if (_rx_draining) {
            _rx_prev->Clear(*this);   // after the frames still queued in the batch being left
            return;
        }
    }
    if (BatchScope::Active())
        BatchScope::Receive().Clear(*this);
    else
        ClearWSBuffers();
}

WSSession::~WSSession()
{
    // frames still queued on any thread's automatic batches
    BatchScope::ForgetEverywhere(*this, _transport);
}

void WSSession::SetReceiveBatch(WSReceiveBatch* batch) { SwapReceiveBatch(batch, true); }

void WSSession::SwapReceiveBatch(WSReceiveBatch* batch, bool deliver)
{
    if (!deliver) {
        WSReceiveBatch* old;
        {
            std::scoped_lock<QueueLock> use(_rx_use);   // (a read still feeding the old batch finishes first)
            old = _rx_batch.exchange(batch, std::memory_order_acq_rel);
        }
        if (old && old != batch)
            old->Forget(*this);
        return;
    }
    WSReceiveBatch* old;
    {
        std::scoped_lock<QueueLock> use(_rx_use);   // (a read still feeding the old batch finishes first)
        old = _rx_batch.exchange(batch, std::memory_order_acq_rel);
        if (old && old != batch) {
            _rx_prev = old;
            _rx_draining = true;
        }
    }
    if (old && old != batch) {
        // the frames this connection queued there are delivered before any
        // later read of it goes the new way (reads wait meanwhile)
        old->Drain(*this);
        std::scoped_lock<QueueLock> use(_rx_use);
        _rx_draining = false;
        _rx_prev = nullptr;
    }
}

bool WSSession::Connect()
{
    if (!_transport.IsConnected())
        return false;
    ResetBuffers();
    _http_buf.clear();
    return true;
}

bool WSSession::Disconnect()
{
    const bool ok = _transport.Disconnect();
    onDisconnected();
    return ok;
}

void WSSession::onDisconnected()
{
    if (_ws_handshaked) {
        _ws_handshaked = false;
        onWSDisconnected();
    }
    ResetBuffers();
    InitWSNonce();
}

void WSSession::onReceived(const void* buffer, size_t size)
{
    BatchScope scope;   // as WSClient::onReceived
    if (!_ws_handshaked) {
        // the upgrade request (reference ws_session.cpp:53-65 via HTTPSession)
        _http_buf.append(static_cast<const char*>(buffer), size);
        HTTP::HTTPRequest request;
        const size_t used = request.Parse(_http_buf);
        if (used == 0)
            return;
        const std::string rest = _http_buf.substr(used);
        _http_buf.clear();
        HTTP::HTTPResponse response;
        if (request.error()) {
            response.MakeErrorResponse(400, "Invalid HTTP request");
            SendResponse(response);
            return;
        }
        if (!PerformServerUpgrade(request, response) || rest.empty())
            return;
        RouteFrames(rest.data(), rest.size());
        return;
    }
    RouteFrames(buffer, size);
}

void WSSession::RouteFrames(const void* buffer, size_t size)
{
    for (;;) {
        {
            std::scoped_lock<QueueLock> use(_rx_use);   // (SetReceiveBatch waits for this feed)
            if (!_rx_draining) {
                if (WSReceiveBatch* b = _rx_batch.load(std::memory_order_acquire)) {
                    b->Feed(*this, buffer, size);
                    return;
                }
                break;
            }
        }
        std::this_thread::yield();   // a batch switch delivers this connection's earlier frames first
    }
    if (BatchScope::Active()) {
        BatchScope::Receive().Feed(*this, buffer, size);
        BatchScope::CheckLimits();
    } else {
        PrepareReceiveFrame(buffer, size);
    }
}

void WSSession::SetSendBatch(WSSendBatch* batch)
{
    WSSendBatch* old;
    {
        std::scoped_lock locker(_ws_send_lock, _tx_use);
        old = _tx_batch.exchange(batch, std::memory_order_acq_rel);
    }
    // not under the send lock: Forget may wait for a flush on another thread
    // whose deliveries take session send locks (a multicast)
    if (old && old != batch)
        old->Forget(_transport);
}

size_t WSSession::SendFrame(uint8_t opcode, const void* buffer, size_t size, int status,
                            const CppCommon::Timespan* timeout)
{
    bool batched = false;
    {
        std::scoped_lock<QueueLock> use(_tx_use);   // (SetSendBatch waits for this flush)
        if (WSSendBatch* b = _tx_batch.load(std::memory_order_acquire)) {
            b->Flush();   // earlier async frames go first
            batched = true;
        }
    }
    if (!batched && BatchScope::Active())
        BatchScope::Send().Flush();
    std::scoped_lock locker(_ws_send_lock);
    PrepareSendFrame(opcode, false, buffer, size, status);
    return timeout ? _transport.Send(_ws_send_buffer.data(), _ws_send_buffer.size(), *timeout)
                   : _transport.Send(_ws_send_buffer.data(), _ws_send_buffer.size());
}

bool WSSession::SendFrameAsync(uint8_t opcode, const void* buffer, size_t size, int status)
{
    if (!_tx_batch.load(std::memory_order_acquire) && BatchScope::Active()) {
        // the thread's own scope: nothing of this connection but its key is
        // touched, and the scope's queue has its own lock
        BatchScope::Send().Queue(_transport, send_key(), opcode, false, buffer, size, status);
        BatchScope::CheckLimits();
        return true;
    }
    {
        std::scoped_lock locker(_ws_send_lock);
        if (WSSendBatch* b = _tx_batch.load(std::memory_order_relaxed)) {
            // an explicit batch: queued under the send lock, so that once
            // SetSendBatch has swapped it out no thread is still queueing into it
            b->Queue(_transport, send_key(), opcode, false, buffer, size, status);
            return true;
        }
        if (!BatchScope::Active()) {
            PrepareSendFrame(opcode, false, buffer, size, status);
            return _transport.SendAsync(_ws_send_buffer.data(), _ws_send_buffer.size());
        }
        BatchScope::Send().Queue(_transport, send_key(), opcode, false, buffer, size, status);
    }
    BatchScope::CheckLimits();
    return true;
}

bool WSSession::ReceiveMessage(std::vector<uint8_t>& out, const CppCommon::Timespan* timeout)
{
    if (!_ws_handshaked)
        return false;
    if (BatchScope::Active())
        BatchScope::Send().Flush();
    return receive_message(
        out, [this]() { return RequiredReceiveFrameSize(); },
        [this](const void* b, size_t n) { PrepareReceiveFrame(b, n); },
        [this, timeout](void* b, size_t n) {
            return timeout ? _transport.Receive(b, n, *timeout) : _transport.Receive(b, n);
        },
        _ws_receive_final_buffer, _ws_frame_received, _ws_final_received);
}

std::string WSSession::ReceiveText()
{
    std::vector<uint8_t> msg;
    if (!ReceiveMessage(msg))
        return std::string();
    return std::string(msg.begin(), msg.end());
}

std::string WSSession::ReceiveText(const CppCommon::Timespan& timeout)
{
    std::vector<uint8_t> msg;
    if (!ReceiveMessage(msg, &timeout))
        return std::string();
    return std::string(msg.begin(), msg.end());
}

std::vector<uint8_t> WSSession::ReceiveBinary()
{
    std::vector<uint8_t> msg;
    ReceiveMessage(msg);
    return msg;
}

std::vector<uint8_t> WSSession::ReceiveBinary(const CppCommon::Timespan& timeout)
{
    std::vector<uint8_t> msg;
    ReceiveMessage(msg, &timeout);
    return msg;
}

// ---------------------------------------------------------------- WSServer

std::shared_ptr<WSReceiveBatch> WSServer::rx_batch() const
{
    std::shared_lock<std::shared_mutex> locker(_sessions_lock);
    return _rx_batch;
}

std::shared_ptr<WSSendBatch> WSServer::tx_batch() const
{
    std::shared_lock<std::shared_mutex> locker(_sessions_lock);
    return _tx_batch;
}

void WSServer::AddSession(const std::shared_ptr<WSSession>& session)
{
    std::unique_lock<std::shared_mutex> locker(_sessions_lock);
    _sessions.push_back(session);
    _snapshot = std::make_shared<const std::vector<std::shared_ptr<WSSession>>>(_sessions);
    if (_rx_batch)
        session->SetReceiveBatch(_rx_batch.get());
    if (_tx_batch)
        session->SetSendBatch(_tx_batch.get());
}

void WSServer::RemoveSession(const std::shared_ptr<WSSession>& session)
{
    bool detach = false;
    std::shared_ptr<WSReceiveBatch> rx;
    std::shared_ptr<WSSendBatch> tx;
    {
        std::unique_lock<std::shared_mutex> locker(_sessions_lock);
        detach = std::find(_sessions.begin(), _sessions.end(), session) != _sessions.end();
        _sessions.erase(std::remove(_sessions.begin(), _sessions.end(), session), _sessions.end());
        _snapshot = std::make_shared<const std::vector<std::shared_ptr<WSSession>>>(_sessions);
        // the batches the session is attached to: an EnableBatch*(false)
        // from now on does not see the session and must not free them under
        // the detach below
        rx = _rx_batch;
        tx = _tx_batch;
    }
    // its queued frames are dropped with it; outside the sessions lock: a
    // batch's Forget may wait for a flush on another thread that is calling
    // into this session, and whose callbacks may take that lock
    if (detach) {
        session->SwapReceiveBatch(nullptr, false);
        session->SetSendBatch(nullptr);
    }
}

void WSServer::EnableBatchReceive(bool on)
{
    std::lock_guard<std::recursive_mutex> one(_rx_switch);
    std::unique_lock<std::shared_mutex> locker(_sessions_lock);
    if (on == (_rx_batch != nullptr))
        return;
    if (on) {
        _rx_batch = std::make_shared<WSReceiveBatch>(nullptr);   // flushes decode on the flushing thread's codec
        if (!_batch_devices.empty())
            _rx_batch->SetDevices(_batch_devices);
        const std::shared_ptr<WSReceiveBatch> batch = _rx_batch;
        const auto sessions = _sessions;
        locker.unlock();
        // outside the sessions lock: a session leaving a batch of its own
        // delivers the frames it queued there, and their callbacks may call
        // Multicast or sessions() (sessions added meanwhile got the batch
        // from AddSession)
        for (auto& s : sessions)
            s->SetReceiveBatch(batch.get());
        // a session removed meanwhile may have been attached after
        // RemoveSession detached it: detach it again
        std::vector<std::shared_ptr<WSSession>> removed;
        {
            std::shared_lock<std::shared_mutex> still(_sessions_lock);
            std::unordered_set<const WSSession*> live;
            for (auto& s : _sessions)
                live.insert(s.get());
            for (auto& s : sessions)
                if (!live.count(s.get()))
                    removed.push_back(s);
        }
        for (auto& s : removed)
            s->SwapReceiveBatch(nullptr, false);
        return;
    }
    // detach outside the sessions lock (see RemoveSession); a flush in
    // progress on another thread holds its own reference (FlushReceived),
    // so the batch is freed when its last user lets go, not here
    std::shared_ptr<WSReceiveBatch> gone = std::move(_rx_batch);
    const auto sessions = _sessions;
    locker.unlock();
    for (auto& s : sessions)
        s->SetReceiveBatch(nullptr);
    // a read that picked the batch up before its session let go framed its
    // frames into it: deliver them rather than lose them
    gone->Flush();
}

void WSServer::SetBatchDevices(const std::vector<int>& devices)
{
    std::unique_lock<std::shared_mutex> locker(_sessions_lock);
    _batch_devices = devices;
    if (_rx_batch)
        _rx_batch->SetDevices(devices);
    if (_tx_batch)
        _tx_batch->SetDevices(devices);
}

void WSServer::EnableBatchSend(bool on)
{
    if (!on)
        if (const auto b = tx_batch())
            b->Flush();   // nothing queued is lost
    std::unique_lock<std::shared_mutex> locker(_sessions_lock);
    if (on == (_tx_batch != nullptr))
        return;
    if (on) {
        _tx_batch = std::make_shared<WSSendBatch>(nullptr);
        if (!_batch_devices.empty())
            _tx_batch->SetDevices(_batch_devices);
        for (auto& s : _sessions)
            s->SetSendBatch(_tx_batch.get());
        return;
    }
    std::shared_ptr<WSSendBatch> gone = std::move(_tx_batch);
    const auto sessions = _sessions;
    locker.unlock();
    for (auto& s : sessions)
        s->SetSendBatch(nullptr);
    gone->Flush();   // frames queued between the flush above and the detach
}

size_t WSServer::FlushSend()
{
    const auto b = tx_batch();   // kept alive for the flush (see rx_batch)
    return b ? b->Flush() : 0;
}

size_t WSServer::FlushReceived()
{
    // not under _sessions_lock: callbacks may add or remove sessions
    const auto b = rx_batch();
    return b ? b->Flush() : 0;
}

size_t WSServer::sessions() const
{
    std::shared_lock<std::shared_mutex> locker(_sessions_lock);
    return _sessions.size();
}

bool WSServer::Multicast(const void* buffer, size_t size)
{
    if (size == 0)
        return true;
    if (buffer == nullptr)
        return false;
    if (const auto b = tx_batch())
        b->Flush();   // queued frames precede the multicast on every session
    else if (BatchScope::Active())
        BatchScope::Send().Flush();
    std::shared_lock<std::shared_mutex> locker(_sessions_lock);
    for (auto& session : _sessions) {
        std::scoped_lock ws_locker(session->_ws_send_lock);
        if (session->_ws_handshaked)
            session->_transport.SendAsync(buffer, size);
    }
    return true;
}

size_t WSServer::MulticastFrame(uint8_t opcode, const void* buffer, size_t size)
{
    const std::shared_ptr<WSSendBatch> own = tx_batch();
    WSSendBatch* batch = own ? own.get() : BatchScope::Active() ? &BatchScope::Send() : nullptr;
    if (batch && size) {
        // batched: the frame is encoded with the batch's other frames (one
        // GPU pass per tick, ws_multicast's `messages_rate` calls included)
        // and then queued on every session that was registered at this call
        // and is handshaked at the flush
        std::shared_ptr<const std::vector<std::shared_ptr<WSSession>>> group;
        {
            std::shared_lock<std::shared_mutex> locker(_sessions_lock);
            group = _snapshot;
        }
        uint32_t key;
        {
            std::scoped_lock locker(_ws_send_lock);
            key = send_key();
        }
        batch->QueueFanout(
            [group](const uint8_t* frame, size_t len) {
                if (!group)
                    return;
                for (const auto& session : *group) {
                    std::scoped_lock ws_locker(session->_ws_send_lock);
                    if (session->_ws_handshaked)
                        session->_transport.SendAsync(frame, len);
                }
            },
            key, opcode, false, buffer, size);
        if (batch != own.get())
            BatchScope::CheckLimits();
        return true;   // the reference returns Multicast()'s bool (ws_server.h:50-59)
    }
    std::scoped_lock locker(_ws_send_lock);
    PrepareSendFrame(opcode, false, buffer, size);
    return Multicast(_ws_send_buffer.data(), _ws_send_buffer.size());
}

bool WSServer::CloseAll(int status, const void* buffer, size_t size)
{
    std::vector<std::shared_ptr<WSSession>> all;
    {
        std::scoped_lock locker(_ws_send_lock);
        PrepareSendFrame(WS_FIN | WS_CLOSE, false, buffer, size, status);
        if (!Multicast(_ws_send_buffer.data(), _ws_send_buffer.size()))
            return false;
    }
    {
        std::shared_lock<std::shared_mutex> locker(_sessions_lock);
        all = _sessions;
    }
    for (auto& s : all)
        s->Disconnect();
    return true;
}

} // namespace WS
} // namespace CppServer
