/*
 * server/ws/ws_session.h — server-side WebSocket session over a Transport.
 *
 * Same surface as the reference WSSession (include/server/ws/ws_session.h:40-89):
 * sends are unmasked (mask = false) with the server key 0 (ws.cpp:206).
 */
#ifndef CPPSERVER_AMD_WS_SESSION_H
#define CPPSERVER_AMD_WS_SESSION_H

#include "server/ws/ws.h"
#include "server/ws/ws_batch.h"
#include "server/ws/ws_transport.h"

namespace CppServer {
namespace WS {

class WSServer;

class WSSession : protected WebSocket
{
    friend class WSServer;

public:
    explicit WSSession(Transport& transport, wsg_ctx* codec = nullptr) : WebSocket(codec), _transport(transport) {}
    virtual ~WSSession();

    //! Accept a connected transport: clear buffers and wait for the client's
    //! upgrade request, answered through onReceived (PerformServerUpgrade,
    //! reference ws_session.cpp:53-65)
    virtual bool Connect();
    virtual bool Disconnect();
    bool IsConnected() const { return _transport.IsConnected() && _ws_handshaked; }

    virtual bool Close() { return Close(0, nullptr, 0); }
    virtual bool Close(int status) { return Close(status, nullptr, 0); }
    virtual bool Close(int status, const void* buffer, size_t size) { SendCloseAsync(status, buffer, size); return Disconnect(); }
    virtual bool Close(int status, std::string_view text) { SendCloseAsync(status, text); return Disconnect(); }

    size_t SendText(const void* buffer, size_t size) { return SendFrame(WS_FIN | WS_TEXT, buffer, size); }
    size_t SendText(std::string_view text) { return SendFrame(WS_FIN | WS_TEXT, text.data(), text.size()); }
    size_t SendText(const void* buffer, size_t size, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_TEXT, buffer, size, 0, &timeout); }
    size_t SendText(std::string_view text, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_TEXT, text.data(), text.size(), 0, &timeout); }
    bool SendTextAsync(const void* buffer, size_t size) { return SendFrameAsync(WS_FIN | WS_TEXT, buffer, size); }
    bool SendTextAsync(std::string_view text) { return SendFrameAsync(WS_FIN | WS_TEXT, text.data(), text.size()); }

    size_t SendBinary(const void* buffer, size_t size) { return SendFrame(WS_FIN | WS_BINARY, buffer, size); }
    size_t SendBinary(std::string_view text) { return SendFrame(WS_FIN | WS_BINARY, text.data(), text.size()); }
    size_t SendBinary(const void* buffer, size_t size, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_BINARY, buffer, size, 0, &timeout); }
    size_t SendBinary(std::string_view text, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_BINARY, text.data(), text.size(), 0, &timeout); }
    bool SendBinaryAsync(const void* buffer, size_t size) { return SendFrameAsync(WS_FIN | WS_BINARY, buffer, size); }
    bool SendBinaryAsync(std::string_view text) { return SendFrameAsync(WS_FIN | WS_BINARY, text.data(), text.size()); }

    size_t SendClose(int status, const void* buffer, size_t size) { return SendFrame(WS_FIN | WS_CLOSE, buffer, size, status); }
    size_t SendClose(int status, std::string_view text) { return SendFrame(WS_FIN | WS_CLOSE, text.data(), text.size(), status); }
    size_t SendClose(int status, const void* buffer, size_t size, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_CLOSE, buffer, size, status, &timeout); }
    size_t SendClose(int status, std::string_view text, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_CLOSE, text.data(), text.size(), status, &timeout); }
    bool SendCloseAsync(int status, const void* buffer, size_t size) { return SendFrameAsync(WS_FIN | WS_CLOSE, buffer, size, status); }
    bool SendCloseAsync(int status, std::string_view text) { return SendFrameAsync(WS_FIN | WS_CLOSE, text.data(), text.size(), status); }

    size_t SendPing(const void* buffer, size_t size) { return SendFrame(WS_FIN | WS_PING, buffer, size); }
    size_t SendPing(std::string_view text) { return SendFrame(WS_FIN | WS_PING, text.data(), text.size()); }
    size_t SendPing(const void* buffer, size_t size, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_PING, buffer, size, 0, &timeout); }
    size_t SendPing(std::string_view text, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_PING, text.data(), text.size(), 0, &timeout); }
    bool SendPingAsync(const void* buffer, size_t size) { return SendFrameAsync(WS_FIN | WS_PING, buffer, size); }
    bool SendPingAsync(std::string_view text) { return SendFrameAsync(WS_FIN | WS_PING, text.data(), text.size()); }

    size_t SendPong(const void* buffer, size_t size) { return SendFrame(WS_FIN | WS_PONG, buffer, size); }
    size_t SendPong(std::string_view text) { return SendFrame(WS_FIN | WS_PONG, text.data(), text.size()); }
    size_t SendPong(const void* buffer, size_t size, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_PONG, buffer, size, 0, &timeout); }
    size_t SendPong(std::string_view text, const CppCommon::Timespan& timeout) { return SendFrame(WS_FIN | WS_PONG, text.data(), text.size(), 0, &timeout); }
    bool SendPongAsync(const void* buffer, size_t size) { return SendFrameAsync(WS_FIN | WS_PONG, buffer, size); }
    bool SendPongAsync(std::string_view text) { return SendFrameAsync(WS_FIN | WS_PONG, text.data(), text.size()); }

    std::string ReceiveText();
    std::string ReceiveText(const CppCommon::Timespan& timeout);
    std::vector<uint8_t> ReceiveBinary();
    std::vector<uint8_t> ReceiveBinary(const CppCommon::Timespan& timeout);

    //! Bytes read by the transport (reference ws_session.cpp:40-51).  With a
    //! receive batch set they are framed into the batch, and the onWS*
    //! callbacks fire at the batch's next Flush() (ws_batch.h).
    void onReceived(const void* buffer, size_t size);
    //! Route this session's receive path through `batch` (nullptr: per call)
    void SetReceiveBatch(WSReceiveBatch* batch);
    //! Route Send*Async through `batch`: frames are encoded at its next
    //! Flush() (nullptr: encode per call).  Sync Send* flush it first, so the
    //! connection's frames keep their order.
    void SetSendBatch(WSSendBatch* batch);
    //! Transport closed (reference ws_session.cpp:20-38)
    void onDisconnected();

protected:
    void onWSClose(const void* buffer, size_t size, int status = 1000) override { Close(); }
    void onWSPing(const void* buffer, size_t size) override { SendPongAsync(buffer, size); }
    //! The upgrade response goes out on the transport (reference ws_session.h:107)
    void SendResponse(const HTTP::HTTPResponse& response) override
    {
        _transport.SendAsync(response.cache().data(), response.cache().size());
    }

    Transport& _transport;

private:
    std::string _http_buf;   // upgrade request bytes until its header block is complete
    std::atomic<WSReceiveBatch*> _rx_batch{nullptr};   // swapped by SetReceiveBatch, read by the IO thread
    // SetReceiveBatch; deliver = false (WSServer::RemoveSession): the frames
    // it queued in the batch it leaves are dropped instead of delivered
    void SwapReceiveBatch(WSReceiveBatch* batch, bool deliver);
    std::atomic<WSSendBatch*> _tx_batch{nullptr};
    // held while a read (or a sync send) uses the batch it loaded; the swaps
    // take it, so a batch swapped out has no user left and may be freed
    QueueLock _rx_use, _tx_use;
    // a receive batch this connection is leaving (SetReceiveBatch): until its
    // queued frames of this connection are delivered, reads wait and a
    // ResetBuffers queues its reset there (both under _rx_use)
    bool _rx_draining = false;
    WSReceiveBatch* _rx_prev = nullptr;
    void ResetBuffers();
    void RouteFrames(const void* buffer, size_t size);
    size_t SendFrame(uint8_t opcode, const void* buffer, size_t size, int status = 0,
                     const CppCommon::Timespan* timeout = nullptr);
    bool SendFrameAsync(uint8_t opcode, const void* buffer, size_t size, int status = 0);
    bool ReceiveMessage(std::vector<uint8_t>& out, const CppCommon::Timespan* timeout = nullptr);
};

} // namespace WS
} // namespace CppServer

#endif // CPPSERVER_AMD_WS_SESSION_H
