/*
 * server/ws/ws.h — CppServer::WS::WebSocket for the MI355X codec.
 *
 * Drop-in for the reference mix-in class (include/server/ws/ws.h:29 of
 * chronoxor/CppServer 1.0.5.0): same constants, same per-connection state,
 * same PrepareSendFrame / PrepareReceiveFrame / RequiredReceiveFrameSize /
 * ClearWSBuffers contract and onWS* callbacks.  The payload mask/unmask of
 * every frame runs on the GPU through the C-ABI (include/wsg_capi.h); the
 * header state machine stays on the host thread that owns the connection,
 * as it does in the reference.
 *
 * The upgrade handshake is here too:
 * PerformClientUpgrade / PerformServerUpgrade over the HTTP request/response
 * subset of include/server/http/, with the reference's onWSConnecting /
 * onWSConnected hooks.  The reference's client variant also takes the
 * connection's UUID (ws.h:62), which its body does not use; both forms are
 * here.
 */
#ifndef CPPSERVER_AMD_WS_H
#define CPPSERVER_AMD_WS_H

#include "wsg_capi.h"
#include "server/http/http_request.h"
#include "server/ws/ws_common.h"
#include "server/http/http_response.h"

#include <array>
#include <cstddef>
#include <cstdint>
#include <mutex>
#include <string>
#include <string_view>
#include <vector>

namespace CppServer {
namespace WS {

class WSReceiveBatch;

//! GPU codec context of the calling thread (one wsg_ctx per host thread,
//! device from $WSG_DEVICE, default 0).  Throws std::runtime_error when no
//! device is available: there is no CPU fallback.
wsg_ctx* ThreadCodec();

class WebSocket
{
public:
    // First-byte values; callers pass WS_FIN | opcode as the whole byte.
    static const uint8_t WS_FIN = WSG_FIN;
    static const uint8_t WS_TEXT = WSG_TEXT;
    static const uint8_t WS_BINARY = WSG_BINARY;
    static const uint8_t WS_CLOSE = WSG_CLOSE;
    static const uint8_t WS_PING = WSG_PING;
    static const uint8_t WS_PONG = WSG_PONG;

    WebSocket() { ClearWSBuffers(); InitWSNonce(); }
    //! Bind the connection to an explicit codec context (else ThreadCodec()).
    explicit WebSocket(wsg_ctx* codec) : _codec(codec) { ClearWSBuffers(); InitWSNonce(); }
    WebSocket(const WebSocket&) = delete;
    WebSocket(WebSocket&&) = delete;
    virtual ~WebSocket() = default;

    WebSocket& operator=(const WebSocket&) = delete;
    WebSocket& operator=(WebSocket&&) = delete;

    std::string_view ws_nonce() const noexcept { return std::string_view((const char*)_ws_nonce.data(), _ws_nonce.size()); }

    //! Prepare WebSocket send frame into _ws_send_buffer (reference ws.cpp:212)
    void PrepareSendFrame(uint8_t opcode, bool mask, const void* buffer, size_t size, int status = 0);
    //! Prepare WebSocket receive frame, firing onWS* callbacks (reference ws.cpp:273)
    void PrepareReceiveFrame(const void* buffer, size_t size);
    //! Required WebSocket receive frame size (reference ws.cpp:458)
    size_t RequiredReceiveFrameSize();
    //! Clear WebSocket send/receive buffers (reference ws.cpp:484)
    void ClearWSBuffers();
    //! Initialize WebSocket random nonce
    void InitWSNonce();

    //! Validate the server's upgrade response (reference ws.cpp:26-101):
    //! status 101, Connection: Upgrade, Upgrade: websocket and the
    //! Sec-WebSocket-Accept digest of this connection's nonce.  On success
    //! the connection is handshaked with a random send key, onWSConnected(response).
    bool PerformClientUpgrade(const HTTP::HTTPResponse& response);
    //! The reference's signature (ws.h:62): the connection id is not used
    bool PerformClientUpgrade(const HTTP::HTTPResponse& response, const CppCommon::UUID& id)
    {
        (void)id;
        return PerformClientUpgrade(response);
    }
    //! Answer a client's upgrade request (reference ws.cpp:103-210): validate
    //! it, build the 101 response (or a 400 error), let onWSConnecting veto
    //! it, SendResponse(), handshake with send key 0, onWSConnected(request).
    //! Returns false for a request that is not a WebSocket upgrade at all.
    bool PerformServerUpgrade(const HTTP::HTTPRequest& request, HTTP::HTTPResponse& response);

    //! Mark the upgrade as done and install the send key: a client draws a
    //! random key per connection (reference ws.cpp:97), a server session
    //! uses 0 (ws.cpp:206).
    void Handshaked(bool client);
    bool IsHandshaked() const noexcept { return _ws_handshaked; }
    //! Current send key as the little-endian uint32 the ABI carries.
    uint32_t send_key() const noexcept;
    void set_send_key(uint32_t key) noexcept;

protected:
    //! Codec context of this connection (the explicit one, else ThreadCodec())
    wsg_ctx* codec();

    //! Client: fill the upgrade request (reference ws.h:107)
    virtual void onWSConnecting(HTTP::HTTPRequest& request) {}
    //! Client: upgrade accepted (reference ws.h:112)
    virtual void onWSConnected(const HTTP::HTTPResponse& response) {}
    //! Server: veto or amend the upgrade response (reference ws.h:124)
    virtual bool onWSConnecting(const HTTP::HTTPRequest& request, HTTP::HTTPResponse& response) { return true; }
    //! Server: upgrade done (reference ws.h:129)
    virtual void onWSConnected(const HTTP::HTTPRequest& request) {}
    virtual void onWSDisconnected() {}
    virtual void onWSReceived(const void* buffer, size_t size) {}
    virtual void onWSClose(const void* buffer, size_t size, int status = 1000) {}
    virtual void onWSPing(const void* buffer, size_t size) {}
    virtual void onWSPong(const void* buffer, size_t size) {}
    virtual void onWSError(const std::string& message) {}

    //! Send the upgrade response (reference ws.h:202; sessions override it)
    virtual void SendResponse(const HTTP::HTTPResponse& response) {}

protected:
    // Per-connection codec state, named as in the reference so that
    // subclasses written against it keep compiling.
    bool _ws_handshaked{false};

    // receive side: opcode of the message being assembled (0 here where the
    // reference leaves it uninitialised), frame/message completion flags,
    // geometry of the current frame, the raw frame, the unmasked message
    // and the current frame's key
    uint8_t _ws_opcode{0};
    bool _ws_frame_received{false};
    bool _ws_final_received{false};
    size_t _ws_header_size{0};
    size_t _ws_payload_size{0};
    std::vector<uint8_t> _ws_receive_frame_buffer;
    std::vector<uint8_t> _ws_receive_final_buffer;
    uint8_t _ws_receive_mask[4]{};

    // send side: the lock every Send* wrapper holds, the encoded frame and
    // the per-connection key
    std::mutex _ws_send_lock;
    std::vector<uint8_t> _ws_send_buffer;
    uint8_t _ws_send_mask[4]{};

    std::array<uint8_t, 16> _ws_nonce{};

private:
    friend class WSReceiveBatch;   // batched receive: framing here, unmask in one launch per flush

    wsg_ctx* _codec{nullptr};
    // append `want` bytes of the input to the frame buffer (full field width,
    // the reference's split-header behaviour)
    bool PullHeaderField(const uint8_t*& data, size_t& size, size_t want, uint8_t* mirror = nullptr);
    void ResetFrame();
    void ResetMessage();
    void DispatchMessage(uint8_t opcode, const uint8_t* msg, size_t len);
    // message half of PrepareReceiveFrame for one decoded frame (batched
    // receive): append to the message, dispatch on FIN (ws.cpp:399-452)
    void DeliverFrame(uint8_t opcode, bool fin, const uint8_t* payload, size_t len);
};

} // namespace WS
} // namespace CppServer

#endif // CPPSERVER_AMD_WS_H
