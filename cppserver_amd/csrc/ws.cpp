// ws.cpp — CppServer::WS::WebSocket on the MI355X codec, and the
// wsg_session_* C-ABI entry points built on it.
//
// The per-connection header state machine runs on the host thread that owns
// the connection, exactly where the reference runs it; every masked
// payload byte (send mask, receive unmask, close-status bytes) is XORed by
// the gfx950 kernel behind wsg_xor_host.  Reference semantics followed:
// source/server/ws/ws.cpp:212-498, including the quirks of SURVEY.md §8a.
#include "server/ws/ws.h"
#include "wsg_env.h"
#include "server/ws/ws_handshake.h"
#include "ws_session_impl.h"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>
#include <string>

namespace CppServer {
namespace WS {

namespace {

struct ThreadCtx {
    wsg_ctx* ctx = nullptr;
    ~ThreadCtx()
    {
        if (ctx)
            wsg_destroy(ctx);
    }
};

void check(int rc, const char* what)
{
    if (rc != WSG_OK)
        throw std::runtime_error(std::string(what) + ": " + wsg_strerror(rc));
}

bool iequal(std::string_view a, std::string_view b)
{
    if (a.size() != b.size())
        return false;
    for (size_t i = 0; i < a.size(); ++i)
        if (std::tolower(static_cast<unsigned char>(a[i])) != std::tolower(static_cast<unsigned char>(b[i])))
            return false;
    return true;
}

std::string remove_blank(std::string_view s)
{
    std::string out;
    for (char c : s)
        if (!std::isspace(static_cast<unsigned char>(c)))
            out.push_back(c);
    return out;
}

uint32_t le32(const uint8_t k[4])
{
    return uint32_t(k[0]) | uint32_t(k[1]) << 8 | uint32_t(k[2]) << 16 | uint32_t(k[3]) << 24;
}

} // namespace

// The library's thread_locals use the initial-exec TLS model: a direct
// thread-pointer access.  Under the default model each access calls
// __tls_get_addr, and with glibc before 2.39 every call took its slow path
// once a later dlopen (the HIP runtime's) had raised the TLS generation: 8-9 %
// of a batched echo's host time (tools/sampler.cpp).  The library's TLS is
// 113 bytes, well inside the static TLS a dlopen (ctypes) may still take.
#define WSG_TLS __attribute__((tls_model("initial-exec")))

wsg_ctx* ThreadCodec()
{
    thread_local ThreadCtx holder WSG_TLS;
    if (!holder.ctx) {
        const char* dev = wsg::envp("WSG_DEVICE");
        check(wsg_create(dev ? std::atoi(dev) : 0, &holder.ctx), "wsg_create");
    }
    return holder.ctx;
}

wsg_ctx* WebSocket::codec() { return _codec ? _codec : ThreadCodec(); }

uint32_t WebSocket::send_key() const noexcept { return le32(_ws_send_mask); }

void WebSocket::set_send_key(uint32_t key) noexcept
{
    for (int j = 0; j < 4; ++j)
        _ws_send_mask[j] = uint8_t(key >> (8 * j));
}

void WebSocket::InitWSNonce()
{
    // one rand() byte per nonce byte, as the reference (ws.cpp:21-24)
    for (auto& b : _ws_nonce)
        b = uint8_t(std::rand());
}

bool WebSocket::PerformClientUpgrade(const HTTP::HTTPResponse& response)
{
    if (response.status() != 101)
        return false;
    bool error = false, accept = false, connection = false, upgrade = false;
    for (size_t i = 0; i < response.headers(); ++i) {
        const auto [key, value] = response.header(i);
        if (iequal(key, "Connection")) {
            if (!iequal(value, "Upgrade")) {
                error = true;
                onWSError("Invalid WebSocket handshaked response: 'Connection' header value must be 'Upgrade'");
                break;
            }
            connection = true;
        } else if (iequal(key, "Upgrade")) {
            if (!iequal(value, "websocket")) {
                error = true;
                onWSError("Invalid WebSocket handshaked response: 'Upgrade' header value must be 'websocket'");
                break;
            }
            upgrade = true;
        } else if (iequal(key, "Sec-WebSocket-Accept")) {
            const std::string expect = WSAcceptDigest(Base64Encode(ws_nonce()));
            const std::string got = Base64Decode(value);
            // compared as the reference does (ws.cpp:72-73): strncmp over the
            // shorter length, so the bytes after a NUL in either are not compared
            if (std::strncmp(got.c_str(), expect.c_str(), std::min(got.size(), expect.size())) != 0) {
                error = true;
                onWSError("Invalid WebSocket handshaked response: 'Sec-WebSocket-Accept' value validation failed");
                break;
            }
            accept = true;
        }
    }
    if (!accept || !connection || !upgrade) {
        if (!error)
            onWSError("Invalid WebSocket response");
        return false;
    }
    Handshaked(true);
    onWSConnected(response);
    return true;
}

bool WebSocket::PerformServerUpgrade(const HTTP::HTTPRequest& request, HTTP::HTTPResponse& response)
{
    if (request.method() != "GET")
        return false;
    bool error = false, connection = false, upgrade = false, ws_key = false, ws_version = false;
    std::string accept;
    for (size_t i = 0; i < request.headers(); ++i) {
        const auto [key, value] = request.header(i);
        if (iequal(key, "Connection")) {
            if (!iequal(value, "Upgrade") && !iequal(remove_blank(value), "keep-alive,Upgrade")) {
                error = true;
                response.MakeErrorResponse(400, "Invalid WebSocket handshaked request: 'Connection' header value "
                                                "must be 'Upgrade' or 'keep-alive, Upgrade'");
                break;
            }
            connection = true;
        } else if (iequal(key, "Upgrade")) {
            if (!iequal(value, "websocket")) {
                error = true;
                response.MakeErrorResponse(400, "Invalid WebSocket handshaked request: 'Upgrade' header value must "
                                                "be 'websocket'");
                break;
            }
            upgrade = true;
        } else if (iequal(key, "Sec-WebSocket-Key")) {
            if (value.empty()) {
                error = true;
                response.MakeErrorResponse(400, "Invalid WebSocket handshaked request: 'Sec-WebSocket-Key' header "
                                                "value must be non empty");
                break;
            }
            accept = WSAcceptKey(value);
            ws_key = true;
        } else if (iequal(key, "Sec-WebSocket-Version")) {
            if (!iequal(value, "13")) {
                error = true;
                response.MakeErrorResponse(400, "Invalid WebSocket handshaked request: 'Sec-WebSocket-Version' "
                                                "header value must be '13'");
                break;
            }
            ws_version = true;
        }
    }
    // not a WebSocket upgrade request at all: left to the HTTP layer
    if (!connection && !upgrade && !ws_key && !ws_version)
        return false;
    if (!connection || !upgrade || !ws_key || !ws_version) {
        if (!error)
            response.MakeErrorResponse(400, "Invalid WebSocket response");
        SendResponse(response);
        return false;
    }
    response.Clear();
    response.SetBegin(101, "HTTP/1.1");
    response.SetHeader("Connection", "Upgrade");
    response.SetHeader("Upgrade", "websocket");
    response.SetHeader("Sec-WebSocket-Accept", accept);
    response.SetBody();
    if (!onWSConnecting(request, response))
        return false;
    SendResponse(response);
    Handshaked(false);
    onWSConnected(request);
    return true;
}

void WebSocket::Handshaked(bool client)
{
    _ws_handshaked = true;
    // one key per connection: rand() for a client (ws.cpp:97; glibc rand()
    // never sets bit 31), 0 for a server session (ws.cpp:206)
    set_send_key(client ? uint32_t(std::rand()) : 0u);
}

void WebSocket::PrepareSendFrame(uint8_t opcode, bool mask, const void* buffer, size_t size, int status)
{
    const uint32_t key = send_key();
    const uint64_t total = wsg_frame_size(opcode, mask ? 1 : 0, size, status);
    _ws_send_buffer.resize(total);
    const int hdr = wsg_header_pack(opcode, mask ? 1 : 0, size, status, key, _ws_send_buffer.data());
    check(hdr < 0 ? hdr : WSG_OK, "wsg_header_pack");
    uint8_t* body = _ws_send_buffer.data() + hdr;
    const size_t prefix = size_t(total) - size_t(hdr) - size;   // close status bytes: 0 or 2
    if (prefix) {
        body[0] = uint8_t((status >> 8) & 0xFF);
        body[1] = uint8_t(status & 0xFF);
    }
    if (size)
        std::memcpy(body + prefix, buffer, size);
    // the XOR is applied whatever `mask` says (ws.cpp:269-270);
    // with the server key 0 it is the identity and there is nothing to run
    if (key != 0 && prefix + size != 0)
        check(wsg_xor_host(codec(), body, body, prefix + size, key, 0), "wsg_xor_host");
}

void WebSocket::ResetFrame()
{
    _ws_frame_received = false;
    _ws_header_size = 0;
    _ws_payload_size = 0;
    _ws_receive_frame_buffer.clear();
    std::memset(_ws_receive_mask, 0, sizeof(_ws_receive_mask));
}

void WebSocket::ResetMessage()
{
    _ws_final_received = false;
    _ws_receive_final_buffer.clear();
}

bool WebSocket::PullHeaderField(const uint8_t*& data, size_t& size, size_t want, uint8_t* mirror)
{
    for (size_t k = 0; k < want; ++k, ++data, --size) {
        if (size == 0)
            return false;
        _ws_receive_frame_buffer.push_back(*data);
        if (mirror)
            mirror[k] = *data;
    }
    return true;
}

void WebSocket::DispatchMessage(uint8_t opcode, const uint8_t* msg, size_t len)
{
    switch (opcode) {
    case WS_PING:
        onWSPing(msg, len);
        break;
    case WS_PONG:
        onWSPong(msg, len);
        break;
    case WS_CLOSE:
        // a 2-byte big-endian status leads the payload when present (ws.cpp:431-442)
        if (len >= 2)
            onWSClose(msg + 2, len - 2, (msg[0] << 8) | msg[1]);
        else
            onWSClose(msg, len, 1000);
        break;
    case WS_TEXT:
    case WS_BINARY:
        onWSReceived(msg, len);
        break;
    default:
        break;   // other opcodes are accumulated without a callback
    }
}

void WebSocket::PrepareReceiveFrame(const void* buffer, size_t size)
{
    const uint8_t* data = static_cast<const uint8_t*>(buffer);
    do {
        if (_ws_frame_received)
            ResetFrame();
        if (_ws_final_received)
            ResetMessage();
        if (size == 0)
            return;

        if (_ws_receive_frame_buffer.size() < 2 && !PullHeaderField(data, size, 2))
            return;
        const uint8_t b0 = _ws_receive_frame_buffer[0];
        const uint8_t b1 = _ws_receive_frame_buffer[1];
        const bool fin = (b0 & 0x80) != 0;
        const bool masked = (b1 & 0x80) != 0;
        if ((b0 & 0x0F) != 0)
            _ws_opcode = b0 & 0x0F;   // opcode 0 continues the previous message

        const size_t len7 = b1 & 0x7F;
        const size_t ext = len7 == 126 ? 2 : len7 == 127 ? 8 : 0;
        size_t len = len7;
        if (ext) {
            if (_ws_receive_frame_buffer.size() < 2 + ext && !PullHeaderField(data, size, ext))
                return;
            len = 0;
            for (size_t k = 0; k < ext; ++k)
                len = (len << 8) | _ws_receive_frame_buffer[2 + k];
        }
        _ws_header_size = 2 + ext + (masked ? 4 : 0);
        _ws_payload_size = len;
        _ws_receive_frame_buffer.reserve(_ws_header_size + _ws_payload_size);
        _ws_receive_final_buffer.reserve(_ws_header_size + _ws_payload_size);

        if (masked && _ws_receive_frame_buffer.size() < _ws_header_size &&
            !PullHeaderField(data, size, 4, _ws_receive_mask))
            return;

        const size_t total = _ws_header_size + _ws_payload_size;
        const size_t take = std::min(total - _ws_receive_frame_buffer.size(), size);
        _ws_receive_frame_buffer.insert(_ws_receive_frame_buffer.end(), data, data + take);
        data += take;
        size -= take;
        if (_ws_receive_frame_buffer.size() != total)
            continue;

        // frame complete: its payload joins the message, unmasked on the GPU
        const size_t base = _ws_receive_final_buffer.size();
        _ws_receive_final_buffer.resize(base + _ws_payload_size);
        const uint8_t* src = _ws_receive_frame_buffer.data() + _ws_header_size;
        const uint32_t key = le32(_ws_receive_mask);
        if (masked && key != 0 && _ws_payload_size != 0)
            check(wsg_xor_host(codec(), src, _ws_receive_final_buffer.data() + base, _ws_payload_size, key, 0),
                  "wsg_xor_host");
        else if (_ws_payload_size)
            std::memcpy(_ws_receive_final_buffer.data() + base, src, _ws_payload_size);
        _ws_frame_received = true;
        if (fin) {
            _ws_final_received = true;
            DispatchMessage(_ws_opcode, _ws_receive_final_buffer.data(), _ws_receive_final_buffer.size());
        }
    } while (size > 0);
}

void WebSocket::DeliverFrame(uint8_t opcode, bool fin, const uint8_t* payload, size_t len)
{
    if (_ws_final_received)
        ResetMessage();
    if (fin && _ws_receive_final_buffer.empty()) {
        // a whole message in one frame: hand out the decoded payload where it
        // lies (the reference hands out a pointer into its message buffer)
        _ws_final_received = true;
        DispatchMessage(opcode, payload, len);
        return;
    }
    _ws_receive_final_buffer.insert(_ws_receive_final_buffer.end(), payload, payload + len);
    if (fin) {
        _ws_final_received = true;
        DispatchMessage(opcode, _ws_receive_final_buffer.data(), _ws_receive_final_buffer.size());
    }
}

size_t WebSocket::RequiredReceiveFrameSize()
{
    if (_ws_frame_received)
        return 0;
    const size_t have = _ws_receive_frame_buffer.size();
    if (have < 2)
        return 2 - have;
    const uint8_t b1 = _ws_receive_frame_buffer[1];
    const size_t len7 = b1 & 0x7F;
    if (len7 == 126 && have < 4)
        return 4 - have;
    if (len7 == 127 && have < 10)
        return 10 - have;
    if ((b1 & 0x80) && have < _ws_header_size)
        return _ws_header_size - have;
    return _ws_header_size + _ws_payload_size - have;
}

void WebSocket::ClearWSBuffers()
{
    ResetFrame();
    ResetMessage();
    std::scoped_lock locker(_ws_send_lock);
    _ws_send_buffer.clear();
    std::memset(_ws_send_mask, 0, sizeof(_ws_send_mask));
}

} // namespace WS
} // namespace CppServer

// ===========================================================================
// C-ABI sessions (include/wsg_capi.h)
// ===========================================================================

thread_local wsg_rx_dispatch g_rx_dispatch WSG_TLS;

extern "C" {

int wsg_session_create(wsg_ctx* ctx, wsg_session** out)
{
    if (!ctx || !out)
        return WSG_EINVAL;
    try {
        *out = new wsg_session(ctx);
        return WSG_OK;
    } catch (...) {
        return WSG_ENOMEM;
    }
}

int wsg_session_destroy(wsg_session* s)
{
    if (!s)
        return WSG_EINVAL;
    delete s;
    return WSG_OK;
}

int wsg_session_set_send_key(wsg_session* s, uint32_t key)
{
    if (!s)
        return WSG_EINVAL;
    s->set_send_key(key);
    return WSG_OK;
}

int wsg_session_prepare_send(wsg_session* s, uint8_t opcode, int mask, const void* buf, size_t size, int32_t status,
                             uint8_t* out, size_t out_cap, size_t* out_len)
{
    if (!s || !out_len || (size && !buf))
        return WSG_EINVAL;
    try {
        std::scoped_lock locker(s->send_lock());
        s->PrepareSendFrame(opcode, mask != 0, buf, size, status);
        const auto& frame = s->send_buffer();
        *out_len = frame.size();
        if (frame.size() > out_cap || (frame.size() && !out))
            return WSG_ENOMEM;
        std::memcpy(out, frame.data(), frame.size());
        return WSG_OK;
    } catch (...) {
        return WSG_EHIP;
    }
}

int wsg_session_prepare_receive(wsg_session* s, const void* buf, size_t size, wsg_receive_cb cb, void* user)
{
    if (!s || (size && !buf))
        return WSG_EINVAL;
    s->cb = cb;
    s->user = user;
    try {
        s->PrepareReceiveFrame(buf, size);
    } catch (...) {
        s->cb = nullptr;
        return WSG_EHIP;
    }
    s->cb = nullptr;
    return WSG_OK;
}

size_t wsg_session_required(wsg_session* s) { return s ? s->RequiredReceiveFrameSize() : 0; }

int wsg_session_clear(wsg_session* s)
{
    if (!s)
        return WSG_EINVAL;
    s->ClearWSBuffers();
    return WSG_OK;
}

} // extern "C"
