// wss.cpp — WSSClient / WSSSession: the WebSocket classes over a
// TLSTransport (reference source/server/ws/wss_client.cpp,
// wss_session.cpp).  Host control plane; the frames go through the same
// codec paths as WSClient / WSSession.
#include "server/ws/wss_client.h"
#include "server/ws/wss_server.h"
#include "server/ws/wss_session.h"

namespace CppServer {
namespace WS {

bool WSSClient::Connect()
{
    _sync_connect = true;
    return _tls.lower().IsConnected() && _tls.Handshake();
}

bool WSSClient::ConnectAsync()
{
    _sync_connect = false;
    return _tls.lower().IsConnected() && _tls.Handshake();
}

void WSSClient::onHandshaked()
{
    // reference wss_client.cpp onHandshaked: the upgrade request, sent
    // synchronously after Connect and queued after ConnectAsync
    if (_sync_connect)
        WSClient::Connect();
    else
        WSClient::ConnectAsync();
}

void WSSClient::onReceived(const void* buffer, size_t size)
{
    const bool ok = _tls.Feed(
        buffer, size, [this](const void* p, size_t n) { WSClient::onReceived(p, n); }, [this] { onHandshaked(); });
    if (!ok) {
        onWSError("TLS error: " + _tls.error());
        WSClient::Disconnect();
    }
}

bool WSSSession::Connect()
{
    return WSSession::Connect() && _tls.Handshake();
}

void WSSSession::onReceived(const void* buffer, size_t size)
{
    const bool ok = _tls.Feed(
        buffer, size, [this](const void* p, size_t n) { WSSession::onReceived(p, n); }, [this] { onHandshaked(); });
    if (!ok) {
        onWSError("TLS error: " + _tls.error());
        WSSession::Disconnect();
    }
}

} // namespace WS
} // namespace CppServer
