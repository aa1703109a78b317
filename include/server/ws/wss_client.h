/*
 * server/ws/wss_client.h — WebSocket client over TLS.
 *
 * The reference's WSSClient (include/server/ws/wss_client.h:26) is WSClient's
 * Send/Close/Receive surface over HTTPSClient: the frames, the masking and
 * the upgrade are identical, TLS record encryption sits below them, and the
 * upgrade request goes out when the TLS handshake completes
 * (wss_client.cpp onHandshaked; synchronously for Connect, queued for
 * ConnectAsync).  Here that layer is a TLSTransport (server/ws/
 * tls_transport.h: OpenSSL over the connection's byte Transport) that the
 * inherited WSClient runs on, so every Send* / Receive* / batching path of
 * WSClient works unchanged through it.
 *
 * The owner of the byte transport hands the records it reads to
 * onReceived (the reference's SSLClient::onReceived path); Connect /
 * ConnectAsync start the TLS handshake.
 */
#ifndef CPPSERVER_AMD_WSS_CLIENT_H
#define CPPSERVER_AMD_WSS_CLIENT_H

#include "server/asio/ssl_context.h"
#include "server/ws/tls_transport.h"
#include "server/ws/ws_client.h"

#include <memory>
#include <string>

namespace CppServer {
namespace WS {

namespace detail {
// the TLS layer, constructed before the WebSocket layer that runs on it
struct TLSHolder {
    TLSTransport _tls;
    TLSHolder(const std::shared_ptr<Asio::SSLContext>& context, Transport& lower, TLSTransport::Role role)
        : _tls(context, lower, role)
    {
    }
};
} // namespace detail

class WSSClient : private detail::TLSHolder, public WSClient
{
public:
    //! `transport` carries the TLS records (the reference's TCP socket)
    WSSClient(const std::shared_ptr<Asio::SSLContext>& context, Transport& transport, wsg_ctx* codec = nullptr)
        : TLSHolder(context, transport, TLSTransport::Role::client), WSClient(_tls, codec), _context(context)
    {
    }

    //! Start the TLS handshake; the upgrade request follows it with a sync
    //! Send (Connect) or SendAsync (ConnectAsync), reference wss_client.cpp
    bool Connect() override;
    bool ConnectAsync() override;

    //! TLS records read from the byte transport: decrypted and handed to the
    //! WebSocket layer (WSClient::onReceived); a TLS failure is reported
    //! through onWSError and disconnects
    void onReceived(const void* buffer, size_t size);

    const std::shared_ptr<Asio::SSLContext>& context() const noexcept { return _context; }
    TLSTransport& tls() noexcept { return _tls; }
    bool IsHandshaked() const { return _tls.IsHandshaked(); }

protected:
    //! TLS handshake done (reference SSLClient::onHandshaked): sends the upgrade
    virtual void onHandshaked();

private:
    std::shared_ptr<Asio::SSLContext> _context;
    bool _sync_connect{false};
};

} // namespace WS
} // namespace CppServer

#endif
