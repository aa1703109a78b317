/*
 * server/ws/wss_session.h — server-side WebSocket session over TLS.
 *
 * The reference's WSSSession (include/server/ws/wss_session.h:24) is
 * WSSession over HTTPSSession: the same frames and upgrade answer, TLS below
 * them.  Here the inherited WSSession runs on a TLSTransport in the server
 * role (server/ws/tls_transport.h); the owner of the byte transport hands
 * the records it reads to onReceived.
 */
#ifndef CPPSERVER_AMD_WSS_SESSION_H
#define CPPSERVER_AMD_WSS_SESSION_H

#include "server/ws/wss_client.h"   // detail::TLSHolder
#include "server/ws/ws_session.h"

namespace CppServer {
namespace WS {

class WSSSession : private detail::TLSHolder, public WSSession
{
public:
    WSSSession(const std::shared_ptr<Asio::SSLContext>& context, Transport& transport, wsg_ctx* codec = nullptr)
        : TLSHolder(context, transport, TLSTransport::Role::server), WSSession(_tls, codec), _context(context)
    {
    }

    //! Accept: the TLS handshake starts with the client's hello, the
    //! upgrade request follows it (WSSession::Connect)
    bool Connect() override;
    //! TLS records read from the byte transport (see WSSClient::onReceived)
    void onReceived(const void* buffer, size_t size);

    const std::shared_ptr<Asio::SSLContext>& context() const noexcept { return _context; }
    TLSTransport& tls() noexcept { return _tls; }
    bool IsHandshaked() const { return _tls.IsHandshaked(); }

protected:
    //! TLS handshake done (reference SSLSession::onHandshaked)
    virtual void onHandshaked() {}

private:
    std::shared_ptr<Asio::SSLContext> _context;
};

} // namespace WS
} // namespace CppServer

#endif
