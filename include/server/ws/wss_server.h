/*
 * server/ws/wss_server.h — WebSocket server over TLS.
 *
 * The reference's WSSServer (include/server/ws/wss_server.h:24) is WSServer
 * over HTTPSServer: the same Multicast* / CloseAll over sessions whose bytes
 * cross TLS.  Here it is WSServer holding the SSL context its WSSSession
 * objects are made with (context()); every multicast and batched path
 * reaches the sessions' TLS transports through WSSession.
 */
#ifndef CPPSERVER_AMD_WSS_SERVER_H
#define CPPSERVER_AMD_WSS_SERVER_H

#include "server/ws/ws_server.h"
#include "server/ws/wss_session.h"

namespace CppServer {
namespace WS {

class WSSServer : public WSServer
{
public:
    explicit WSSServer(const std::shared_ptr<Asio::SSLContext>& context, wsg_ctx* codec = nullptr)
        : WSServer(codec), _context(context)
    {
    }

    //! The context sessions of this server are made with (reference SSLServer::context)
    const std::shared_ptr<Asio::SSLContext>& context() const noexcept { return _context; }

private:
    std::shared_ptr<Asio::SSLContext> _context;
};

} // namespace WS
} // namespace CppServer

#endif
