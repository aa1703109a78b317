/*
 * server/ws/wss_server.h — WebSocket server over TLS.
 *
 * The reference's WSSServer (include/server/ws/wss_server.h) is WSServer over
 * HTTPSServer: Multicast and CloseAll encode once and send to every handshaked
 * WSSSession.  TLS is each session's Transport here, so WSSServer is WSServer
 * under the reference's name (batch receive/send included).
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
    using WSServer::WSServer;
};

} // namespace WS
} // namespace CppServer

#endif
