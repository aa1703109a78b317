/*
 * server/ws/wss_session.h — server-side WebSocket session over TLS.
 *
 * The reference's WSSSession (include/server/ws/wss_session.h) is WSSession
 * over HTTPSSession: same frames, same unmasked key-0 sends (ws.cpp:206),
 * TLS below.  TLS is the Transport's job here, so WSSSession is WSSession
 * under the reference's name.
 */
#ifndef CPPSERVER_AMD_WSS_SESSION_H
#define CPPSERVER_AMD_WSS_SESSION_H

#include "server/ws/ws_session.h"

namespace CppServer {
namespace WS {

class WSSSession : public WSSession
{
public:
    using WSSession::WSSession;
};

} // namespace WS
} // namespace CppServer

#endif
