/*
 * server/ws/wss_client.h — WebSocket client over TLS.
 *
 * The reference's WSSClient (include/server/ws/wss_client.h:26) is WSClient's
 * Send/Close/Receive surface over HTTPSClient instead of HTTPClient: the
 * frames, the masking and the upgrade handshake are identical, TLS record
 * encryption sits below them.  Here TLS is the Transport's job (a Transport
 * whose Send/Receive run through the TLS session), so WSSClient is WSClient
 * under the reference's name.
 */
#ifndef CPPSERVER_AMD_WSS_CLIENT_H
#define CPPSERVER_AMD_WSS_CLIENT_H

#include "server/ws/ws_client.h"

namespace CppServer {
namespace WS {

class WSSClient : public WSClient
{
public:
    using WSClient::WSClient;
};

} // namespace WS
} // namespace CppServer

#endif
