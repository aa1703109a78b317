/*
 * server/ws/ws_transport.h — the byte transport under a WebSocket connection.
 *
 * In the reference this role is played by Asio's TCPClient / TCPSession
 * (source/server/asio/tcp_client.cpp Send/SendAsync, tcp_session.cpp:257-307
 * SendAsync, :429-485 TryReceive -> onReceived).  Sockets are out of scope
 * for the MI355X build: a deployment plugs its own
 * transport in here and calls WSClient/WSSession::onReceived with the bytes
 * it reads, exactly where TCPSession::TryReceive calls onReceived.
 */
#ifndef CPPSERVER_AMD_WS_TRANSPORT_H
#define CPPSERVER_AMD_WS_TRANSPORT_H

#include "server/ws/ws_common.h"

#include <cstddef>

namespace CppServer {
namespace WS {

class Transport
{
public:
    virtual ~Transport() = default;
    //! Send synchronously; returns the bytes sent (TCPClient::Send)
    virtual size_t Send(const void* buffer, size_t size) = 0;
    //! Queue for sending; the transport copies the bytes (TCPSession::SendAsync)
    virtual bool SendAsync(const void* buffer, size_t size) = 0;
    //! Blocking receive of up to size bytes (TCPClient::Receive)
    virtual size_t Receive(void* buffer, size_t size) = 0;
    //! The same with a timeout (TCPClient::Send / Receive(..., timeout)); a
    //! transport without timeouts of its own may keep these defaults
    virtual size_t Send(const void* buffer, size_t size, const CppCommon::Timespan& timeout)
    {
        (void)timeout;
        return Send(buffer, size);
    }
    virtual size_t Receive(void* buffer, size_t size, const CppCommon::Timespan& timeout)
    {
        (void)timeout;
        return Receive(buffer, size);
    }
    virtual bool Disconnect() = 0;
    virtual bool IsConnected() const = 0;
};

} // namespace WS
} // namespace CppServer

#endif // CPPSERVER_AMD_WS_TRANSPORT_H
