/*
 * server/ws/tls_transport.h — a TLS session over another Transport.
 *
 * The reference's WSS classes are its WS classes over SSLClient /
 * SSLSession (include/server/ws/wss_client.h:26, wss_session.h:24): asio's
 * ssl::stream encrypts below the WebSocket layer, and the WebSocket upgrade
 * starts when the TLS handshake is done (SSLClient::onHandshaked,
 * source/server/ws/wss_client.cpp).  Here TLSTransport is that layer: an
 * OpenSSL session with memory BIOs over any byte Transport (`lower`, which
 * carries the TLS records).  It is itself a Transport, so WSClient /
 * WSSession run on it unchanged — per-call and batched paths alike: a batch
 * flush hands each encoded frame to SendAsync, which encrypts it.
 *
 *  - Send / SendAsync: plaintext in, records out through lower.Send /
 *    lower.SendAsync (one call per Send, after SSL_write).  SendAsync calls
 *    made from inside Feed's callbacks (an echo, a batch flush at the end
 *    of a read) are held back and encrypted together when the callbacks
 *    return: full 16 KiB records instead of one record per frame; likewise
 *    SendAsync inside a BatchScope (an event-loop tick, ws_batch.h) is
 *    encrypted when the outermost scope on that thread ends.
 *  - Feed: records read from `lower` (what its owner's onReceived gets);
 *    advances the handshake, hands decrypted bytes to `plain` and calls
 *    `handshaked` once when the handshake completes.
 *  - Receive: the synchronous path (reference SSLClient::Receive): reads
 *    records from lower.Receive until plaintext is available.
 *
 * One TLSTransport per connection; its calls are serialized by an internal
 * mutex (an OpenSSL session is not thread-safe).
 */
#ifndef CPPSERVER_AMD_WS_TLS_TRANSPORT_H
#define CPPSERVER_AMD_WS_TLS_TRANSPORT_H

#include "server/asio/ssl_context.h"
#include "server/ws/ws_transport.h"

#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

typedef struct ssl_st SSL;
typedef struct bio_st BIO;

namespace CppServer {
namespace WS {

class TLSTransport : public Transport
{
public:
    enum class Role { client, server };

    TLSTransport(std::shared_ptr<Asio::SSLContext> context, Transport& lower, Role role);
    ~TLSTransport() override;
    TLSTransport(const TLSTransport&) = delete;
    TLSTransport& operator=(const TLSTransport&) = delete;

    //! Client: send the ClientHello (the handshake then advances in Feed);
    //! server: nothing to send, the handshake starts with the peer's hello.
    //! Returns false on a TLS error.
    bool Handshake();
    //! The whole handshake on the calling thread over lower.Send /
    //! lower.Receive (the reference's synchronous SSLClient::Connect)
    bool HandshakeSync();
    bool IsHandshaked() const;

    using Plain = std::function<void(const void* buffer, size_t size)>;
    //! Records read from `lower`; returns false on a TLS error (see error())
    bool Feed(const void* buffer, size_t size, const Plain& plain, const std::function<void()>& handshaked);

    size_t Send(const void* buffer, size_t size) override;
    bool SendAsync(const void* buffer, size_t size) override;
    size_t Receive(void* buffer, size_t size) override;
    size_t Send(const void* buffer, size_t size, const CppCommon::Timespan& timeout) override;
    size_t Receive(void* buffer, size_t size, const CppCommon::Timespan& timeout) override;
    //! Sends close_notify, then disconnects `lower`
    bool Disconnect() override;
    bool IsConnected() const override { return _lower.IsConnected(); }

    //! The last TLS error (OpenSSL's text), empty if none
    std::string error() const;
    //! Negotiated protocol ("TLSv1.3", ...) and cipher, once handshaked
    std::string protocol() const;
    std::string cipher() const;

    Transport& lower() noexcept { return _lower; }

private:
    std::shared_ptr<Asio::SSLContext> _context;
    Transport& _lower;
    Role _role;
    SSL* _ssl{nullptr};
    BIO* _rbio{nullptr};   // records in (owned by _ssl)
    BIO* _wbio{nullptr};   // records out (owned by _ssl)
    bool _handshaked{false};
    bool _failed{false};
    std::string _error;
    std::vector<uint8_t> _pending;   // plaintext decrypted by Receive beyond what was asked
    size_t _pending_at{0};
    std::vector<uint8_t> _out_plain;   // SendAsync bytes held back while a Feed runs its callbacks / a batch scope is open
    int _feeding{0};
    bool _scope_held{false};           // registered to flush _out_plain when this thread's batch scope ends
    mutable std::recursive_mutex _lock;

    // encrypted bytes waiting in _wbio (handshake records, application records)
    std::vector<uint8_t> drain_records();
    // SSL_do_handshake step; true when done (sets _handshaked)
    bool step_handshake();
    bool fail(const char* what);
    size_t encrypt(const void* buffer, size_t size, std::vector<uint8_t>& records);
    size_t encrypt_after_pending(const void* buffer, size_t size, std::vector<uint8_t>& records);
    static void scope_end(void* self);
};

} // namespace WS
} // namespace CppServer

#endif // CPPSERVER_AMD_WS_TLS_TRANSPORT_H
