/*
 * server/asio/ssl_context.h — TLS context of the WSS classes.
 *
 * The reference's CppServer::Asio::SSLContext (include/server/asio/
 * ssl_context.h:24) is asio::ssl::context plus set_root_certs(); its WSS
 * examples configure it through asio's member functions
 * (examples/wss_chat_server.cpp:98-102, wss_chat_client.cpp:105-109,
 * performance/wss_echo_client.cpp:144-148).  Here the same class name and
 * the same member functions sit directly on an OpenSSL SSL_CTX (the library
 * asio::ssl wraps), so that this configuration code compiles unchanged.
 * Failures throw std::runtime_error carrying OpenSSL's error text (asio
 * throws asio::system_error from the same calls).
 *
 * Without Asio on the include path, a minimal `asio::ssl` namespace supplies
 * the names that configuration code spells through asio
 * (asio::ssl::context::tlsv13, asio::ssl::context::pem,
 * asio::ssl::context::password_purpose, asio::ssl::verify_peer, ...), as
 * server/ws/ws_common.h does for CppCommon.
 */
#ifndef CPPSERVER_AMD_ASIO_SSL_CONTEXT_H
#define CPPSERVER_AMD_ASIO_SSL_CONTEXT_H

#include <cstddef>
#include <functional>
#include <memory>
#include <mutex>
#include <string>

typedef struct ssl_ctx_st SSL_CTX;

namespace CppServer {
namespace Asio {

class SSLContext
{
public:
    //! asio::ssl::context::method values the reference uses, plus the generic ones
    enum method { sslv23, tls, tlsv12, tlsv13, tls_client, tls_server, tlsv12_client, tlsv12_server, tlsv13_client, tlsv13_server };
    enum file_format { asn1, pem };
    enum password_purpose { for_reading, for_writing };

    explicit SSLContext(method m);
    SSLContext(const SSLContext&) = delete;
    SSLContext(SSLContext&&) = delete;
    ~SSLContext();
    SSLContext& operator=(const SSLContext&) = delete;
    SSLContext& operator=(SSLContext&&) = delete;

    //! Pass phrase of encrypted private keys (asio: set_password_callback)
    void set_password_callback(std::function<std::string(std::size_t, password_purpose)> callback);
    //! Certificate chain (leaf first) from a PEM file / PEM bytes
    void use_certificate_chain_file(const std::string& filename);
    void use_certificate_chain(const void* pem, std::size_t size);
    //! Private key from a file / bytes (PEM or DER)
    void use_private_key_file(const std::string& filename, file_format format);
    void use_private_key(const void* data, std::size_t size, file_format format);
    //! Diffie-Hellman parameters for the DHE suites (TLS 1.2); OpenSSL 3
    //! picks FFDHE groups by itself, the file is loaded and checked
    void use_tmp_dh_file(const std::string& filename);
    //! Peer verification: verify_peer | verify_fail_if_no_peer_cert | ...
    void set_verify_mode(int mode);
    //! Trusted CAs: the system store, a PEM file, PEM bytes
    void set_default_verify_paths();
    void load_verify_file(const std::string& filename);
    void add_certificate_authority(const void* pem, std::size_t size);
    //! The reference's addition: the platform root certificates
    //! (reference source/server/asio/ssl_context.cpp; here the OpenSSL
    //! default store, as set_default_verify_paths)
    void set_root_certs();

    SSL_CTX* native_handle() const noexcept { return _ctx; }

private:
    SSL_CTX* _ctx{nullptr};
    std::function<std::string(std::size_t, password_purpose)> _password;
    static int password_thunk(char* buf, int size, int rwflag, void* user);
};

constexpr int verify_none = 0x00;
constexpr int verify_peer = 0x01;
constexpr int verify_fail_if_no_peer_cert = 0x02;
constexpr int verify_client_once = 0x04;

} // namespace Asio
} // namespace CppServer

#if !defined(ASIO_VERSION) && !defined(WSG_NO_ASIO_NAMES)
// the asio::ssl names of context configuration code (see the header comment)
namespace asio {
namespace ssl {
using context = CppServer::Asio::SSLContext;
using CppServer::Asio::verify_client_once;
using CppServer::Asio::verify_fail_if_no_peer_cert;
using CppServer::Asio::verify_none;
using CppServer::Asio::verify_peer;
} // namespace ssl
} // namespace asio
#endif

#endif // CPPSERVER_AMD_ASIO_SSL_CONTEXT_H
