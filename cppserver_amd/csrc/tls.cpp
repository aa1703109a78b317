// tls.cpp — SSLContext (OpenSSL SSL_CTX) and TLSTransport (an OpenSSL
// session with memory BIOs over a byte Transport): the TLS layer under the
// WSS classes (reference include/server/ws/wss_*.h over
// include/server/asio/ssl_*.h).  Host control plane; no GPU code.
#include "server/asio/ssl_context.h"
#include "server/ws/tls_transport.h"
#include "server/ws/ws_batch.h"

#include <openssl/bio.h>
#include <openssl/err.h>
#include <openssl/pem.h>
#include <openssl/ssl.h>
#include <openssl/x509.h>

#include <cstring>
#include <stdexcept>

namespace CppServer {
namespace Asio {

namespace {

std::string ossl_error(const char* what)
{
    std::string s = what;
    unsigned long e;
    char buf[256];
    bool first = true;
    while ((e = ERR_get_error()) != 0) {
        ERR_error_string_n(e, buf, sizeof buf);
        s += first ? ": " : "; ";
        s += buf;
        first = false;
    }
    return s;
}

[[noreturn]] void raise(const char* what) { throw std::runtime_error(ossl_error(what)); }

struct BioMem {
    BIO* b;
    BioMem(const void* p, std::size_t n) : b(BIO_new_mem_buf(p, int(n))) {}
    ~BioMem() { BIO_free(b); }
};

} // namespace

SSLContext::SSLContext(method m)
{
    const SSL_METHOD* meth = TLS_method();
    switch (m) {
    case tls_client:
    case tlsv12_client:
    case tlsv13_client:
        meth = TLS_client_method();
        break;
    case tls_server:
    case tlsv12_server:
    case tlsv13_server:
        meth = TLS_server_method();
        break;
    default:
        break;
    }
    _ctx = SSL_CTX_new(meth);
    if (!_ctx)
        raise("SSL_CTX_new");
    // tlsvNN: exactly that version, as asio's context does
    int v = 0;
    if (m == tlsv12 || m == tlsv12_client || m == tlsv12_server)
        v = TLS1_2_VERSION;
    if (m == tlsv13 || m == tlsv13_client || m == tlsv13_server)
        v = TLS1_3_VERSION;
    if (v && (!SSL_CTX_set_min_proto_version(_ctx, v) || !SSL_CTX_set_max_proto_version(_ctx, v)))
        raise("SSL_CTX_set_proto_version");
    SSL_CTX_set_mode(_ctx, SSL_MODE_ACCEPT_MOVING_WRITE_BUFFER);
    SSL_CTX_set_default_passwd_cb(_ctx, &SSLContext::password_thunk);
    SSL_CTX_set_default_passwd_cb_userdata(_ctx, this);
}

SSLContext::~SSLContext()
{
    if (_ctx)
        SSL_CTX_free(_ctx);
}

int SSLContext::password_thunk(char* buf, int size, int rwflag, void* user)
{
    auto* self = static_cast<SSLContext*>(user);
    if (!self || !self->_password || size <= 0)
        return 0;
    const std::string p = self->_password(std::size_t(size), rwflag ? for_writing : for_reading);
    const int n = int(std::min<std::size_t>(p.size(), std::size_t(size)));
    std::memcpy(buf, p.data(), std::size_t(n));
    return n;
}

void SSLContext::set_password_callback(std::function<std::string(std::size_t, password_purpose)> callback)
{
    _password = std::move(callback);
}

void SSLContext::use_certificate_chain_file(const std::string& filename)
{
    if (SSL_CTX_use_certificate_chain_file(_ctx, filename.c_str()) != 1)
        raise("use_certificate_chain_file");
}

void SSLContext::use_certificate_chain(const void* pem, std::size_t size)
{
    BioMem bio(pem, size);
    X509* leaf = PEM_read_bio_X509_AUX(bio.b, nullptr, &SSLContext::password_thunk, this);
    if (!leaf)
        raise("use_certificate_chain");
    const int ok = SSL_CTX_use_certificate(_ctx, leaf);
    X509_free(leaf);
    if (ok != 1)
        raise("use_certificate_chain");
    SSL_CTX_clear_chain_certs(_ctx);
    while (X509* ca = PEM_read_bio_X509(bio.b, nullptr, &SSLContext::password_thunk, this)) {
        if (SSL_CTX_add0_chain_cert(_ctx, ca) != 1) {
            X509_free(ca);
            raise("use_certificate_chain");
        }
    }
    ERR_clear_error();   // the end of the PEM stream reads as an error
}

void SSLContext::use_private_key_file(const std::string& filename, file_format format)
{
    if (SSL_CTX_use_PrivateKey_file(_ctx, filename.c_str(), format == pem ? SSL_FILETYPE_PEM : SSL_FILETYPE_ASN1) != 1)
        raise("use_private_key_file");
}

void SSLContext::use_private_key(const void* data, std::size_t size, file_format format)
{
    BioMem bio(data, size);
    EVP_PKEY* key = format == pem ? PEM_read_bio_PrivateKey(bio.b, nullptr, &SSLContext::password_thunk, this)
                                  : d2i_PrivateKey_bio(bio.b, nullptr);
    if (!key)
        raise("use_private_key");
    const int ok = SSL_CTX_use_PrivateKey(_ctx, key);
    EVP_PKEY_free(key);
    if (ok != 1)
        raise("use_private_key");
}

void SSLContext::use_tmp_dh_file(const std::string& filename)
{
    BIO* bio = BIO_new_file(filename.c_str(), "r");
    if (!bio)
        raise("use_tmp_dh_file");
    EVP_PKEY* dh = PEM_read_bio_Parameters(bio, nullptr);
    BIO_free(bio);
    if (!dh)
        raise("use_tmp_dh_file");
    if (SSL_CTX_set0_tmp_dh_pkey(_ctx, dh) != 1) {   // takes ownership on success
        EVP_PKEY_free(dh);
        raise("use_tmp_dh_file");
    }
}

void SSLContext::set_verify_mode(int mode)
{
    int m = SSL_VERIFY_NONE;
    if (mode & verify_peer)
        m |= SSL_VERIFY_PEER;
    if (mode & verify_fail_if_no_peer_cert)
        m |= SSL_VERIFY_FAIL_IF_NO_PEER_CERT;
    if (mode & verify_client_once)
        m |= SSL_VERIFY_CLIENT_ONCE;
    SSL_CTX_set_verify(_ctx, m, nullptr);
}

void SSLContext::set_default_verify_paths()
{
    if (SSL_CTX_set_default_verify_paths(_ctx) != 1)
        raise("set_default_verify_paths");
}

void SSLContext::set_root_certs() { set_default_verify_paths(); }

void SSLContext::load_verify_file(const std::string& filename)
{
    if (SSL_CTX_load_verify_locations(_ctx, filename.c_str(), nullptr) != 1)
        raise("load_verify_file");
}

void SSLContext::add_certificate_authority(const void* pem, std::size_t size)
{
    BioMem bio(pem, size);
    X509_STORE* store = SSL_CTX_get_cert_store(_ctx);
    int added = 0;
    while (X509* ca = PEM_read_bio_X509(bio.b, nullptr, nullptr, nullptr)) {
        const int ok = X509_STORE_add_cert(store, ca);
        X509_free(ca);
        if (ok != 1)
            raise("add_certificate_authority");
        ++added;
    }
    ERR_clear_error();
    if (!added)
        throw std::runtime_error("add_certificate_authority: no certificate in the PEM data");
}

} // namespace Asio

namespace WS {

TLSTransport::TLSTransport(std::shared_ptr<Asio::SSLContext> context, Transport& lower, Role role)
    : _context(std::move(context)), _lower(lower), _role(role)
{
    if (!_context || !_context->native_handle())
        throw std::invalid_argument("TLSTransport: no SSL context");
    _ssl = SSL_new(_context->native_handle());
    _rbio = BIO_new(BIO_s_mem());
    _wbio = BIO_new(BIO_s_mem());
    if (!_ssl || !_rbio || !_wbio) {
        if (_rbio)
            BIO_free(_rbio);
        if (_wbio)
            BIO_free(_wbio);
        if (_ssl)
            SSL_free(_ssl);
        throw std::runtime_error(Asio::ossl_error("TLSTransport"));
    }
    BIO_set_mem_eof_return(_rbio, -1);   // an empty input BIO means "retry", not EOF
    SSL_set_bio(_ssl, _rbio, _wbio);     // _ssl owns both
    if (_role == Role::client)
        SSL_set_connect_state(_ssl);
    else
        SSL_set_accept_state(_ssl);
}

TLSTransport::~TLSTransport()
{
    BatchScope::Cancel(this);
    if (_ssl)
        SSL_free(_ssl);
}

void TLSTransport::scope_end(void* self)
{
    auto* t = static_cast<TLSTransport*>(self);
    std::lock_guard<std::recursive_mutex> g(t->_lock);
    t->_scope_held = false;
    if (t->_out_plain.empty() || t->_feeding)
        return;
    std::vector<uint8_t> p, rec;
    p.swap(t->_out_plain);
    t->encrypt(p.data(), p.size(), rec);
    if (!rec.empty())
        t->_lower.SendAsync(rec.data(), rec.size());
}

bool TLSTransport::fail(const char* what)
{
    _failed = true;
    _error = Asio::ossl_error(what);
    return false;
}

std::vector<uint8_t> TLSTransport::drain_records()
{
    std::vector<uint8_t> out;
    const size_t avail = size_t(BIO_ctrl_pending(_wbio));
    if (!avail)
        return out;
    out.resize(avail);
    const int n = BIO_read(_wbio, out.data(), int(avail));
    out.resize(n > 0 ? size_t(n) : 0);
    return out;
}

bool TLSTransport::step_handshake()
{
    if (_handshaked)
        return true;
    const int r = SSL_do_handshake(_ssl);
    if (r == 1) {
        _handshaked = true;
        return true;
    }
    const int e = SSL_get_error(_ssl, r);
    if (e != SSL_ERROR_WANT_READ && e != SSL_ERROR_WANT_WRITE)
        fail("TLS handshake");
    return false;
}

bool TLSTransport::Handshake()
{
    std::vector<uint8_t> out;
    {
        std::lock_guard<std::recursive_mutex> g(_lock);
        if (_failed)
            return false;
        if (_role == Role::server)
            return true;   // waits for the ClientHello (Feed)
        step_handshake();
        if (_failed)
            return false;
        out = drain_records();
        return out.empty() || _lower.SendAsync(out.data(), out.size());
    }
}

bool TLSTransport::HandshakeSync()
{
    std::vector<uint8_t> in(16384);
    for (int guard = 0; guard < 1000; ++guard) {
        std::vector<uint8_t> out;
        bool done;
        {
            std::lock_guard<std::recursive_mutex> g(_lock);
            if (_failed)
                return false;
            done = step_handshake();
            if (_failed)
                return false;
            out = drain_records();
        }
        if (!out.empty() && _lower.Send(out.data(), out.size()) != out.size())
            return false;
        if (done)
            return true;
        const size_t n = _lower.Receive(in.data(), in.size());
        if (n == 0)
            return false;
        std::lock_guard<std::recursive_mutex> g(_lock);
        if (BIO_write(_rbio, in.data(), int(n)) != int(n))
            return fail("BIO_write");
    }
    return false;
}

bool TLSTransport::IsHandshaked() const
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    return _handshaked;
}

bool TLSTransport::Feed(const void* buffer, size_t size, const Plain& plain, const std::function<void()>& handshaked)
{
    std::vector<uint8_t> out, text;
    bool just_handshaked = false;
    {
        std::lock_guard<std::recursive_mutex> g(_lock);
        if (_failed)
            return false;
        ++_feeding;
        if (size && BIO_write(_rbio, buffer, int(size)) != int(size)) {
            --_feeding;
            return fail("BIO_write");
        }
        if (!_handshaked) {
            just_handshaked = step_handshake();
            if (_failed) {
                --_feeding;
                out = drain_records();   // the alert, if any
                if (!out.empty())
                    _lower.SendAsync(out.data(), out.size());
                return false;
            }
        }
        if (_handshaked) {
            uint8_t buf[16384];
            for (;;) {
                const int n = SSL_read(_ssl, buf, int(sizeof buf));
                if (n > 0) {
                    text.insert(text.end(), buf, buf + n);
                    continue;
                }
                const int e = SSL_get_error(_ssl, n);
                if (e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE || e == SSL_ERROR_ZERO_RETURN)
                    break;   // no more whole records / peer's close_notify
                fail("TLS read");
                break;
            }
        }
        out = drain_records();   // handshake replies, session tickets, key updates
        if (!out.empty())
            _lower.SendAsync(out.data(), out.size());
    }
    // what the callbacks send (an echo, the upgrade after the handshake)
    // is held back and encrypted once they return: one SSL_write, full
    // records, instead of one record per frame
    // the held-back bytes go out when the callbacks return, also when one
    // of them throws (the exception then continues to the caller)
    struct Release {
        TLSTransport* t;
        ~Release()
        {
            std::lock_guard<std::recursive_mutex> g(t->_lock);
            if (--t->_feeding == 0 && !t->_out_plain.empty()) {
                std::vector<uint8_t> p, rec;
                p.swap(t->_out_plain);
                t->encrypt(p.data(), p.size(), rec);
                if (!rec.empty())
                    t->_lower.SendAsync(rec.data(), rec.size());
            }
        }
    } release{this};
    if (just_handshaked && handshaked)
        handshaked();
    if (!text.empty() && plain)
        plain(text.data(), text.size());
    return !_failed;
}

size_t TLSTransport::encrypt(const void* buffer, size_t size, std::vector<uint8_t>& records)
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    if (_failed || !_handshaked)
        return 0;
    const uint8_t* p = static_cast<const uint8_t*>(buffer);
    size_t done = 0;
    while (done < size) {
        const int chunk = int(std::min<size_t>(size - done, size_t(1) << 30));
        const int n = SSL_write(_ssl, p + done, chunk);
        if (n <= 0) {
            fail("TLS write");
            break;
        }
        done += size_t(n);
    }
    records = drain_records();
    return done;
}

size_t TLSTransport::encrypt_after_pending(const void* buffer, size_t size, std::vector<uint8_t>& records)
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    if (!_out_plain.empty()) {   // bytes held back by a feed in progress go first
        std::vector<uint8_t> p;
        p.swap(_out_plain);
        if (encrypt(p.data(), p.size(), records) != p.size())
            return 0;
    }
    std::vector<uint8_t> more;
    const size_t n = encrypt(buffer, size, more);
    records.insert(records.end(), more.begin(), more.end());
    return n;
}

// Records go to the lower transport under the session lock: records are
// sequence-numbered, so two threads' records must reach it in the order
// they were encrypted.
size_t TLSTransport::Send(const void* buffer, size_t size)
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    std::vector<uint8_t> rec;
    if (encrypt_after_pending(buffer, size, rec) != size)
        return 0;
    return rec.empty() || _lower.Send(rec.data(), rec.size()) == rec.size() ? size : 0;
}

size_t TLSTransport::Send(const void* buffer, size_t size, const CppCommon::Timespan& timeout)
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    std::vector<uint8_t> rec;
    if (encrypt_after_pending(buffer, size, rec) != size)
        return 0;
    return rec.empty() || _lower.Send(rec.data(), rec.size(), timeout) == rec.size() ? size : 0;
}

bool TLSTransport::SendAsync(const void* buffer, size_t size)
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    if (_failed || !_handshaked)
        return false;
    if (_feeding) {   // inside a feed's callbacks: encrypted when they return
        const uint8_t* p = static_cast<const uint8_t*>(buffer);
        _out_plain.insert(_out_plain.end(), p, p + size);
        return true;
    }
    if (BatchScope::Active()) {   // inside a batch scope (an event-loop tick): encrypted when it ends
        const uint8_t* p = static_cast<const uint8_t*>(buffer);
        _out_plain.insert(_out_plain.end(), p, p + size);
        if (!_scope_held) {
            _scope_held = true;
            BatchScope::AtEnd(this, &TLSTransport::scope_end);
        }
        return true;
    }
    std::vector<uint8_t> rec;
    if (encrypt_after_pending(buffer, size, rec) != size)
        return false;
    return rec.empty() || _lower.SendAsync(rec.data(), rec.size());
}

size_t TLSTransport::Receive(void* buffer, size_t size)
{
    return Receive(buffer, size, CppCommon::Timespan(0));
}

size_t TLSTransport::Receive(void* buffer, size_t size, const CppCommon::Timespan& timeout)
{
    if (size == 0)
        return 0;
    std::vector<uint8_t> in(16384);
    for (int guard = 0; guard < 1 << 20; ++guard) {
        {
            std::lock_guard<std::recursive_mutex> g(_lock);
            if (_pending_at < _pending.size()) {
                const size_t k = std::min(size, _pending.size() - _pending_at);
                std::memcpy(buffer, _pending.data() + _pending_at, k);
                _pending_at += k;
                if (_pending_at == _pending.size()) {
                    _pending.clear();
                    _pending_at = 0;
                }
                return k;
            }
            if (_failed || !_handshaked)
                return 0;
            // bytes held back for a batch scope or a feed in progress go out
            // before we wait for the reply to them (a request sent with
            // SendAsync inside a scope, then a synchronous receive)
            if (!_out_plain.empty()) {
                std::vector<uint8_t> p, rec;
                p.swap(_out_plain);
                encrypt(p.data(), p.size(), rec);
                if (!rec.empty())
                    _lower.SendAsync(rec.data(), rec.size());
            }
        }
        const size_t n = timeout.total() ? _lower.Receive(in.data(), in.size(), timeout)
                                         : _lower.Receive(in.data(), in.size());
        if (n == 0)
            return 0;
        Feed(in.data(), n,
             [this](const void* p, size_t k) {
                 std::lock_guard<std::recursive_mutex> g(_lock);
                 const uint8_t* b = static_cast<const uint8_t*>(p);
                 _pending.insert(_pending.end(), b, b + k);
             },
             nullptr);
    }
    return 0;
}

bool TLSTransport::Disconnect()
{
    {
        std::lock_guard<std::recursive_mutex> g(_lock);
        if (_handshaked && !_failed) {
            SSL_shutdown(_ssl);   // close_notify
            const std::vector<uint8_t> out = drain_records();
            if (!out.empty())
                _lower.Send(out.data(), out.size());
        }
    }
    return _lower.Disconnect();
}

std::string TLSTransport::error() const
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    return _error;
}

std::string TLSTransport::protocol() const
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    return _handshaked ? SSL_get_version(_ssl) : "";
}

std::string TLSTransport::cipher() const
{
    std::lock_guard<std::recursive_mutex> g(_lock);
    return _handshaked ? SSL_CIPHER_get_name(SSL_get_current_cipher(_ssl)) : "";
}

} // namespace WS
} // namespace CppServer
