// test_handshake.cpp — the WebSocket upgrade (reference ws.cpp:26-210) and
// its HTTP subset, host only (no frame is sent, so no GPU is needed):
// RFC 6455 / RFC 4648 known answers, request/response round trips, the
// reference's accept/reject rules and error texts, and a full client/session
// upgrade over an in-memory transport.
#include "server/http/http_request.h"
#include "server/http/http_response.h"
#include "server/ws/ws_batch.h"
#include "server/ws/ws_client.h"
#include "server/ws/ws_handshake.h"
#include "server/ws/ws_session.h"
#include "server/ws/wss_client.h"
#include "server/ws/wss_server.h"
#include "server/ws/wss_session.h"

#include "tls_test_certs.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

using namespace CppServer;
using namespace CppServer::WS;

#ifdef WSG_TEST_HEAP_PINNED
// Host-only test (it runs in the CPU suite, no device): the batches' page-locked buffers come from
// wsg_host_alloc (HIP); these definitions take the place of libwsg.so's
// (symbol interposition) with heap memory, which is all a batch needs when
// no GPU pass runs (key-0 frames).
extern "C" int wsg_host_alloc(size_t bytes, void** out)
{
    *out = std::malloc(bytes ? bytes : 1);
    return *out ? WSG_OK : WSG_ENOMEM;
}
extern "C" int wsg_host_free(void* p)
{
    std::free(p);
    return WSG_OK;
}
#endif

static int g_failures = 0, g_checks = 0;
#define CHECK(cond)                                                                    \
    do {                                                                               \
        ++g_checks;                                                                    \
        if (!(cond)) {                                                                 \
            ++g_failures;                                                              \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                              \
    } while (0)

static void test_known_answers()
{
    // RFC 6455 §1.3 worked example
    CHECK(WSAcceptKey("dGhlIHNhbXBsZSBub25jZQ==") == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=");
    // RFC 4648 §10 test vectors
    const char* plain[] = {"", "f", "fo", "foo", "foob", "fooba", "foobar"};
    const char* coded[] = {"", "Zg==", "Zm8=", "Zm9v", "Zm9vYg==", "Zm9vYmE=", "Zm9vYmFy"};
    for (int i = 0; i < 7; ++i) {
        CHECK(Base64Encode(plain[i]) == coded[i]);
        CHECK(Base64Decode(coded[i]) == plain[i]);
    }
    char out[29];
    CHECK(wsg_ws_accept("dGhlIHNhbXBsZSBub25jZQ==", 24, out, sizeof(out)) == WSG_OK);
    CHECK(std::string(out) == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=");
    CHECK(wsg_ws_accept("x", 1, out, 10) == WSG_ENOMEM);
}

static void test_http_round_trip()
{
    HTTP::HTTPRequest rq("GET", "/chat");
    rq.SetHeader("Host", "localhost").SetHeader("Upgrade", "websocket").SetBody("xy");
    CHECK(rq.cache() == "GET /chat HTTP/1.1\r\nHost: localhost\r\nUpgrade: websocket\r\nContent-Length: 2\r\n\r\nxy");
    HTTP::HTTPRequest back;
    const std::string wire = rq.cache() + "trailing";
    CHECK(back.Parse(wire) == rq.cache().size());
    CHECK(!back.error() && back.method() == "GET" && back.url() == "/chat" && back.protocol() == "HTTP/1.1");
    CHECK(back.headers() == 3 && std::get<1>(back.header(1)) == "websocket" && back.body() == "xy");
    CHECK(back.Parse(rq.cache().substr(0, 20)) == 0);   // incomplete
    HTTP::HTTPResponse rs;
    rs.MakeErrorResponse(400, "bad");
    CHECK(rs.cache() == "HTTP/1.1 400 Bad Request\r\nContent-Type: text/plain; charset=UTF-8\r\nContent-Length: 3\r\n\r\nbad");
    HTTP::HTTPResponse rb;
    CHECK(rb.Parse(rs.cache()) == rs.cache().size() && rb.status() == 400 && rb.status_phrase() == "Bad Request");
    CHECK(rb.body() == "bad");
    HTTP::HTTPResponse junk;
    junk.Parse("HTTP/1.1 abc Nope\r\n\r\n");
    CHECK(junk.error());
}

struct Server : WebSocket {
    std::vector<std::string> sent;
    bool connected = false;
    bool veto = false;
    void SendResponse(const HTTP::HTTPResponse& r) override { sent.push_back(r.cache()); }
    bool onWSConnecting(const HTTP::HTTPRequest&, HTTP::HTTPResponse&) override { return !veto; }
    void onWSConnected(const HTTP::HTTPRequest&) override { connected = true; }
    using WebSocket::_ws_handshaked;
};

struct Client : WebSocket {
    std::vector<std::string> errors;
    bool connected = false;
    void onWSError(const std::string& m) override { errors.push_back(m); }
    void onWSConnected(const HTTP::HTTPResponse&) override { connected = true; }
    using WebSocket::_ws_handshaked;
};

static HTTP::HTTPRequest upgrade_request(std::string_view key, std::string_view version = "13",
                                         std::string_view connection = "Upgrade")
{
    HTTP::HTTPRequest r("GET", "/");
    r.SetHeader("Host", "localhost").SetHeader("Upgrade", "websocket").SetHeader("Connection", connection);
    r.SetHeader("Sec-WebSocket-Key", key).SetHeader("Sec-WebSocket-Version", version).SetBody();
    return r;
}

static void test_server_rules()
{
    Client c;
    const std::string key = Base64Encode(c.ws_nonce());
    {
        Server s;
        HTTP::HTTPResponse resp;
        CHECK(s.PerformServerUpgrade(upgrade_request(key), resp));
        CHECK(s.connected && s._ws_handshaked && s.send_key() == 0);   // server key 0 (ws.cpp:206)
        CHECK(s.sent.size() == 1 && resp.status() == 101);
        CHECK(s.sent[0] == "HTTP/1.1 101 Switching Protocols\r\nConnection: Upgrade\r\nUpgrade: websocket\r\n"
                           "Sec-WebSocket-Accept: " + WSAcceptKey(key) + "\r\nContent-Length: 0\r\n\r\n");
        // the client accepts that response (random key, ws.cpp:97)
        HTTP::HTTPResponse back;
        back.Parse(s.sent[0]);
        CHECK(c.PerformClientUpgrade(back) && c.connected && c._ws_handshaked && c.errors.empty());
    }
    {
        Server s;   // "keep-alive, Upgrade" is accepted too (ws.cpp:123)
        HTTP::HTTPResponse resp;
        CHECK(s.PerformServerUpgrade(upgrade_request(key, "13", "keep-alive, Upgrade"), resp));
    }
    {
        Server s;   // wrong version: 400 with the reference's text, sent
        HTTP::HTTPResponse resp;
        CHECK(!s.PerformServerUpgrade(upgrade_request(key, "12"), resp));
        CHECK(resp.status() == 400 && s.sent.size() == 1 && !s._ws_handshaked);
        CHECK(resp.body() == "Invalid WebSocket handshaked request: 'Sec-WebSocket-Version' header value must be '13'");
    }
    {
        Server s;   // not an upgrade at all: left alone, nothing sent
        HTTP::HTTPRequest plain("GET", "/index.html");
        plain.SetHeader("Host", "x").SetBody();
        HTTP::HTTPResponse resp;
        CHECK(!s.PerformServerUpgrade(plain, resp) && s.sent.empty());
        HTTP::HTTPRequest post("POST", "/");
        post.SetBody();
        CHECK(!s.PerformServerUpgrade(post, resp) && s.sent.empty());
    }
    {
        Server s;   // onWSConnecting veto: no response, not handshaked
        s.veto = true;
        HTTP::HTTPResponse resp;
        CHECK(!s.PerformServerUpgrade(upgrade_request(key), resp) && s.sent.empty() && !s._ws_handshaked);
    }
}

static void test_client_rules()
{
    Client c;
    HTTP::HTTPResponse r(101);
    r.SetHeader("Connection", "Upgrade").SetHeader("Upgrade", "websocket");
    r.SetHeader("Sec-WebSocket-Accept", WSAcceptKey("some other key")).SetBody();
    CHECK(!c.PerformClientUpgrade(r) && !c._ws_handshaked);
    CHECK(c.errors.size() == 1 &&
          c.errors[0] == "Invalid WebSocket handshaked response: 'Sec-WebSocket-Accept' value validation failed");
    HTTP::HTTPResponse missing(101);
    missing.SetHeader("Connection", "Upgrade").SetBody();
    CHECK(!c.PerformClientUpgrade(missing) && c.errors.back() == "Invalid WebSocket response");
    HTTP::HTTPResponse not101(200);
    not101.SetBody();
    const size_t errs = c.errors.size();
    CHECK(!c.PerformClientUpgrade(not101) && c.errors.size() == errs);   // silently not an upgrade
}

// in-memory transport pair (the WSS tests read the inboxes directly)
struct Loop : Transport {
    Loop* peer = nullptr;
    std::deque<uint8_t> inbox;
    size_t Send(const void* b, size_t n) override
    {
        const uint8_t* p = static_cast<const uint8_t*>(b);
        peer->inbox.insert(peer->inbox.end(), p, p + n);
        return n;
    }
    bool SendAsync(const void* b, size_t n) override { return Send(b, n) == n; }
    size_t Receive(void*, size_t) override { return 0; }
    bool Disconnect() override { return true; }
    bool IsConnected() const override { return true; }
};

struct MyClient : WSClient {
    using WSClient::WSClient;
    bool up = false;
    void onWSConnecting(HTTP::HTTPRequest& request) override
    {
        request.SetBegin("GET", "/");
        request.SetHeader("Host", "localhost");
        request.SetHeader("Upgrade", "websocket");
        request.SetHeader("Connection", "Upgrade");
        request.SetHeader("Sec-WebSocket-Key", Base64Encode(ws_nonce()));
        request.SetHeader("Sec-WebSocket-Version", "13");
    }
    void onWSConnected(const HTTP::HTTPResponse&) override { up = true; }
};

struct MySession : WSSession {
    using WSSession::WSSession;
    bool up = false;
    void onWSConnected(const HTTP::HTTPRequest&) override { up = true; }
};

static void test_client_session_upgrade()
{
    Loop a, b;
    a.peer = &b;
    b.peer = &a;
    MyClient client(a);
    MySession session(b);
    CHECK(session.Connect() && !session.IsConnected());
    CHECK(client.Connect() && !client.IsConnected());
    // deliver the request to the session one byte at a time, the response whole
    std::vector<uint8_t> req(b.inbox.begin(), b.inbox.end());
    b.inbox.clear();
    for (uint8_t byte : req)
        session.onReceived(&byte, 1);
    CHECK(session.up && session.IsConnected());
    std::vector<uint8_t> resp(a.inbox.begin(), a.inbox.end());
    a.inbox.clear();
    client.onReceived(resp.data(), resp.size());
    CHECK(client.up && client.IsConnected());
}

// WSS (reference include/server/ws/wss_*.h): the upgrade over a real TLS
// session (OpenSSL, TLS 1.3, the client verifying the server's certificate
// against a run-time CA), records pumped between the two byte transports.
// No frame is sent, so no GPU is needed.
struct MyWssClient : WSSClient {
    using WSSClient::WSSClient;
    bool up = false, tls_up = false;
    std::string err;
    void onWSConnecting(HTTP::HTTPRequest& request) override
    {
        request.SetBegin("GET", "/");
        request.SetHeader("Host", "localhost");
        request.SetHeader("Upgrade", "websocket");
        request.SetHeader("Connection", "Upgrade");
        request.SetHeader("Sec-WebSocket-Key", Base64Encode(ws_nonce()));
        request.SetHeader("Sec-WebSocket-Version", "13");
    }
    void onWSConnected(const HTTP::HTTPResponse&) override { up = true; }
    void onWSError(const std::string& message) override { err = message; }
    void use_send_key(uint32_t key) { set_send_key(key); }
    void onHandshaked() override
    {
        tls_up = true;
        WSSClient::onHandshaked();
    }
};

struct MyWssSession : WSSSession {
    using WSSSession::WSSSession;
    bool up = false;
    std::string err;
    void onWSConnected(const HTTP::HTTPRequest&) override { up = true; }
    void onWSError(const std::string& message) override { err = message; }
};

template <class C, class S>
static void pump(Loop& a, Loop& b, C& client, S& session, bool tamper_once = false)
{
    for (int guard = 0; guard < 64 && (!a.inbox.empty() || !b.inbox.empty()); ++guard) {
        if (!b.inbox.empty()) {
            std::vector<uint8_t> rec(b.inbox.begin(), b.inbox.end());
            b.inbox.clear();
            if (tamper_once && rec.size() > 40) {
                rec[rec.size() - 20] ^= 0x01;   // one flipped bit in an application record
                tamper_once = false;
            }
            session.onReceived(rec.data(), rec.size());
        }
        if (!a.inbox.empty()) {
            std::vector<uint8_t> rec(a.inbox.begin(), a.inbox.end());
            a.inbox.clear();
            client.onReceived(rec.data(), rec.size());
        }
    }
}

static void test_wss_upgrade()
{
    using CppServer::Asio::SSLContext;
    const TestPki pki = make_test_pki();
    // server: the reference's wss_chat_server configuration calls (examples/wss_chat_server.cpp:98-102)
    auto server_ctx = std::make_shared<SSLContext>(asio::ssl::context::tlsv13);
    server_ctx->set_password_callback([](size_t, asio::ssl::context::password_purpose) -> std::string { return "qwerty"; });
    server_ctx->use_certificate_chain(pki.server_cert_pem.data(), pki.server_cert_pem.size());
    server_ctx->use_private_key(pki.server_key_pem.data(), pki.server_key_pem.size(), asio::ssl::context::pem);
    // client: wss_chat_client's (examples/wss_chat_client.cpp:105-109), the CA from memory
    auto client_ctx = std::make_shared<SSLContext>(asio::ssl::context::tlsv13);
    client_ctx->set_verify_mode(asio::ssl::verify_peer | asio::ssl::verify_fail_if_no_peer_cert);
    client_ctx->add_certificate_authority(pki.ca_pem.data(), pki.ca_pem.size());

    {
        Loop a, b;
        a.peer = &b;
        b.peer = &a;
        WSSServer server(server_ctx);
        MyWssClient client(client_ctx, a);
        auto session = std::make_shared<MyWssSession>(server.context(), b);
        server.AddSession(session);
        CHECK(session->Connect());
        CHECK(client.Connect());
        CHECK(!b.inbox.empty());   // the ClientHello
        pump(a, b, client, *session);
        CHECK(client.tls_up && client.IsHandshaked() && session->IsHandshaked());
        CHECK(client.tls().protocol() == "TLSv1.3");
        CHECK(session->up && session->IsConnected());
        CHECK(client.up && client.IsConnected());
        CHECK(client.err.empty() && session->err.empty());
        // the upgrade bytes crossed as TLS records: no cleartext HTTP on the wire
        server.RemoveSession(session);
    }
    {
        // a client that does not trust the server's CA fails the handshake
        Loop a, b;
        a.peer = &b;
        b.peer = &a;
        auto strict = std::make_shared<SSLContext>(asio::ssl::context::tlsv13);
        strict->set_verify_mode(asio::ssl::verify_peer | asio::ssl::verify_fail_if_no_peer_cert);
        MyWssClient client(strict, a);
        MyWssSession session(server_ctx, b);
        CHECK(session.Connect());
        CHECK(client.Connect());
        pump(a, b, client, session);
        CHECK(!client.IsHandshaked() && !client.up && !client.err.empty());
        CHECK(client.err.find("certificate verify failed") != std::string::npos);
    }
    {
        // a tampered record is rejected (AEAD), not delivered
        Loop a, b;
        a.peer = &b;
        b.peer = &a;
        MyWssClient client(client_ctx, a);
        MyWssSession session(server_ctx, b);
        CHECK(session.Connect());
        CHECK(client.ConnectAsync());
        // handshake records untouched; the upgrade request (first application
        // record to the session) gets one bit flipped
        for (int guard = 0; guard < 64 && !client.IsHandshaked(); ++guard) {
            std::vector<uint8_t> rb(b.inbox.begin(), b.inbox.end()), ra(a.inbox.begin(), a.inbox.end());
            b.inbox.clear();
            a.inbox.clear();
            if (!rb.empty())
                session.onReceived(rb.data(), rb.size());
            if (!ra.empty())
                client.onReceived(ra.data(), ra.size());
        }
        CHECK(client.IsHandshaked());
        pump(a, b, client, session, true);
        CHECK(!session.up && !session.err.empty());
    }
    {
        // records cut at random points (partial records, several per read):
        // the TLS handshake and the upgrade complete
        Loop a, b;
        a.peer = &b;
        b.peer = &a;
        MyWssClient client(client_ctx, a);
        MyWssSession session(server_ctx, b);
        CHECK(session.Connect());
        CHECK(client.Connect());
        uint64_t rng = 12345;
        auto next = [&rng]() {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        auto dribble = [&](Loop& from, auto& to) {
            std::vector<uint8_t> rec(from.inbox.begin(), from.inbox.end());
            from.inbox.clear();
            for (size_t at = 0; at < rec.size();) {
                const size_t n = std::min<size_t>(rec.size() - at, 1 + next() % 700);
                to.onReceived(rec.data() + at, n);
                at += n;
            }
        };
        for (int guard = 0; guard < 64 && (!a.inbox.empty() || !b.inbox.empty()); ++guard) {
            dribble(b, session);
            dribble(a, client);
        }
        CHECK(client.up && session.up && client.err.empty() && session.err.empty());
        // (frames through TLS under random splits: test_ws_api.cpp, GPU)
    }
    {
        // configuration errors surface as exceptions with OpenSSL's text
        auto ctx = std::make_shared<SSLContext>(asio::ssl::context::tlsv12);
        bool threw = false;
        try {
            ctx->use_certificate_chain_file("/nonexistent/server.pem");
        } catch (const std::exception& e) {
            threw = std::string(e.what()).find("use_certificate_chain_file") != std::string::npos;
        }
        CHECK(threw);
    }
}

// a WSS client that queues a request with SendTextAsync inside a
// BatchScope and then waits in a synchronous ReceiveText: the TLS layer held
// the request's records until the scope ends, and the receive waited for a
// reply to bytes never sent.  The server runs on its own thread here (a
// socket peer); records travel through locked inboxes.
struct ThreadLoop : Transport {
    ThreadLoop* peer = nullptr;
    std::mutex m;
    std::condition_variable cv;
    std::deque<uint8_t> inbox;
    size_t Send(const void* b, size_t n) override
    {
        const uint8_t* p = static_cast<const uint8_t*>(b);
        {
            std::lock_guard<std::mutex> g(peer->m);
            peer->inbox.insert(peer->inbox.end(), p, p + n);
        }
        peer->cv.notify_all();
        return n;
    }
    bool SendAsync(const void* b, size_t n) override { return Send(b, n) == n; }
    // what arrived within 2 s (0: nothing came)
    size_t Receive(void* buf, size_t n) override
    {
        std::unique_lock<std::mutex> g(m);
        cv.wait_for(g, std::chrono::seconds(2), [&] { return !inbox.empty(); });
        const size_t k = std::min(n, inbox.size());
        std::copy_n(inbox.begin(), k, static_cast<uint8_t*>(buf));
        inbox.erase(inbox.begin(), inbox.begin() + std::ptrdiff_t(k));
        return k;
    }
    std::vector<uint8_t> take()
    {
        std::lock_guard<std::mutex> g(m);
        std::vector<uint8_t> v(inbox.begin(), inbox.end());
        inbox.clear();
        return v;
    }
    bool Disconnect() override { return true; }
    bool IsConnected() const override { return true; }
};

struct EchoWssSession : MyWssSession {
    using MyWssSession::MyWssSession;
    void onWSReceived(const void* buffer, size_t size) override { SendTextAsync(buffer, size); }
};

static void test_wss_sync_receive_in_scope()
{
    using CppServer::Asio::SSLContext;
    const TestPki pki = make_test_pki();
    auto server_ctx = std::make_shared<SSLContext>(asio::ssl::context::tlsv13);
    server_ctx->use_certificate_chain(pki.server_cert_pem.data(), pki.server_cert_pem.size());
    server_ctx->use_private_key(pki.server_key_pem.data(), pki.server_key_pem.size(), asio::ssl::context::pem);
    auto client_ctx = std::make_shared<SSLContext>(asio::ssl::context::tlsv13);
    client_ctx->set_verify_mode(asio::ssl::verify_peer | asio::ssl::verify_fail_if_no_peer_cert);
    client_ctx->add_certificate_authority(pki.ca_pem.data(), pki.ca_pem.size());

    ThreadLoop a, b;
    a.peer = &b;
    b.peer = &a;
    MyWssClient client(client_ctx, a);
    EchoWssSession session(server_ctx, b);
    CHECK(session.Connect());
    CHECK(client.Connect());
    // the TLS handshake and the upgrade, pumped on this thread
    for (int guard = 0; guard < 64 && !(client.up && session.up); ++guard) {
        const std::vector<uint8_t> rb = b.take(), ra = a.take();
        if (!rb.empty())
            session.onReceived(rb.data(), rb.size());
        if (!ra.empty())
            client.onReceived(ra.data(), ra.size());
    }
    CHECK(client.up && session.up);
    // key 0 on the client: the frames stay masked-format, with nothing to
    // XOR, so no GPU pass runs on either side (this is the CPU suite)
    client.use_send_key(0);
    std::atomic<bool> stop{false};
    std::thread server([&] {
        while (!stop.load()) {
            std::vector<uint8_t> rec;
            {
                std::unique_lock<std::mutex> g(b.m);
                b.cv.wait_for(g, std::chrono::milliseconds(20), [&] { return !b.inbox.empty(); });
                rec.assign(b.inbox.begin(), b.inbox.end());
                b.inbox.clear();
            }
            if (!rec.empty())
                session.onReceived(rec.data(), rec.size());
        }
    });
    std::string got, error;
    try {
        BatchScope scope;   // an event-loop tick on the client's thread
        CHECK(client.SendTextAsync("ping"));
        got = client.ReceiveText();
    } catch (const std::exception& e) {
        error = e.what();
    }
    stop = true;
    server.join();
    if (!error.empty())
        std::fprintf(stderr, "test_wss_sync_receive_in_scope: %s\n", error.c_str());
    CHECK(error.empty());
    CHECK(got == "ping");
}

int main()
{
    try {
        test_known_answers();
        test_http_round_trip();
        test_server_rules();
        test_client_rules();
        test_client_session_upgrade();
        test_wss_upgrade();
        test_wss_sync_receive_in_scope();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 2;
    }
    std::printf("%d checks, %d failures\n", g_checks, g_failures);
    return g_failures == 0 ? 0 : 1;
}
