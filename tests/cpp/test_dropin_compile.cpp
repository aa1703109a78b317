// test_dropin_compile.cpp — compile-only check (g++ -fsyntax-only, no GPU):
// code written against the reference's WebSocket API compiles unchanged
// against this repo's headers.  Every call below uses a signature of the
// reference (include/server/ws/ws.h:62, ws_client.h:39-96, ws_session.h:40-89,
// ws_server.h:41-59), including the CppCommon::Timespan timeout overloads,
// PerformClientUpgrade(response, UUID) and ConnectAsync.  The classes sit on
// this repo's Transport instead of the reference's Asio sockets, so their
// constructors differ; everything called on them is the reference's.
#include "server/ws/ws_client.h"
#include "server/ws/ws_server.h"
#include "server/ws/ws_session.h"
#include "server/ws/wss_client.h"
#include "server/ws/wss_server.h"
#include "server/ws/wss_session.h"

#include <memory>
#include <string>
#include <vector>

using namespace CppServer::WS;

namespace {

// the reference's ws_chat_client / ws_echo_client style subclass
class ChatClient : public WSClient
{
public:
    using WSClient::WSClient;

    void onWSConnecting(CppServer::HTTP::HTTPRequest& request) override
    {
        request.SetBegin("GET", "/");
        request.SetHeader("Upgrade", "websocket");
        request.SetHeader("Connection", "Upgrade");
        request.SetHeader("Sec-WebSocket-Version", "13");
    }
    void onWSConnected(const CppServer::HTTP::HTTPResponse& response) override { SendTextAsync("hello"); }
    void onWSReceived(const void* buffer, size_t size) override { SendBinaryAsync(buffer, size); }
    void onWSPing(const void* buffer, size_t size) override { SendPongAsync(buffer, size); }

    // the upgrade with the connection id, as ws_client.cpp:96 calls it
    bool Upgrade(const CppServer::HTTP::HTTPResponse& response)
    {
        return PerformClientUpgrade(response, CppCommon::UUID::Random());
    }
};

class ChatSession : public WSSession
{
public:
    using WSSession::WSSession;
    void onWSReceived(const void* buffer, size_t size) override { SendTextAsync(buffer, size); }
};

[[maybe_unused]] void use_client(ChatClient& c)
{
    const CppCommon::Timespan t = CppCommon::Timespan::seconds(1);
    size_t n = 0;
    n += c.SendText("a");
    n += c.SendText("a", t);
    n += c.SendText("a", 1, t);
    n += c.SendBinary("b", 1);
    n += c.SendBinary("b", 1, t);
    n += c.SendBinary(std::string_view("b"), t);
    n += c.SendClose(1000, "bye");
    n += c.SendClose(1000, "bye", 3, t);
    n += c.SendClose(1000, std::string_view("bye"), t);
    n += c.SendPing("p", t);
    n += c.SendPong("p", 1, t);
    bool ok = c.SendTextAsync("x") && c.SendBinaryAsync("y", 1) && c.SendCloseAsync(1000, "z") &&
              c.SendPingAsync("p") && c.SendPongAsync("q", 1);
    std::string text = c.ReceiveText();
    text += c.ReceiveText(t);
    std::vector<uint8_t> bin = c.ReceiveBinary();
    bin = c.ReceiveBinary(CppCommon::Timespan::milliseconds(100));
    ok = ok && c.Connect() && c.ConnectAsync();
    ok = ok && c.Close() && c.Close(1000) && c.Close(1000, "bye") && c.CloseAsync(1001);
    (void)n;
    (void)ok;
}

[[maybe_unused]] void use_session(ChatSession& s)
{
    const CppCommon::Timespan t(500000000);
    size_t n = s.SendText("a", t) + s.SendBinary("b", 1, t) + s.SendClose(1000, "bye", t) + s.SendPing("p", t) +
               s.SendPong("p", t);
    std::string text = s.ReceiveText(t);
    std::vector<uint8_t> bin = s.ReceiveBinary(t);
    (void)n;
    (void)text;
    (void)bin;
}

[[maybe_unused]] void use_server(WSServer& server, const std::shared_ptr<WSSession>& session)
{
    server.AddSession(session);
    size_t n = server.MulticastText("all") + server.MulticastBinary("bin", 3) + server.MulticastPing("p");
    bool ok = server.Multicast("raw", 3) && server.CloseAll(1000, "bye");
    server.RemoveSession(session);
    (void)n;
    (void)ok;
}

[[maybe_unused]] void use_wss(WSSClient& c, WSSServer& s) { (void)c.SendTextAsync("tls"); (void)s.MulticastText("tls"); }

// Connect / ConnectAsync with a resolver, as ws_chat_client.cpp calls them
struct TCPResolver {};
[[maybe_unused]] void use_resolver(ChatClient& c, const std::shared_ptr<TCPResolver>& resolver)
{
    (void)c.Connect(resolver);
    (void)c.ConnectAsync(resolver);
}

// the reference's SSL context set-up, verbatim in form
// (examples/wss_chat_server.cpp:98-102, examples/wss_chat_client.cpp:105-109)
[[maybe_unused]] std::shared_ptr<CppServer::Asio::SSLContext> server_context()
{
    auto context = std::make_shared<CppServer::Asio::SSLContext>(asio::ssl::context::tlsv13);
    context->set_password_callback([](size_t max_length, asio::ssl::context::password_purpose purpose) -> std::string { return "qwerty"; });
    context->use_certificate_chain_file("../tools/certificates/server.pem");
    context->use_private_key_file("../tools/certificates/server.pem", asio::ssl::context::pem);
    context->use_tmp_dh_file("../tools/certificates/dh4096.pem");
    return context;
}

[[maybe_unused]] std::shared_ptr<CppServer::Asio::SSLContext> client_context()
{
    auto context = std::make_shared<CppServer::Asio::SSLContext>(asio::ssl::context::tlsv13);
    context->set_default_verify_paths();
    context->set_root_certs();
    context->set_verify_mode(asio::ssl::verify_peer | asio::ssl::verify_fail_if_no_peer_cert);
    context->load_verify_file("../tools/certificates/ca.pem");
    return context;
}

} // namespace
