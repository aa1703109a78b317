// bench_multicast.cpp — the reference's ws_multicast benchmark
// (performance/ws_multicast_server.cpp:104-124, ws_multicast_client.cpp:48-51)
// on this repo's drop-in API over in-memory transports (no sockets: the
// transport is out of scope).
//
// Workload: the server calls MulticastBinary(message) `RATE` times per tick
// (the reference's `messages_rate` loop) to every connected client; clients
// count the bytes they receive (onWSReceived); the metric is the client's:
// messages = total received bytes / message size, throughput = messages /
// time.  Server frames carry key 0 (ws.cpp:206): the XOR is the identity, so
// the frames are built once per call and copied to every session
// (ws_server.cpp:36-64) — no GPU pass, as the reference does no real masking
// there either.  The GPU analogue with a distinct key per client is C4
// (wsg_fanout_encode / _many).
//
// Modes: per_call (each MulticastBinary encodes and queues on its own) and
// tick (one BatchScope around each tick: its multicasts share one encode
// pass, ws_batch.h).  One thread: the multicaster, then the clients' reads.
//
//   bench_multicast MODE CLIENTS RATE SIZE SECONDS
#include "server/ws/ws_batch.h"
#include "driver_options.h"
#include "server/ws/ws_client.h"
#include "server/ws/ws_handshake.h"
#include "server/ws/ws_server.h"
#include "server/ws/ws_session.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <vector>

using namespace CppServer::WS;
using Clock = std::chrono::steady_clock;

namespace {

struct Pipe : Transport {
    Pipe* peer = nullptr;
    std::vector<uint8_t> inbox;
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

struct Client : WSClient {
    using WSClient::WSClient;
    uint64_t total_bytes = 0;
    void onWSConnecting(CppServer::HTTP::HTTPRequest& request) override
    {
        request.SetBegin("GET", "/");
        request.SetHeader("Host", "localhost");
        request.SetHeader("Origin", "http://localhost");
        request.SetHeader("Upgrade", "websocket");
        request.SetHeader("Connection", "Upgrade");
        request.SetHeader("Sec-WebSocket-Key", Base64Encode(ws_nonce()));
        request.SetHeader("Sec-WebSocket-Protocol", "chat, superchat");
        request.SetHeader("Sec-WebSocket-Version", "13");
    }
    void onWSReceived(const void*, size_t size) override { total_bytes += size; }   // ws_multicast_client.cpp:48-51
};

struct Conn {
    Pipe ct, st;
    std::unique_ptr<Client> client;
    std::shared_ptr<WSSession> session;
};

void drain(Pipe& p, std::vector<uint8_t>& buf, WSClient& c)
{
    if (p.inbox.empty())
        return;
    buf.swap(p.inbox);
    p.inbox.clear();
    c.onReceived(buf.data(), buf.size());
    buf.clear();
}

void drain(Pipe& p, std::vector<uint8_t>& buf, WSSession& s)
{
    if (p.inbox.empty())
        return;
    buf.swap(p.inbox);
    p.inbox.clear();
    s.onReceived(buf.data(), buf.size());
    buf.clear();
}

} // namespace

int main(int argc, char** argv)
{
    // positional (bench.py) or the reference's flags (ws_multicast_server -m
    // rate -s size, ws_multicast_client -c clients -z seconds)
    DriverOptions o;
    o.mode = "per_call";
    o.messages = 1000000;   // ws_multicast_server's default rate
    if (argc >= 6 && argv[1][0] != '-') {
        o.mode = argv[1];
        o.clients = std::atoi(argv[2]);
        o.messages = std::atol(argv[3]);
        o.size = std::atol(argv[4]);
        o.seconds = std::atof(argv[5]);
    } else if (!parse_driver_options(argc, argv, o)) {
        std::fprintf(stderr,
                     "usage: %s per_call|tick CLIENTS RATE SIZE SECONDS\n"
                     "   or: %s [--mode per_call|tick] [-c clients] [-m rate] [-s size] [-z seconds]\n",
                     argv[0], argv[0]);
        return 2;
    }
    const std::string mode = o.mode;
    const int clients = std::max(1, o.clients);
    const int rate = int(std::max(1L, o.messages));
    const size_t size = size_t(o.size);
    const double secs = o.seconds;
    const std::vector<uint8_t> message(size, 0);   // ws_multicast_server sends a zero-filled message
    try {
        WSServer server;
        std::vector<std::unique_ptr<Conn>> conns;
        std::vector<uint8_t> buf;
        for (int i = 0; i < clients; ++i) {
            auto c = std::make_unique<Conn>();
            c->ct.peer = &c->st;
            c->st.peer = &c->ct;
            c->client = std::make_unique<Client>(c->ct);
            c->session = std::make_shared<WSSession>(c->st);
            server.AddSession(c->session);
            c->session->Connect();
            c->client->Connect();
            drain(c->st, buf, *c->session);   // upgrade request -> 101
            drain(c->ct, buf, *c->client);
            if (!c->client->IsConnected())
                throw std::runtime_error("upgrade failed");
            conns.push_back(std::move(c));
        }
        const auto t0 = Clock::now();
        double el = 0.0;
        uint64_t ticks = 0;
        while (el < secs) {
            {
                std::unique_ptr<BatchScope> tick;
                if (mode == "tick")
                    tick = std::make_unique<BatchScope>();
                for (int i = 0; i < rate; ++i)
                    server.MulticastBinary(message.data(), message.size());
            }
            for (auto& c : conns)
                drain(c->ct, buf, *c->client);
            ++ticks;
            el = std::chrono::duration<double>(Clock::now() - t0).count();
        }
        uint64_t total = 0;
        for (auto& c : conns)
            total += c->client->total_bytes;
        const uint64_t msgs = size ? total / size : 0;
        const uint64_t expected = ticks * uint64_t(rate) * uint64_t(clients);
        std::printf("{\"mode\": \"%s\", \"clients\": %d, \"rate_per_tick\": %d, \"size\": %zu, \"ticks\": %llu, "
                    "\"seconds\": %.3f, \"total_messages\": %llu, \"msg_per_s\": %.0f, \"MiB_per_s\": %.3f, "
                    "\"latency_ns\": %.1f, \"all_delivered\": %s}\n",
                    mode.c_str(), clients, rate, size, (unsigned long long)ticks, el, (unsigned long long)msgs,
                    msgs / el, total / el / (1 << 20), msgs ? el * 1e9 / double(msgs) : 0.0,
                    msgs == expected ? "true" : "false");
        for (auto& c : conns)
            server.RemoveSession(c->session);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "bench_multicast: %s\n", e.what());
        return 3;
    }
    return 0;
}
