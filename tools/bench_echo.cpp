// bench_echo.cpp — BASELINE config C1 (the reference's ws_echo benchmark) on
// this repo's drop-in API, over in-memory transports (no sockets: the
// transport is out of scope).
//
// Workload of performance/ws_echo_client.cpp / ws_echo_server.cpp:
//   * every client sends `-m` messages of `-s` zero bytes when its upgrade
//     completes (onWSConnected, ws_echo_client.cpp:57-61) and one more for
//     every message it gets back (onWSReceived, :63-73);
//   * the server session echoes what it receives with SendBinaryAsync
//     (ws_echo_server.cpp:23-27);
//   * the metric is the client's (ws_echo_client.cpp:191-201): messages =
//     total received bytes / message size, throughput = messages / time.
// Client frames are masked with the connection's random key (GPU mask on
// send, GPU unmask on the server's receive); server frames are unmasked with
// key 0 (the identity both ways, as in the reference).
//
// The "IO threads" poll their connections: each one with bytes pending gets
// them all in one onReceived call (one socket read).  Modes:
//   per_read  the drop-in default: every onReceived is a batch scope (its
//             frames unmasked in one GPU pass, the sends they trigger
//             encoded in one more) — user code unchanged;
//   tick      one BatchScope around each poll pass over all the thread's
//             connections (an event loop that batches its tick);
//   per_call  automatic batching off ($WSG_AUTO_BATCH=0 semantics): one GPU
//             round trip per masked frame, the round-1 path.
//
//   bench_echo MODE CLIENTS THREADS MESSAGES SIZE SECONDS [tls]
// `tls`: the reference's wss_echo (performance/wss_echo_client.cpp /
// wss_echo_server.cpp): WSSClient / WSSSession over TLS 1.3 (OpenSSL,
// certificates made at start-up), the same echo loop.
// Prints one JSON object.  Links the product library only.
#include "server/ws/ws_batch.h"
#include "server/ws/ws_client.h"
#include "server/ws/ws_handshake.h"
#include "server/ws/ws_session.h"
#include "server/ws/wss_client.h"
#include "server/ws/wss_session.h"

#include "../tests/cpp/tls_test_certs.h"
#include "driver_options.h"

#include <functional>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

using namespace CppServer::WS;
using Clock = std::chrono::steady_clock;

#ifdef ECHO_HOSTONLY
// no device needed: the batches' page-locked buffers from the heap (the
// executable's definitions take the place of libwsg.so's)
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

namespace {

// The thread's codec context and the GPU code up before the clock starts, as
// a server has them from its first connections on: one small masked frame
// through the host decode entry point (context creation, code object load,
// the host lane's first launch: ~0.1-0.2 s once per thread, which a 3-second
// run would otherwise count).
void warm_codec()
{
#ifndef ECHO_HOSTONLY
    wsg_ctx* c = ThreadCodec();
    void* p = nullptr;
    if (!c || wsg_host_alloc(64, &p) != WSG_OK)
        return;
    uint8_t* w = static_cast<uint8_t*>(p);
    const uint8_t frame[] = {0x82, 0x84, 1, 2, 3, 4, 'a' ^ 1, 'b' ^ 2, 'c' ^ 3, 'd' ^ 4};
    std::memcpy(w, frame, sizeof(frame));
    uint64_t fs = 0;
    wsg_recv_info info;
    (void)wsg_decode_batch_host(c, w, sizeof(frame), &fs, 1, w + 32, &info);
    wsg_host_free(p);
#endif
}

struct Pipe : Transport {
    Pipe* peer = nullptr;
    std::vector<uint8_t> inbox;   // bytes the peer sent, not yet read
    bool connected = true;
    size_t Send(const void* b, size_t n) override
    {
        if (!connected || !peer)
            return 0;
        const uint8_t* p = static_cast<const uint8_t*>(b);
        peer->inbox.insert(peer->inbox.end(), p, p + n);
        return n;
    }
    bool SendAsync(const void* b, size_t n) override { return Send(b, n) == n; }
    size_t Receive(void*, size_t) override { return 0; }
    bool Disconnect() override
    {
        connected = false;
        return true;
    }
    bool IsConnected() const override { return connected; }
};

std::vector<uint8_t> g_message;
std::atomic<bool> g_stop{false};

template <class Base>
struct EchoSession : Base {
    using Base::Base;
    void onWSReceived(const void* buffer, size_t size) override { this->SendBinaryAsync(buffer, size); }
};

template <class Base>
struct EchoClient : Base {
    template <class... A>
    explicit EchoClient(size_t messages, A&&... a) : Base(std::forward<A>(a)...), _messages(messages)
    {
    }
    uint64_t total_bytes = 0;
    uint64_t bad = 0;
    void SendMessage() { this->SendBinaryAsync(g_message.data(), g_message.size()); }
    void onWSConnecting(CppServer::HTTP::HTTPRequest& request) override
    {
        request.SetBegin("GET", "/");
        request.SetHeader("Host", "localhost");
        request.SetHeader("Origin", "http://localhost");
        request.SetHeader("Upgrade", "websocket");
        request.SetHeader("Connection", "Upgrade");
        request.SetHeader("Sec-WebSocket-Key", Base64Encode(this->ws_nonce()));
        request.SetHeader("Sec-WebSocket-Protocol", "chat, superchat");
        request.SetHeader("Sec-WebSocket-Version", "13");
    }
    void onWSConnected(const CppServer::HTTP::HTTPResponse&) override
    {
#ifdef ECHO_HOSTONLY
        // measurement build (tools/_build/echo_hostonly): the client key set
        // to 0, so no frame has bytes to XOR and no GPU pass runs; what is
        // left is the API's host work (framing, delivery, queueing)
        this->set_send_key(0);
#endif
        for (size_t i = _messages; i > 0; --i)
            SendMessage();
    }
    void onWSReceived(const void* buffer, size_t size) override
    {
        // the echo of zero bytes must come back as zero bytes (checks the
        // mask -> unmask round trip on every message)
        const uint8_t* b = static_cast<const uint8_t*>(buffer);
        for (size_t i = 0; i < size; ++i)
            bad += b[i] != 0;
        _received += size;
        while (_received >= g_message.size()) {
            if (!g_stop.load(std::memory_order_relaxed))
                SendMessage();
            _received -= g_message.size();
        }
        total_bytes += size;
    }

private:
    size_t _received = 0;
    size_t _messages;
};

// one connection: WS or WSS endpoints behind the same calls (onReceived is
// the TLS record path on the WSS classes, so it is bound to the concrete type)
struct Conn {
    Pipe ct, st;
    std::shared_ptr<void> client, session;
    std::function<void(const void*, size_t)> client_rx, session_rx;
    std::function<void()> connect;
    std::function<uint64_t()> total_bytes, bad;
};

template <class C, class S>
void bind(Conn& cn, std::shared_ptr<C> c, std::shared_ptr<S> s)
{
    cn.client_rx = [c](const void* b, size_t n) { c->onReceived(b, n); };
    cn.session_rx = [s](const void* b, size_t n) { s->onReceived(b, n); };
    cn.connect = [c] { c->Connect(); };
    cn.total_bytes = [c] { return c->total_bytes; };
    cn.bad = [c] { return c->bad; };
    s->Connect();
    cn.client = c;
    cn.session = s;
}

double seconds(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// read everything pending on `p` into `buf` and hand it to `fn` (one read)
template <class F>
bool read_all(Pipe& p, std::vector<uint8_t>& buf, F fn)
{
    if (p.inbox.empty())
        return false;
    buf.swap(p.inbox);
    p.inbox.clear();
    fn(buf.data(), buf.size());
    buf.clear();
    return true;
}

} // namespace

int main(int argc, char** argv)
{
    // positional (bench.py) or the reference's flags (ws_echo_client -c -t -m -s -z)
    DriverOptions o;
    o.mode = "per_read";
    if (argc >= 7 && argv[1][0] != '-') {
        o.mode = argv[1];
        o.clients = std::atoi(argv[2]);
        o.threads = std::max(1, std::atoi(argv[3]));
        o.messages = std::atol(argv[4]);
        o.size = std::atol(argv[5]);
        o.seconds = std::atof(argv[6]);
        o.tls = argc > 7 && std::string(argv[7]) == "tls";
    } else if (!parse_driver_options(argc, argv, o)) {
        std::fprintf(stderr,
                     "usage: %s per_read|tick|per_call CLIENTS THREADS MESSAGES SIZE SECONDS [tls]\n"
                     "   or: %s [--mode per_read|tick|per_call] [-c clients] [-t threads] [-m messages] [-s size] "
                     "[-z seconds] [--tls]\n",
                     argv[0], argv[0]);
        return 2;
    }
    const std::string mode = o.mode;
    const bool tls = o.tls;
    std::shared_ptr<CppServer::Asio::SSLContext> cctx, sctx;
    if (tls) {
        using CppServer::Asio::SSLContext;
        const TestPki pki = make_test_pki();
        sctx = std::make_shared<SSLContext>(SSLContext::tlsv13);
        sctx->use_certificate_chain(pki.server_cert_pem.data(), pki.server_cert_pem.size());
        sctx->use_private_key(pki.server_key_pem.data(), pki.server_key_pem.size(), SSLContext::pem);
        cctx = std::make_shared<SSLContext>(SSLContext::tlsv13);
        cctx->set_verify_mode(CppServer::Asio::verify_peer | CppServer::Asio::verify_fail_if_no_peer_cert);
        cctx->add_certificate_authority(pki.ca_pem.data(), pki.ca_pem.size());
    }
    const int clients = o.clients, threads = std::max(1, o.threads);
    const size_t messages = size_t(o.messages), size = size_t(o.size);
    const double secs = o.seconds;
    g_message.assign(size, 0);   // ws_echo_client sends zero bytes

    std::vector<std::unique_ptr<Conn>> conns(size_t(std::max(clients, 1)));
    std::vector<uint64_t> bytes(size_t(threads), 0), bad(size_t(threads), 0);
    std::vector<double> elapsed(size_t(threads), 0.0);
    std::vector<std::string> errors(static_cast<size_t>(threads));
    std::atomic<int> ready{0};
    const auto t_start = Clock::now();

    auto worker = [&](int t) {
        try {
            BatchScope::SetEnabled(mode != "per_call");
            // this thread's connections: upgrade them (the handshake runs
            // through onReceived like any read)
            std::vector<Conn*> mine;
            for (int c = t; c < clients; c += threads) {
                auto cn = std::make_unique<Conn>();
                cn->ct.peer = &cn->st;
                cn->st.peer = &cn->ct;
                if (tls)
                    bind(*cn, std::make_shared<EchoClient<WSSClient>>(messages, cctx, cn->ct),
                         std::make_shared<EchoSession<WSSSession>>(sctx, cn->st));
                else
                    bind(*cn, std::make_shared<EchoClient<WSClient>>(messages, cn->ct),
                         std::make_shared<EchoSession<WSSession>>(cn->st));
                mine.push_back(cn.get());
                conns[size_t(c)] = std::move(cn);
            }
            warm_codec();
            ready.fetch_add(1);
            while (ready.load() < threads)
                std::this_thread::yield();
            const auto t0 = Clock::now();
            for (Conn* c : mine)
                c->connect();
            std::vector<uint8_t> buf;
            uint64_t polls = 0;
            for (;;) {
                bool any = false;
                {
                    // tick mode: every connection's reads of this pass share
                    // one receive pass and one send pass on the GPU
                    std::unique_ptr<BatchScope> tick;
                    if (mode == "tick")
                        tick = std::make_unique<BatchScope>();
                    for (Conn* c : mine) {
                        any |= read_all(c->st, buf, c->session_rx);
                        any |= read_all(c->ct, buf, c->client_rx);
                    }
                }
                ++polls;
                if ((polls & 15) == 0 && seconds(t0, Clock::now()) >= secs)
                    g_stop.store(true, std::memory_order_relaxed);
                if (!any)
                    break;   // every echo drained after the stop
            }
            elapsed[size_t(t)] = seconds(t0, Clock::now());
            for (Conn* c : mine) {
                bytes[size_t(t)] += c->total_bytes();
                bad[size_t(t)] += c->bad();
            }
        } catch (const std::exception& e) {
            errors[size_t(t)] = e.what();
            ready.fetch_add(1);
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back(worker, t);
    for (auto& th : pool)
        th.join();
    (void)t_start;
    uint64_t total = 0, total_bad = 0;
    double el = 0.0;
    for (int t = 0; t < threads; ++t) {
        if (!errors[size_t(t)].empty()) {
            std::fprintf(stderr, "bench_echo: thread %d: %s\n", t, errors[size_t(t)].c_str());
            return 3;
        }
        total += bytes[size_t(t)];
        total_bad += bad[size_t(t)];
        el = std::max(el, elapsed[size_t(t)]);
    }
    const uint64_t msgs = size ? total / size : 0;
    std::printf("{\"mode\": \"%s\", \"tls\": %s, \"clients\": %d, \"threads\": %d, \"messages_in_flight\": %zu, \"size\": %zu, "
                "\"seconds\": %.3f, \"total_messages\": %llu, \"msg_per_s\": %.0f, \"MiB_per_s\": %.3f, "
                "\"latency_ns\": %.1f, \"payload_ok\": %s}\n",
                mode.c_str(), tls ? "true" : "false", clients, threads, messages, size, el, (unsigned long long)msgs, msgs / el,
                total / el / (1 << 20), msgs ? el * 1e9 / double(msgs) : 0.0, total_bad == 0 ? "true" : "false");
    return 0;
}
