// bench_echo_ref.cpp — BASELINE config C1's CPU reference leg: the echo loop
// of tools/bench_echo.cpp (in-memory transports, polling IO threads, the
// ws_echo_client.cpp:191-201 metric) with both endpoints running the
// reference's codec algorithm on the CPU: the oracle's restatement of
// PrepareSendFrame / PrepareReceiveFrame (source/server/ws/ws.cpp:212-456,
// byte-at-a-time, std::vector buffers), one call per send and per read, the
// onWS* callbacks by borrowed pointer.  No GPU.  Measurement tool: links the
// oracle (test infrastructure), never the product library.
//
// Workload (performance/ws_echo_client.cpp / ws_echo_server.cpp): every
// client sends `-m` messages of `-s` zero bytes at start (onWSConnected,
// :57-61; the upgrade handshake is not part of this loop) and one more per
// message echoed back (:63-73); the server echoes with SendBinaryAsync
// (ws_echo_server.cpp:23-27): mask=false, key 0.  Client key: rand() per
// connection (ws.cpp:97).
//
//   bench_echo_ref CLIENTS THREADS MESSAGES SIZE SECONDS
// Prints one JSON object.
#include "../oracle/ws_oracle.h"
#include "driver_options.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <string>
#include <thread>
#include <vector>

using Clock = std::chrono::steady_clock;

namespace {

struct Pipe {
    Pipe* peer = nullptr;
    std::vector<uint8_t> inbox;
    // TCPSession::SendAsync copies the frame into the transport's buffer
    void SendAsync(const uint8_t* p, size_t n) { peer->inbox.insert(peer->inbox.end(), p, p + n); }
};

std::vector<uint8_t> g_message;
std::atomic<bool> g_stop{false};

struct Endpoint {
    wso_session* ws = wso_new();
    Pipe* out = nullptr;
    ~Endpoint() { wso_free(ws); }
    // WSClient/WSSession::SendBinaryAsync: PrepareSendFrame, then SendAsync
    void SendBinaryAsync(const void* buf, size_t n, bool mask)
    {
        wso_prepare_send(ws, 0x82, mask ? 1 : 0, buf, n, 0);
        size_t len = 0;
        const uint8_t* f = wso_send_buffer(ws, &len);
        out->SendAsync(f, len);
    }
};

struct Conn {
    Pipe ct, st;
    Endpoint client, session;
    uint64_t total_bytes = 0, received = 0, bad = 0;
};

// EchoSession::onWSReceived (ws_echo_server.cpp:23-27)
void session_cb(void* user, int kind, const uint8_t* data, size_t len, int)
{
    if (kind == WSO_EV_RECEIVED)
        static_cast<Conn*>(user)->session.SendBinaryAsync(data, len, false);
}

// EchoClient::onWSReceived (ws_echo_client.cpp:63-73)
void client_cb(void* user, int kind, const uint8_t* data, size_t len, int)
{
    if (kind != WSO_EV_RECEIVED)
        return;
    Conn* c = static_cast<Conn*>(user);
    for (size_t i = 0; i < len; ++i)
        c->bad += data[i] != 0;
    c->received += len;
    while (c->received >= g_message.size()) {
        if (!g_stop.load(std::memory_order_relaxed))
            c->client.SendBinaryAsync(g_message.data(), g_message.size(), true);
        c->received -= g_message.size();
    }
    c->total_bytes += len;
}

double seconds(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

} // namespace

int main(int argc, char** argv)
{
    DriverOptions o;
    if (argc >= 6 && argv[1][0] != '-') {
        o.clients = std::atoi(argv[1]);
        o.threads = std::max(1, std::atoi(argv[2]));
        o.messages = std::atol(argv[3]);
        o.size = std::atol(argv[4]);
        o.seconds = std::atof(argv[5]);
    } else if (!parse_driver_options(argc, argv, o)) {
        std::fprintf(stderr, "usage: %s CLIENTS THREADS MESSAGES SIZE SECONDS\n   or: %s [-c] [-t] [-m] [-s] [-z]\n",
                     argv[0], argv[0]);
        return 2;
    }
    const int clients = std::max(1, o.clients), threads = std::max(1, o.threads);
    const size_t messages = size_t(o.messages), size = size_t(o.size);
    g_message.assign(size, 0);
    std::vector<uint64_t> bytes(size_t(threads), 0), bad(size_t(threads), 0);
    std::vector<double> elapsed(size_t(threads), 0.0);
    std::atomic<int> ready{0};
    std::srand(1);

    auto worker = [&](int t) {
        std::vector<std::unique_ptr<Conn>> mine;
        for (int c = t; c < clients; c += threads) {
            auto cn = std::make_unique<Conn>();
            cn->ct.peer = &cn->st;
            cn->st.peer = &cn->ct;
            cn->client.out = &cn->ct;
            cn->session.out = &cn->st;
            wso_set_send_key(cn->client.ws, uint32_t(std::rand()));   // ws.cpp:97
            wso_set_callback(cn->client.ws, client_cb, cn.get());
            wso_set_callback(cn->session.ws, session_cb, cn.get());
            mine.push_back(std::move(cn));
        }
        ready.fetch_add(1);
        while (ready.load() < threads)
            std::this_thread::yield();
        const auto t0 = Clock::now();
        for (auto& c : mine)   // onWSConnected: -m messages in flight
            for (size_t i = 0; i < messages; ++i)
                c->client.SendBinaryAsync(g_message.data(), g_message.size(), true);
        std::vector<uint8_t> buf;
        uint64_t polls = 0;
        for (;;) {
            bool any = false;
            for (auto& c : mine) {
                // one socket read each way: everything pending, one
                // PrepareReceiveFrame call (WSSession/WSClient::onReceived)
                if (!c->st.inbox.empty()) {
                    buf.swap(c->st.inbox);
                    c->st.inbox.clear();
                    wso_prepare_receive(c->session.ws, buf.data(), buf.size());
                    any = true;
                }
                if (!c->ct.inbox.empty()) {
                    buf.swap(c->ct.inbox);
                    c->ct.inbox.clear();
                    wso_prepare_receive(c->client.ws, buf.data(), buf.size());
                    any = true;
                }
            }
            ++polls;
            if ((polls & 15) == 0 && seconds(t0, Clock::now()) >= o.seconds)
                g_stop.store(true, std::memory_order_relaxed);
            if (!any)
                break;
        }
        elapsed[size_t(t)] = seconds(t0, Clock::now());
        for (auto& c : mine) {
            bytes[size_t(t)] += c->total_bytes;
            bad[size_t(t)] += c->bad;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back(worker, t);
    for (auto& th : pool)
        th.join();
    uint64_t total = 0, total_bad = 0;
    double el = 0.0;
    for (int t = 0; t < threads; ++t) {
        total += bytes[size_t(t)];
        total_bad += bad[size_t(t)];
        el = std::max(el, elapsed[size_t(t)]);
    }
    const uint64_t msgs = size ? total / size : 0;
    std::printf("{\"codec\": \"oracle (reference algorithm, CPU)\", \"clients\": %d, \"threads\": %d, "
                "\"messages_in_flight\": %zu, \"size\": %zu, \"seconds\": %.3f, \"total_messages\": %llu, "
                "\"msg_per_s\": %.0f, \"MiB_per_s\": %.3f, \"latency_ns\": %.1f, \"payload_ok\": %s}\n",
                clients, threads, messages, size, el, (unsigned long long)msgs, msgs / el, total / el / (1 << 20),
                msgs ? el * 1e9 / double(msgs) : 0.0, total_bad == 0 ? "true" : "false");
    return 0;
}
