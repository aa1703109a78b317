// bench_echo_tcp.cpp — BASELINE config C1 over real loopback TCP, the way the
// reference measures it (performance/ws_echo_server.cpp + ws_echo_client.cpp
// on 127.0.0.1; README.md:3312-3352): so the published figures have a
// like-for-like counterpart on this host.  A measurement tool: the socket
// layer here is a minimal non-blocking epoll loop (sockets are out of the
// product's scope; §7 step 9 asks for one for C1 only).
//
// Workload (ws_echo_client.cpp:32-90, ws_echo_server.cpp:17-33): C clients,
// each sends -m messages of -s zero bytes once its WebSocket upgrade
// completes and one more per message echoed back; the server session echoes
// with SendBinaryAsync.  Metric (ws_echo_client.cpp:191-201): messages =
// echoed bytes / size over the wall time.  Server and client run in one
// process, each side on T threads of its own (an epoll set per thread,
// connections dealt round-robin), like the two reference processes.
//
// Codecs:
//   gpu       this repo's WSClient / WSSession (upgrade handshake included;
//             every read is a BatchScope: one GPU unmask pass for its
//             frames, one encode pass for the echoes it triggers)
//   gpu_tick  the same with one BatchScope around each epoll pass
//   cpu_ref   the reference's algorithm on the CPU: the oracle's restatement
//             of PrepareSendFrame / PrepareReceiveFrame (ws.cpp:212-456),
//             frames from the first byte (no upgrade), no GPU
//
//   bench_echo_tcp CODEC CLIENTS THREADS MESSAGES SIZE SECONDS
// Prints one JSON object.
#include "server/ws/ws_batch.h"
#include "server/ws/ws_client.h"
#include "server/ws/ws_handshake.h"
#include "server/ws/ws_session.h"

#include "../oracle/ws_oracle.h"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

using namespace CppServer::WS;
using Clock = std::chrono::steady_clock;

namespace {

std::vector<uint8_t> g_message;
std::atomic<bool> g_stop{false};

void fail(const char* what)
{
    throw std::runtime_error(std::string(what) + ": " + std::strerror(errno));
}

void nonblocking(int fd)
{
    if (fcntl(fd, F_SETFL, fcntl(fd, F_GETFL) | O_NONBLOCK) < 0)
        fail("fcntl");
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof one);
}

// A socket as the connection's Transport: sends append to an output buffer
// that the loop writes out after every pass (TCPSession::SendAsync copies
// into its send buffer, tcp_session.cpp:257-307).
struct TcpTransport : Transport {
    int fd = -1;
    std::vector<uint8_t> out;
    size_t sent = 0;   // bytes of `out` already written
    bool closed = false;
    size_t Send(const void* b, size_t n) override { return SendAsync(b, n) ? n : 0; }
    bool SendAsync(const void* b, size_t n) override
    {
        const uint8_t* p = static_cast<const uint8_t*>(b);
        out.insert(out.end(), p, p + n);
        return !closed;
    }
    size_t Receive(void*, size_t) override { return 0; }
    bool Disconnect() override
    {
        closed = true;
        return true;
    }
    bool IsConnected() const override { return !closed; }
    // write what is pending; false when the peer went away
    bool flush()
    {
        while (sent < out.size()) {
            const ssize_t k = ::send(fd, out.data() + sent, out.size() - sent, MSG_NOSIGNAL);
            if (k > 0) {
                sent += size_t(k);
                continue;
            }
            if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK))
                return true;
            return false;
        }
        out.clear();
        sent = 0;
        return true;
    }
};

struct EchoSession : WSSession {
    using WSSession::WSSession;
    void onWSReceived(const void* buffer, size_t size) override { SendBinaryAsync(buffer, size); }
};

struct EchoClient : WSClient {
    EchoClient(size_t messages, Transport& t) : WSClient(t), _messages(messages) {}
    uint64_t total_bytes = 0, bad = 0;
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
    void onWSConnected(const CppServer::HTTP::HTTPResponse&) override
    {
        for (size_t i = _messages; i > 0; --i)
            SendBinaryAsync(g_message.data(), g_message.size());
    }
    void onWSReceived(const void* buffer, size_t size) override
    {
        const uint8_t* b = static_cast<const uint8_t*>(buffer);
        for (size_t i = 0; i < size; ++i)
            bad += b[i] != 0;
        _received += size;
        while (_received >= g_message.size()) {
            if (!g_stop.load(std::memory_order_relaxed))
                SendBinaryAsync(g_message.data(), g_message.size());
            _received -= g_message.size();
        }
        total_bytes += size;
    }

private:
    size_t _received = 0;
    size_t _messages;
};

// One end of one connection, either codec.
struct End {
    TcpTransport t;
    bool client = false;
    // gpu codecs
    std::unique_ptr<EchoClient> wc;
    std::unique_ptr<EchoSession> ws;
    // cpu_ref codec
    wso_session* os = nullptr;
    uint64_t total_bytes = 0, received = 0, bad = 0;
    ~End()
    {
        if (os)
            wso_free(os);
        if (t.fd >= 0)
            ::close(t.fd);
    }
    void send_ref(const void* b, size_t n, bool mask)
    {
        wso_prepare_send(os, 0x82, mask ? 1 : 0, b, n, 0);
        size_t len = 0;
        const uint8_t* f = wso_send_buffer(os, &len);
        t.SendAsync(f, len);
    }
    void on_bytes(const uint8_t* b, size_t n)
    {
        if (os)
            wso_prepare_receive(os, b, n);
        else if (wc)
            wc->onReceived(b, n);
        else
            ws->onReceived(b, n);
    }
};

// cpu_ref callbacks: the server echoes (ws_echo_server.cpp:23-27), the client
// counts and re-sends (ws_echo_client.cpp:63-73)
void ref_cb(void* user, int kind, const uint8_t* data, size_t len, int)
{
    End* e = static_cast<End*>(user);
    if (kind != WSO_EV_RECEIVED)
        return;
    if (!e->client) {
        e->send_ref(data, len, false);
        return;
    }
    for (size_t i = 0; i < len; ++i)
        e->bad += data[i] != 0;
    e->received += len;
    while (e->received >= g_message.size()) {
        if (!g_stop.load(std::memory_order_relaxed))
            e->send_ref(g_message.data(), g_message.size(), true);
        e->received -= g_message.size();
    }
    e->total_bytes += len;
}

double seconds(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// One IO thread: its connections' ends (client ends or server ends), one epoll set.
// Per-run path counters: socket reads, and this process's lane use as the
// IO threads' codec contexts saw it (wsg_lane_stats at each thread's end).
std::atomic<uint64_t> g_reads{0}, g_lane_requests{0}, g_lane_launches{0}, g_lane_give_ups{0};
std::atomic<int> g_lane_state{2};   // lowest seen: -1 given up, 0 not running, 1 running (2: none read)

void io_loop(std::vector<End*>& ends, bool tick, double secs, bool client_side, std::atomic<int>& done_clients,
             int n_client_threads, double& elapsed, bool gpu)
{
    const int ep = epoll_create1(0);
    if (ep < 0)
        fail("epoll_create1");
    for (End* e : ends) {
        epoll_event ev{};
        ev.events = EPOLLIN;
        ev.data.ptr = e;
        if (epoll_ctl(ep, EPOLL_CTL_ADD, e->t.fd, &ev) < 0)
            fail("epoll_ctl");
    }
    std::vector<epoll_event> evs(256);
    std::vector<uint8_t> buf(1 << 16);
    uint64_t reads = 0;
    const auto t0 = Clock::now();
    auto idle_since = Clock::now();
    for (;;) {
        for (End* e : ends)
            if (!e->t.flush())
                e->t.closed = true;
        const int k = epoll_wait(ep, evs.data(), int(evs.size()), 1);
        {
            std::unique_ptr<BatchScope> scope;
            if (tick)
                scope = std::make_unique<BatchScope>();   // one GPU pass each way for the whole pass
            for (int i = 0; i < k; ++i) {
                End* e = static_cast<End*>(evs[size_t(i)].data.ptr);
                for (;;) {   // drain the socket: every read is one onReceived (TCPSession::TryReceive)
                    const ssize_t r = ::recv(e->t.fd, buf.data(), buf.size(), 0);
                    if (r > 0) {
                        ++reads;
                        e->on_bytes(buf.data(), size_t(r));
                        if (size_t(r) < buf.size())
                            break;
                        continue;
                    }
                    if (r == 0)
                        e->t.closed = true;
                    break;
                }
            }
        }
        const auto now = Clock::now();
        if (client_side && seconds(t0, now) >= secs)
            g_stop.store(true, std::memory_order_relaxed);
        if (k > 0)
            idle_since = now;
        // clients: done once stopped and nothing arrived for 50 ms (every
        // echo drained); servers: once every client thread is done
        if (client_side && g_stop.load() && seconds(idle_since, now) > 0.05) {
            elapsed = seconds(t0, idle_since);
            done_clients.fetch_add(1);
            break;
        }
        if (!client_side && done_clients.load() >= n_client_threads)
            break;
    }
    ::close(ep);
    g_reads.fetch_add(reads);
    if (gpu) {
        uint64_t rq = 0, la = 0;
        int st = 0;
        if (wsg_lane_stats(ThreadCodec(), &rq, &la, &st) == WSG_OK) {
            g_lane_requests.fetch_add(rq);
            uint64_t m = g_lane_launches.load();
            while (la > m && !g_lane_launches.compare_exchange_weak(m, la)) {
            }
            int cur = g_lane_state.load();
            while (st < cur && !g_lane_state.compare_exchange_weak(cur, st)) {
            }
        }
        uint64_t gu = 0;
        if (wsg_lane_events(ThreadCodec(), &gu, nullptr) == WSG_OK) {   // (the device's lane: the same for all)
            uint64_t m = g_lane_give_ups.load();
            while (gu > m && !g_lane_give_ups.compare_exchange_weak(m, gu)) {
            }
        }
    }
}

} // namespace

int main(int argc, char** argv)
{
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s gpu|gpu_tick|cpu_ref CLIENTS THREADS MESSAGES SIZE SECONDS\n", argv[0]);
        return 2;
    }
    const std::string codec = argv[1];
    const int clients = std::max(1, std::atoi(argv[2])), threads = std::max(1, std::atoi(argv[3]));
    const size_t messages = size_t(std::atol(argv[4])), size = size_t(std::atol(argv[5]));
    const double secs = std::atof(argv[6]);
    const bool ref = codec == "cpu_ref", tick = codec == "gpu_tick";
    g_message.assign(size, 0);
    std::srand(1);
    try {
        // listening socket on an ephemeral loopback port
        const int ls = ::socket(AF_INET, SOCK_STREAM, 0);
        if (ls < 0)
            fail("socket");
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        a.sin_port = 0;
        if (::bind(ls, reinterpret_cast<sockaddr*>(&a), sizeof a) < 0 || ::listen(ls, 1024) < 0)
            fail("bind/listen");
        socklen_t al = sizeof a;
        getsockname(ls, reinterpret_cast<sockaddr*>(&a), &al);

        std::vector<std::unique_ptr<End>> cends, sends;
        for (int c = 0; c < clients; ++c) {
            auto ce = std::make_unique<End>();
            ce->client = true;
            ce->t.fd = ::socket(AF_INET, SOCK_STREAM, 0);
            if (ce->t.fd < 0 || ::connect(ce->t.fd, reinterpret_cast<sockaddr*>(&a), sizeof a) < 0)
                fail("connect");
            auto se = std::make_unique<End>();
            se->t.fd = ::accept(ls, nullptr, nullptr);
            if (se->t.fd < 0)
                fail("accept");
            nonblocking(ce->t.fd);
            nonblocking(se->t.fd);
            if (ref) {
                ce->os = wso_new();
                se->os = wso_new();
                wso_set_send_key(ce->os, uint32_t(std::rand()));   // ws.cpp:97
                wso_set_callback(ce->os, ref_cb, ce.get());
                wso_set_callback(se->os, ref_cb, se.get());
            } else {
                ce->wc = std::make_unique<EchoClient>(messages, ce->t);
                se->ws = std::make_unique<EchoSession>(se->t);
                se->ws->Connect();   // waits for the upgrade request
            }
            cends.push_back(std::move(ce));
            sends.push_back(std::move(se));
        }
        ::close(ls);
        // start: the upgrade (gpu) or -m messages at once (cpu_ref, no upgrade)
        for (auto& ce : cends) {
            if (ref)
                for (size_t i = 0; i < messages; ++i)
                    ce->send_ref(g_message.data(), g_message.size(), true);
            else
                ce->wc->Connect();
        }
        std::vector<std::vector<End*>> cpart(static_cast<size_t>(threads)), spart(static_cast<size_t>(threads));
        for (int c = 0; c < clients; ++c) {
            cpart[size_t(c % threads)].push_back(cends[size_t(c)].get());
            spart[size_t(c % threads)].push_back(sends[size_t(c)].get());
        }
        std::atomic<int> done{0};
        std::vector<double> elapsed(size_t(threads), 0.0), unused(size_t(threads), 0.0);
        std::vector<std::string> errors(size_t(2 * threads));
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t) {
            pool.emplace_back([&, t] {
                try {
                    BatchScope::SetEnabled(true);
                    io_loop(spart[size_t(t)], tick, secs, false, done, threads, unused[size_t(t)], !ref);
                } catch (const std::exception& e) {
                    errors[size_t(t)] = e.what();
                }
            });
            pool.emplace_back([&, t] {
                try {
                    BatchScope::SetEnabled(true);
                    io_loop(cpart[size_t(t)], tick, secs, true, done, threads, elapsed[size_t(t)], !ref);
                } catch (const std::exception& e) {
                    errors[size_t(threads + t)] = e.what();
                    done.fetch_add(1);
                }
            });
        }
        for (auto& th : pool)
            th.join();
        for (auto& e : errors)
            if (!e.empty())
                throw std::runtime_error(e);
        uint64_t total = 0, bad = 0;
        for (auto& ce : cends) {
            total += ref ? ce->total_bytes : ce->wc->total_bytes;
            bad += ref ? ce->bad : ce->wc->bad;
        }
        double el = 0;
        for (double x : elapsed)
            el = std::max(el, x);
        const uint64_t msgs = size ? total / size : 0;
        std::printf("{\"codec\": \"%s\", \"transport\": \"TCP 127.0.0.1 (epoll)\", \"clients\": %d, \"threads\": %d, "
                    "\"messages_in_flight\": %zu, \"size\": %zu, \"seconds\": %.3f, \"total_messages\": %llu, "
                    "\"msg_per_s\": %.0f, \"MiB_per_s\": %.3f, \"latency_ns\": %.1f, \"payload_ok\": %s, \"reads\": %llu, "
                    "\"lane_requests\": %llu, \"lane_launches\": %llu, \"lane_state\": %d, \"lane_give_ups\": %llu}\n",
                    codec.c_str(), clients, threads, messages, size, el, (unsigned long long)msgs, msgs / el,
                    total / el / (1 << 20), msgs ? el * 1e9 / double(msgs) : 0.0, bad == 0 ? "true" : "false",
                    (unsigned long long)g_reads.load(), (unsigned long long)g_lane_requests.load(),
                    (unsigned long long)g_lane_launches.load(), g_lane_state.load(),
                    (unsigned long long)g_lane_give_ups.load());
    } catch (const std::exception& e) {
        std::fprintf(stderr, "bench_echo_tcp: %s\n", e.what());
        return 3;
    }
    return 0;
}
