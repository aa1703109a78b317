// test_ws_api.cpp — WSClient / WSSession / WSServer behaviour over an
// in-memory loopback transport, re-expressing the reference's
// tests/test_ws.cpp scenarios (echo :115-183, multicast byte totals
// 4/8/12 :185-307, random soak :309-437) plus ping/pong and sync receive.
// Payload masking runs on the GPU (needs a HIP device).
#include "server/ws/ws_batch.h"
#include "server/ws/ws_client.h"
#include "server/ws/ws_handshake.h"
#include "server/ws/ws_server.h"
#include "server/ws/ws_session.h"
#include "server/ws/wss_client.h"
#include "server/ws/wss_server.h"
#include "server/ws/wss_session.h"

#include "tls_test_certs.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <functional>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <cstring>
#include <vector>

using namespace CppServer::WS;

static int g_failures = 0, g_checks = 0;
#define CHECK(cond)                                                                    \
    do {                                                                               \
        ++g_checks;                                                                    \
        if (!(cond)) {                                                                 \
            ++g_failures;                                                              \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                              \
    } while (0)

// Bytes written by one endpoint land in the peer's inbox; pump() hands each
// inbox to its endpoint's onReceived, as TCPSession::TryReceive does.
struct Loopback : Transport {
    Loopback* peer = nullptr;
    std::deque<uint8_t> inbox;
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
    size_t Receive(void* b, size_t n) override
    {
        const size_t k = std::min(n, inbox.size());
        std::copy(inbox.begin(), inbox.begin() + k, static_cast<uint8_t*>(b));
        inbox.erase(inbox.begin(), inbox.begin() + k);
        return k;
    }
    bool Disconnect() override
    {
        const bool was = connected;
        connected = false;
        if (peer)
            peer->connected = false;
        return was;
    }
    bool IsConnected() const override { return connected; }
};

struct EchoClient : WSClient {
    using WSClient::WSClient;
    size_t received = 0;
    std::vector<std::vector<uint8_t>> messages, pongs;
    bool connected = false, disconnected = false;
    // the upgrade request, as the reference's ws_chat_client example fills it
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
    void onWSConnected(const CppServer::HTTP::HTTPResponse& response) override { connected = true; }
    void onWSDisconnected() override { disconnected = true; }
    void onWSReceived(const void* b, size_t n) override
    {
        received += n;
        messages.emplace_back((const uint8_t*)b, (const uint8_t*)b + n);
    }
    void onWSPong(const void* b, size_t n) override { pongs.emplace_back((const uint8_t*)b, (const uint8_t*)b + n); }
};

// echo session of test_ws.cpp:72-87
struct EchoSession : WSSession {
    using WSSession::WSSession;
    bool echo = true;
    int closes = 0;
    int close_status = 0;
    std::vector<uint8_t> last;
    void onWSReceived(const void* b, size_t n) override
    {
        last.assign((const uint8_t*)b, (const uint8_t*)b + n);
        if (echo)
            SendBinaryAsync(b, n);
    }
    void onWSClose(const void* b, size_t n, int status) override
    {
        ++closes;
        close_status = status;
        WSSession::onWSClose(b, n, status);
    }
};

template <class S = EchoSession>
struct PairT {
    Loopback ct, st;
    std::shared_ptr<EchoClient> client;
    std::shared_ptr<S> session;
    PairT()
    {
        ct.peer = &st;
        st.peer = &ct;
        client = std::make_shared<EchoClient>(ct);
        session = std::make_shared<S>(st);
        session->Connect();
        client->Connect();
        pump();   // upgrade request -> 101 response
    }
    // deliver queued bytes until both inboxes are empty
    void pump()
    {
        for (int guard = 0; guard < 1000 && (!ct.inbox.empty() || !st.inbox.empty()); ++guard) {
            if (!st.inbox.empty()) {
                std::vector<uint8_t> b(st.inbox.begin(), st.inbox.end());
                st.inbox.clear();
                session->onReceived(b.data(), b.size());
            }
            if (!ct.inbox.empty()) {
                std::vector<uint8_t> b(ct.inbox.begin(), ct.inbox.end());
                ct.inbox.clear();
                client->onReceived(b.data(), b.size());
            }
        }
    }
};
using Pair = PairT<>;

static void test_echo()
{
    Pair p;
    CHECK(p.client->connected);
    CHECK(p.client->send_key() != 0 || true);   // client key = rand() (ws.cpp:97), may be 0
    CHECK(p.client->SendTextAsync("test"));
    p.pump();
    CHECK(p.client->received == 4);
    CHECK(p.client->messages.size() == 1 && std::string(p.client->messages[0].begin(), p.client->messages[0].end()) == "test");
}

static void test_multicast()
{
    WSServer server;
    std::vector<std::unique_ptr<Pair>> pairs;
    auto join = [&]() {
        pairs.emplace_back(new Pair());
        pairs.back()->session->echo = false;
        server.AddSession(pairs.back()->session);
    };
    auto pump_all = [&]() {
        for (auto& p : pairs)
            p->pump();
    };
    auto totals = [&]() {
        std::vector<size_t> t;
        for (auto& p : pairs)
            t.push_back(p->client->received);
        return t;
    };
    join();
    server.MulticastText("test");
    pump_all();
    CHECK(totals() == std::vector<size_t>({4}));
    join();
    server.MulticastText("test");
    pump_all();
    CHECK(totals() == std::vector<size_t>({8, 4}));
    join();
    server.MulticastText("test");
    pump_all();
    CHECK(totals() == std::vector<size_t>({12, 8, 4}));
    // client 1 leaves with status 1000 (test_ws.cpp:242)
    pairs[0]->client->CloseAsync(1000);
    CHECK(pairs[0]->client->disconnected);
    server.RemoveSession(pairs[0]->session);
    server.MulticastText("test");
    pump_all();
    CHECK(totals() == std::vector<size_t>({12, 12, 8}));
    server.RemoveSession(pairs[1]->session);
    server.MulticastText("test");
    pump_all();
    CHECK(totals() == std::vector<size_t>({12, 12, 12}));
    CHECK(server.sessions() == 1);
    CHECK(server.CloseAll(1001));
    CHECK(!pairs[2]->session->IsConnected());
}

static void test_ping_pong_and_close()
{
    Pair p;
    p.client->SendPingAsync("ab");
    p.pump();
    // the session answers the ping (payload 00 00 'a' 'b') with a
    // pong, which prepends its own 00 00
    CHECK(p.client->pongs.size() == 1);
    CHECK(p.client->pongs[0] == std::vector<uint8_t>({0, 0, 0, 0, 'a', 'b'}));
    p.client->SendCloseAsync(1001, "bye");
    p.pump();
    CHECK(p.session->closes == 1 && p.session->close_status == 1001);
}

static void test_sync_receive()
{
    Pair p;
    p.session->echo = false;
    std::mt19937 gen(7);
    for (size_t n : {0u, 1u, 125u, 126u, 65535u, 65536u, 200000u}) {
        std::vector<uint8_t> payload(n);
        for (auto& b : payload)
            b = uint8_t(gen());
        CHECK(p.client->SendBinary(payload.data(), payload.size()) == payload.size() + (n < 126 ? 6 : n < 65536 ? 8 : 14));
        // the server reads it with the sync framing loop; the whole message
        // comes back (the reference's +header_size copy offset is not reproduced)
        CHECK(p.session->ReceiveBinary() == payload);
    }
    p.session->SendText("hello");
    CHECK(p.client->ReceiveText() == "hello");
    // the reference's timeout overloads (ws_client.h:55-96, ws_session.h:48-89)
    const CppCommon::Timespan t = CppCommon::Timespan::seconds(1);
    CHECK(p.client->SendText("with timeout", t) == 6 + 12);
    CHECK(p.session->ReceiveText(t) == "with timeout");
    CHECK(p.session->SendBinary("xy", 2, t) == 2 + 2);
    CHECK(p.client->ReceiveBinary(t) == std::vector<uint8_t>({'x', 'y'}));
}

// ConnectAsync (reference ws_client.h:41): the upgrade request is queued on
// the transport; the 101 response completes it through onReceived
static void test_connect_async()
{
    Loopback ct, st;
    ct.peer = &st;
    st.peer = &ct;
    EchoClient client(ct);
    EchoSession session(st);
    session.Connect();
    CHECK(client.ConnectAsync());
    for (int i = 0; i < 4; ++i) {
        if (!st.inbox.empty()) {
            std::vector<uint8_t> b(st.inbox.begin(), st.inbox.end());
            st.inbox.clear();
            session.onReceived(b.data(), b.size());
        }
        if (!ct.inbox.empty()) {
            std::vector<uint8_t> b(ct.inbox.begin(), ct.inbox.end());
            ct.inbox.clear();
            client.onReceived(b.data(), b.size());
        }
    }
    CHECK(client.connected && client.IsConnected());
}

static void test_soak()
{
    std::mt19937 gen(12345);
    std::vector<std::unique_ptr<Pair>> pairs;
    for (int i = 0; i < 4; ++i)
        pairs.emplace_back(new Pair());
    size_t sent_total = 0, echoed_total = 0;
    for (int it = 0; it < 200; ++it) {
        auto& p = *pairs[gen() % pairs.size()];
        const size_t n = (gen() % 4 == 0) ? gen() % 70000 : gen() % 300;
        std::vector<uint8_t> payload(n);
        for (auto& b : payload)
            b = uint8_t(gen());
        const size_t before = p.client->messages.size();
        if (gen() % 2)
            p.client->SendBinaryAsync(payload.data(), payload.size());
        else
            p.client->SendTextAsync(payload.data(), payload.size());
        p.pump();
        sent_total += n;
        CHECK(p.client->messages.size() == before + 1);
        if (p.client->messages.size() == before + 1) {
            CHECK(p.client->messages.back() == payload);
            echoed_total += p.client->messages.back().size();
        }
    }
    CHECK(sent_total == echoed_total);
}

// Server-side batched receive: sessions' bytes are
// framed into one batch and unmasked in one GPU pass per FlushReceived();
// callbacks (and so the echoes) happen only at the flush, in arrival order.
static void test_batched_server_receive(const std::vector<int>& devices = {})
{
    WSServer server;
    std::vector<std::unique_ptr<Pair>> pairs;
    for (int i = 0; i < 8; ++i) {
        pairs.emplace_back(new Pair());
        server.AddSession(pairs.back()->session);
    }
    server.EnableBatchReceive(true);
    if (!devices.empty())
        server.SetBatchDevices(devices);   // flushes spread over these GPUs' links
    CHECK(server.IsBatchReceive());
    std::mt19937 gen(99);
    std::vector<std::vector<std::vector<uint8_t>>> sent(pairs.size());
    // hand a session its inbox in random-sized reads, as TryReceive would
    auto deliver = [&](Pair& p) {
        std::vector<uint8_t> b(p.st.inbox.begin(), p.st.inbox.end());
        p.st.inbox.clear();
        for (size_t at = 0; at < b.size();) {
            const size_t n = std::min<size_t>(b.size() - at, 1 + gen() % 5000);
            p.session->onReceived(b.data() + at, n);
            at += n;
        }
    };
    for (int round = 0; round < 6; ++round) {
        size_t frames = 0;
        for (size_t i = 0; i < pairs.size(); ++i) {
            const int k = 1 + int(gen() % 3);
            for (int j = 0; j < k; ++j) {
                std::vector<uint8_t> payload((gen() % 4 == 0) ? gen() % 70000 : gen() % 300);
                for (auto& b : payload)
                    b = uint8_t(gen());
                pairs[i]->client->SendBinaryAsync(payload.data(), payload.size());
                sent[i].push_back(payload);
                ++frames;
            }
        }
        for (auto& p : pairs)
            deliver(*p);
        bool quiet = true;
        for (auto& p : pairs)
            quiet = quiet && p->ct.inbox.empty() && p->session->last.empty();
        CHECK(quiet);   // nothing delivered before the flush
        CHECK(server.FlushReceived() == frames);
        for (auto& p : pairs) {
            p->session->last.clear();
            p->pump();   // echoes back to the (per-call) clients
        }
    }
    for (size_t i = 0; i < pairs.size(); ++i)
        CHECK(pairs[i]->client->messages == sent[i]);

    // control frames through the batch: ping -> pong, close with status
    pairs[0]->client->SendPingAsync("ab");
    deliver(*pairs[0]);
    CHECK(pairs[0]->client->pongs.empty());
    CHECK(server.FlushReceived() == 1);
    pairs[0]->pump();
    CHECK(pairs[0]->client->pongs.size() == 1 &&
          pairs[0]->client->pongs[0] == std::vector<uint8_t>({0, 0, 0, 0, 'a', 'b'}));
    pairs[1]->client->SendCloseAsync(1001, "bye");
    deliver(*pairs[1]);
    CHECK(server.FlushReceived() == 1);
    CHECK(pairs[1]->session->closes == 1 && pairs[1]->session->close_status == 1001);

    // a removed session's queued frames are dropped, the others still arrive
    pairs[2]->client->SendTextAsync("gone");
    pairs[3]->client->SendTextAsync("kept");
    deliver(*pairs[2]);
    deliver(*pairs[3]);
    server.RemoveSession(pairs[2]->session);
    CHECK(server.FlushReceived() == 1);
    CHECK(std::string(pairs[3]->session->last.begin(), pairs[3]->session->last.end()) == "kept");
    server.EnableBatchReceive(false);
    CHECK(!server.IsBatchReceive());
}

// Batched send: clients share one send batch (masked
// frames, one key per connection), the server batches its sessions' echoes;
// nothing reaches a transport before the flush, and every connection's
// frames keep their order (sync sends and multicasts flush first).
static void test_batched_send()
{
    WSServer server;
    std::vector<std::unique_ptr<Pair>> pairs;
    for (int i = 0; i < 6; ++i) {
        pairs.emplace_back(new Pair());
        server.AddSession(pairs.back()->session);
    }
    server.EnableBatchSend(true);
    CHECK(server.IsBatchSend());
    WSSendBatch client_batch;
    for (auto& p : pairs)
        p->client->SetSendBatch(&client_batch);
    std::mt19937 gen(5);
    std::vector<std::vector<std::vector<uint8_t>>> sent(pairs.size());
    for (int round = 0; round < 4; ++round) {
        size_t frames = 0;
        for (size_t i = 0; i < pairs.size(); ++i) {
            const int k = 1 + int(gen() % 3);
            for (int j = 0; j < k; ++j) {
                std::vector<uint8_t> payload((gen() % 4 == 0) ? gen() % 70000 : gen() % 300);
                for (auto& b : payload)
                    b = uint8_t(gen());
                CHECK(pairs[i]->client->SendBinaryAsync(payload.data(), payload.size()));
                sent[i].push_back(payload);
                ++frames;
            }
        }
        bool quiet = true;
        for (auto& p : pairs)
            quiet = quiet && p->st.inbox.empty();
        CHECK(quiet);
        CHECK(client_batch.Flush() == frames);
        for (auto& p : pairs)
            p->pump();   // sessions receive and queue their echoes
        for (auto& p : pairs)
            quiet = quiet && p->ct.inbox.empty();
        CHECK(quiet);
        CHECK(server.FlushSend() == frames);
        for (auto& p : pairs)
            p->pump();
    }
    for (size_t i = 0; i < pairs.size(); ++i)
        CHECK(pairs[i]->client->messages == sent[i]);

    // order: an async frame queued before a sync send / a multicast goes first
    auto& p = *pairs[0];
    p.client->messages.clear();
    p.session->SendTextAsync("a");
    p.session->SendText("b");
    server.MulticastText("c");   // batched too: one frame for every session at the flush
    p.session->SendTextAsync("d");
    CHECK(server.FlushSend() == 2);
    p.pump();
    std::vector<std::string> got;
    for (auto& m : p.client->messages)
        got.emplace_back(m.begin(), m.end());
    CHECK(got == std::vector<std::string>({"a", "b", "c", "d"}));
    for (auto& q : pairs)
        q->client->SetSendBatch(nullptr);
    server.EnableBatchSend(false);
}

// A flush hands each transport its frames in runs: consecutive frames for one
// transport lie contiguous in the wire and go out in one SendAsync; the bytes
// and their order are exactly the per-frame hand-outs'.
static void test_send_batch_runs()
{
    struct Counting : Transport {
        std::vector<std::vector<uint8_t>> calls;
        size_t Send(const void* b, size_t n) override { return SendAsync(b, n) ? n : 0; }
        bool SendAsync(const void* b, size_t n) override
        {
            calls.emplace_back(static_cast<const uint8_t*>(b), static_cast<const uint8_t*>(b) + n);
            return true;
        }
        size_t Receive(void*, size_t) override { return 0; }
        bool Disconnect() override { return true; }
        bool IsConnected() const override { return true; }
    } a, b;
    WSSendBatch batch;
    const std::vector<std::pair<Counting*, std::string>> order = {
        {&a, "a1"}, {&a, "a2"}, {&a, std::string(300, 'x')}, {&b, "b1"}, {&a, "a3"}, {&b, "b2"}, {&b, ""}};
    std::vector<uint8_t> want_a, want_b;
    for (const auto& [t, text] : order) {
        batch.Queue(*t, 0, WSG_FIN | WSG_BINARY, false, text.data(), text.size(), 0);
        std::vector<uint8_t>& w = t == &a ? want_a : want_b;
        w.push_back(WSG_FIN | WSG_BINARY);
        if (text.size() < 126) {
            w.push_back(uint8_t(text.size()));
        } else {
            w.push_back(126);
            w.push_back(uint8_t(text.size() >> 8));
            w.push_back(uint8_t(text.size()));
        }
        w.insert(w.end(), text.begin(), text.end());
    }
    CHECK(batch.Flush() == order.size());
    CHECK(a.calls.size() == 2 && b.calls.size() == 2);   // runs: a a a | b | a | b b
    std::vector<uint8_t> got_a, got_b;
    for (auto& c : a.calls)
        got_a.insert(got_a.end(), c.begin(), c.end());
    for (auto& c : b.calls)
        got_b.insert(got_b.end(), c.begin(), c.end());
    CHECK(got_a == want_a && got_b == want_b);
    CHECK(a.calls.size() == 2 && a.calls[1].size() == 4);   // "a3" alone: its own hand-out
}

// Automatic batching (ws_batch.h BatchScope): the drop-in path, no batch
// set up by the user.  Sends inside a tick leave in one encode pass at its
// end; a read's frames are unmasked in one pass and the echoes they trigger
// go out in one more; messages and their order are the per-call path's.
static void test_auto_batch_echo()
{
    for (int enabled = 1; enabled >= 0; --enabled) {
        BatchScope::SetEnabled(enabled != 0);
        Pair p;
        std::vector<std::vector<uint8_t>> sent;
        std::mt19937 gen(11 + enabled);
        {
            BatchScope tick;
            for (int i = 0; i < 300; ++i) {
                std::vector<uint8_t> m(gen() % 7 == 0 ? 70000 + gen() % 100 : gen() % 64);
                for (auto& b : m)
                    b = uint8_t(gen());
                CHECK(p.client->SendBinaryAsync(m.data(), m.size()));
                sent.push_back(m);
            }
            if (enabled)
                CHECK(p.st.inbox.empty());   // queued until the tick ends
        }
        CHECK(!p.st.inbox.empty());
        p.pump();
        CHECK(p.client->messages == sent);
        CHECK(p.session->last == sent.back());
        // a sync send inside a tick flushes what the tick queued first
        p.client->messages.clear();
        {
            BatchScope tick;
            p.client->SendTextAsync("x");
            p.client->SendText("y");
            p.client->SendTextAsync("z");
        }
        p.pump();
        std::vector<std::string> got;
        for (auto& m : p.client->messages)
            got.emplace_back(m.begin(), m.end());
        CHECK(got == std::vector<std::string>({"x", "y", "z"}));
    }
    BatchScope::SetEnabled(true);
}

// ws_multicast's tick: `messages_rate` MulticastBinary calls in one scope are
// encoded in one pass and reach every session registered at the call, in order.
static void test_multicast_tick()
{
    WSServer server;
    std::vector<std::unique_ptr<Pair>> pairs;
    for (int i = 0; i < 5; ++i) {
        pairs.emplace_back(new Pair());
        pairs.back()->session->echo = false;
        server.AddSession(pairs.back()->session);
    }
    std::vector<std::vector<uint8_t>> msgs;
    {
        BatchScope tick;
        for (int i = 0; i < 10; ++i) {
            std::vector<uint8_t> m(32, uint8_t(i));
            msgs.push_back(m);
            CHECK(server.MulticastBinary(m.data(), m.size()) == 1);
        }
        pairs.emplace_back(new Pair());   // joins after the calls: gets none of them
        pairs.back()->session->echo = false;
        server.AddSession(pairs.back()->session);
        for (auto& p : pairs)
            CHECK(p->ct.inbox.empty());
    }
    for (auto& p : pairs)
        p->pump();
    for (size_t i = 0; i + 1 < pairs.size(); ++i)
        CHECK(pairs[i]->client->messages == msgs);
    CHECK(pairs.back()->client->messages.empty());
}

// One explicit send batch fed from several threads at once (a WSServer's
// sessions on different IO threads), flushed from yet another.
// A session whose first delivery runs a hook (test_cross_thread_drain_keyed)
struct HookSession : EchoSession {
    using EchoSession::EchoSession;
    std::function<void()> on_first;
    int calls = 0;
    void onWSReceived(const void* b, size_t n) override
    {
        EchoSession::onWSReceived(b, n);
        if (calls++ == 0 && on_first)
            on_first();
    }
};

// Two threads flushing two receive batches, each from inside a callback
// moving a session off the OTHER batch while its masked frame is still
// queued there (WSReceiveBatch::Drain): the frame is unmasked on
// the moving thread's own codec — the other batch's contexts (one batch split
// over two contexts of the GPU) belong to its running flush — and delivered
// before SetReceiveBatch returns, bit-exact; the flushes do not wait for
// each other.  The host-only form of this test (unmasked frames) runs under
// the sanitizers (tests/cpp/test_batch_threads.cpp).
static void test_cross_thread_drain_keyed()
{
    setenv("WSG_HOST_MULTI_SHARE", "1", 1);
    for (int iter = 0; iter < 20; ++iter) {
        WSReceiveBatch x(nullptr), y(nullptr);
        y.SetDevices({0, 0});
        PairT<HookSession> tx, ty;   // the first delivery of each flush
        Pair sx, sy;                 // moved off y (by x's flusher) / off x (by y's flusher)
        for (EchoSession* s : {static_cast<EchoSession*>(tx.session.get()), static_cast<EchoSession*>(ty.session.get()),
                               sx.session.get(), sy.session.get()})
            s->echo = false;
        tx.session->SetReceiveBatch(&x);
        ty.session->SetReceiveBatch(&y);
        sx.session->SetReceiveBatch(&y);
        sy.session->SetReceiveBatch(&x);
        std::mt19937 gen(1000 + iter);
        auto frame = [&](auto& p, size_t n) {
            std::vector<uint8_t> payload(n);
            for (auto& b : payload)
                b = uint8_t(gen());
            CHECK(p.client->SendBinaryAsync(payload.data(), payload.size()));   // masked with the client's key
            return payload;
        };
        const auto ptx = frame(tx, 700), pty = frame(ty, 3000), psx = frame(sx, 40 + iter), psy = frame(sy, 5000);
        std::mutex m;
        std::condition_variable cv;
        int inside = 0;
        std::atomic<int> done{0};
        auto both_inside = [&] {
            std::unique_lock<std::mutex> g(m);
            ++inside;
            cv.notify_all();
            cv.wait(g, [&] { return inside == 2; });
        };
        auto move_off = [&](Pair& p, const std::vector<uint8_t>& want) {
            std::vector<uint8_t> b(p.st.inbox.begin(), p.st.inbox.end());
            p.st.inbox.clear();
            p.session->onReceived(b.data(), b.size());   // queued in the batch the other thread flushes
            p.session->SetReceiveBatch(nullptr);         // delivered before this returns
            CHECK(p.session->last == want);
        };
        tx.session->on_first = [&] { both_inside(); move_off(sx, psx); };
        ty.session->on_first = [&] { both_inside(); move_off(sy, psy); };
        auto feed = [](auto& p) {
            std::vector<uint8_t> b(p.st.inbox.begin(), p.st.inbox.end());
            p.st.inbox.clear();
            p.session->onReceived(b.data(), b.size());
        };
        feed(tx);
        feed(ty);
        std::thread watchdog([&] {
            for (int i = 0; i < 300 && done.load() < 2; ++i)
                std::this_thread::sleep_for(std::chrono::milliseconds(100));
            if (done.load() < 2) {
                std::fprintf(stderr, "cross-thread drain (keyed): flushes blocked on each other\n");
                std::_Exit(3);
            }
        });
        std::thread a([&] { x.Flush(); ++done; });
        std::thread b([&] { y.Flush(); ++done; });
        a.join();
        b.join();
        watchdog.join();
        CHECK(tx.session->last == ptx && ty.session->last == pty);
        CHECK(x.Flush() == 0 && y.Flush() == 0);   // nothing left behind
        tx.session->SetReceiveBatch(nullptr);
        ty.session->SetReceiveBatch(nullptr);
    }
    unsetenv("WSG_HOST_MULTI_SHARE");
}

static void test_batch_threads()
{
    WSSendBatch batch;
    const int T = 4, N = 2000;
    std::vector<std::thread> th;
    std::vector<int> tags(T);
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t]() {
            for (int i = 0; i < N; ++i) {
                const uint32_t v = uint32_t(t * N + i);
                batch.Queue(&tags[t], 0x01020304u, WSG_FIN | WSG_BINARY, true, &v, sizeof(v));
            }
        });
    size_t flushed = 0;
    struct Count {
        std::vector<uint32_t> last;
        size_t n = 0;
        bool ordered = true;
        int* base;
    } cnt{std::vector<uint32_t>(T, 0), 0, true, tags.data()};
    auto sink = [](void* user, void* tag, const uint8_t* f, size_t len) {
        Count* c = static_cast<Count*>(user);
        const int t = int(static_cast<int*>(tag) - c->base);
        uint32_t v;
        std::memcpy(&v, f + len - 4, 4);
        const uint8_t k[4] = {4, 3, 2, 1};
        uint8_t* b = reinterpret_cast<uint8_t*>(&v);
        for (int j = 0; j < 4; ++j)
            b[j] ^= k[j];   // unmask (key bytes little-endian, ws.cpp:244-247)
        if (c->last[size_t(t)] && v <= c->last[size_t(t)])
            c->ordered = false;
        c->last[size_t(t)] = v;
        ++c->n;
    };
    for (int round = 0; round < 50; ++round)
        flushed += batch.Flush(sink, &cnt);
    for (auto& x : th)
        x.join();
    flushed += batch.Flush(sink, &cnt);
    CHECK(flushed == size_t(T) * N);
    CHECK(cnt.n == size_t(T) * N);
    CHECK(cnt.ordered);
}

// WSS (reference include/server/ws/wss_*.h): the same codec over a real TLS
// session (OpenSSL TLS 1.3 through TLSTransport, certificates made at run
// time), records pumped between the two byte transports.  Frames both ways,
// a 70 KB one (several TLS records), a multicast, and the batched paths: the
// server's batched receive and send run on the decrypted bytes / encrypt
// the encoded frames.
struct TlsClient : WSSClient {
    using WSSClient::WSSClient;
    std::vector<std::vector<uint8_t>> messages;
    void onWSConnecting(CppServer::HTTP::HTTPRequest& request) override
    {
        request.SetBegin("GET", "/");
        request.SetHeader("Host", "localhost");
        request.SetHeader("Upgrade", "websocket");
        request.SetHeader("Connection", "Upgrade");
        request.SetHeader("Sec-WebSocket-Key", Base64Encode(ws_nonce()));
        request.SetHeader("Sec-WebSocket-Version", "13");
    }
    void onWSReceived(const void* b, size_t n) override { messages.emplace_back((const uint8_t*)b, (const uint8_t*)b + n); }
};

struct TlsSession : WSSSession {
    using WSSSession::WSSSession;
    void onWSReceived(const void* b, size_t n) override { SendBinaryAsync(b, n); }
};

static void test_wss()
{
    using CppServer::Asio::SSLContext;
    const TestPki pki = make_test_pki();
    auto sctx = std::make_shared<SSLContext>(asio::ssl::context::tlsv13);
    sctx->use_certificate_chain(pki.server_cert_pem.data(), pki.server_cert_pem.size());
    sctx->use_private_key(pki.server_key_pem.data(), pki.server_key_pem.size(), asio::ssl::context::pem);
    auto cctx = std::make_shared<SSLContext>(asio::ssl::context::tlsv13);
    cctx->set_verify_mode(asio::ssl::verify_peer | asio::ssl::verify_fail_if_no_peer_cert);
    cctx->add_certificate_authority(pki.ca_pem.data(), pki.ca_pem.size());

    for (int batched = 0; batched < 2; ++batched) {
        Loopback ct, st;
        ct.peer = &st;
        st.peer = &ct;
        TlsClient client(cctx, ct);
        WSSServer server(sctx);
        auto session = std::make_shared<TlsSession>(server.context(), st);
        server.AddSession(session);
        if (batched) {
            server.EnableBatchReceive(true);
            server.EnableBatchSend(true);
        }
        size_t wire_bytes = 0;
        auto pump = [&] {
            for (int guard = 0; guard < 200 && (!ct.inbox.empty() || !st.inbox.empty()); ++guard) {
                if (!st.inbox.empty()) {
                    std::vector<uint8_t> b(st.inbox.begin(), st.inbox.end());
                    st.inbox.clear();
                    wire_bytes += b.size();
                    session->onReceived(b.data(), b.size());
                    if (batched) {
                        server.FlushReceived();
                        server.FlushSend();
                    }
                }
                if (!ct.inbox.empty()) {
                    std::vector<uint8_t> b(ct.inbox.begin(), ct.inbox.end());
                    ct.inbox.clear();
                    wire_bytes += b.size();
                    client.onReceived(b.data(), b.size());
                }
            }
        };
        CHECK(session->Connect());
        CHECK(client.Connect());
        pump();
        CHECK(client.IsHandshaked() && client.IsConnected() && session->IsConnected());
        std::vector<uint8_t> big(70000);
        for (size_t i = 0; i < big.size(); ++i)
            big[i] = uint8_t(i * 7 + 1);
        CHECK(client.SendBinaryAsync(big.data(), big.size()));
        CHECK(client.SendTextAsync("over tls"));
        pump();
        CHECK(client.messages.size() == 2 && client.messages[0] == big &&
              std::string(client.messages[1].begin(), client.messages[1].end()) == "over tls");
        CHECK(wire_bytes > 2 * big.size());   // both directions, plus record overhead
        CHECK(server.MulticastText("all") > 0);
        if (batched)
            server.FlushSend();
        pump();
        CHECK(client.messages.size() == 3 && std::string(client.messages[2].begin(), client.messages[2].end()) == "all");
        server.RemoveSession(session);
    }

    // records cut at random points both ways (partial records, several per
    // read), 60 messages of 0-5000 bytes echoed: same messages, same order
    {
        Loopback ct, st;
        ct.peer = &st;
        st.peer = &ct;
        TlsClient client(cctx, ct);
        auto session = std::make_shared<TlsSession>(sctx, st);
        uint64_t rng = 777;
        auto next = [&rng]() {
            rng ^= rng << 13;
            rng ^= rng >> 7;
            rng ^= rng << 17;
            return rng;
        };
        auto dribble = [&](Loopback& from, auto&& feed) {
            std::vector<uint8_t> rec(from.inbox.begin(), from.inbox.end());
            from.inbox.clear();
            for (size_t at = 0; at < rec.size();) {
                const size_t n = std::min<size_t>(rec.size() - at, 1 + next() % 900);
                feed(rec.data() + at, n);
                at += n;
            }
        };
        auto pump = [&] {
            for (int guard = 0; guard < 400 && (!ct.inbox.empty() || !st.inbox.empty()); ++guard) {
                dribble(st, [&](const void* p, size_t n) { session->onReceived(p, n); });
                dribble(ct, [&](const void* p, size_t n) { client.onReceived(p, n); });
            }
        };
        CHECK(session->Connect());
        CHECK(client.Connect());
        pump();
        CHECK(client.IsConnected() && session->IsConnected());
        std::vector<std::vector<uint8_t>> sent;
        for (int i = 0; i < 60; ++i) {
            std::vector<uint8_t> m(size_t(next() % 5000));
            for (auto& x : m)
                x = uint8_t(next());
            sent.push_back(m);
            CHECK(client.SendBinaryAsync(m.data(), m.size()));
            if (i % 7 == 0)
                pump();
        }
        pump();
        CHECK(client.messages == sent);

        // four threads sending on the one TLS connection at once (outside
        // any read): records stay in sequence, every thread's messages
        // arrive in its own order
        client.messages.clear();
        constexpr int T = 4, M = 50;
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t)
            th.emplace_back([&client, t] {
                for (int m = 0; m < M; ++m) {
                    const uint8_t msg[3] = {uint8_t(t), uint8_t(m), uint8_t(t ^ m)};
                    client.SendBinaryAsync(msg, sizeof msg);
                }
            });
        for (auto& x : th)
            x.join();
        pump();
        CHECK(client.messages.size() == size_t(T) * M);
        int next_of[T] = {0, 0, 0, 0};
        bool ordered = true;
        for (const auto& m : client.messages) {
            if (m.size() != 3 || m[0] >= T || m[1] != next_of[m[0]] || m[2] != uint8_t(m[0] ^ m[1]))
                ordered = false;
            else
                ++next_of[m[0]];
        }
        CHECK(ordered);
    }
}

int main()
{
    try {
        test_echo();
        test_multicast();
        test_ping_pong_and_close();
        test_sync_receive();
        test_connect_async();
        test_soak();
        test_batched_server_receive();
        // the same with every flush split over three contexts of the one GPU
        // (as over three GPUs: wsg_decode_batch_host_multi)
        setenv("WSG_HOST_MULTI_SHARE", "1", 1);
        test_batched_server_receive({0, 0, 0});
        unsetenv("WSG_HOST_MULTI_SHARE");
        test_batched_send();
        test_send_batch_runs();
        test_auto_batch_echo();
        test_multicast_tick();
        test_batch_threads();
        test_cross_thread_drain_keyed();
        test_wss();
    } catch (const std::exception& e) {
        std::fprintf(stderr, "exception: %s\n", e.what());
        return 2;
    }
    std::printf("%d checks, %d failures\n", g_checks, g_failures);
    return g_failures == 0 ? 0 : 1;
}
