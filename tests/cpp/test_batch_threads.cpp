// test_batch_threads.cpp — the batches across threads (host only, no GPU):
// one thread flushes (delivering frames to connections, handing frames to
// transports) while another Forgets and destroys connections and
// transports; a connection destroyed on one thread while another thread's
// BatchScope still holds frames it queued; and a server's batched receive
// and send switched on and off while IO threads read and send (a
// read that had loaded the batch fed it after EnableBatchReceive(false) had
// freed it).  Built twice by
// tests/cpp/Makefile, under ThreadSanitizer and under AddressSanitizer, and
// run by tests/test_sanitize.py.  Every frame carries key 0 (the server
// direction, reference ws.cpp:206) or no mask, so no GPU pass runs: the batches
// frame and hand out the bytes on the host exactly as they do around a GPU pass.
#include "server/ws/ws_batch.h"
#include "server/ws/ws_server.h"
#include "server/ws/ws_session.h"
#include "server/ws/ws_transport.h"

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

using namespace CppServer::WS;

// The batches keep their frames in page-locked memory (wsg_host_alloc, HIP)
// for the GPU pass; this host-only test has no device, so the executable's
// own definitions take the place of libwsg.so's (symbol interposition): plain
// heap memory, which is all a batch needs when no GPU pass runs.
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

static std::atomic<int> g_failures{0}, g_checks{0};
#define CHECK(cond)                                                                    \
    do {                                                                               \
        ++g_checks;                                                                    \
        if (!(cond)) {                                                                 \
            ++g_failures;                                                              \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                              \
    } while (0)

constexpr uint64_t kAlive = 0xA11CEA11CEA11CEull;

// a connection whose callbacks check it is still alive
struct Conn : WebSocket {
    uint64_t magic = kAlive;
    uint64_t bytes = 0;   // written by the delivering thread only
    ~Conn() override { magic = 0; }

protected:
    void onWSReceived(const void* buffer, size_t size) override
    {
        CHECK(magic == kAlive);
        bytes += size;
        std::this_thread::yield();   // widen the window for the other thread
    }
};

// a transport that counts what it is handed, checking it is still alive
struct Sink : Transport {
    uint64_t magic = kAlive;
    std::atomic<uint64_t> bytes{0}, frames{0};
    ~Sink() override { magic = 0; }
    size_t Send(const void* b, size_t n) override { return SendAsync(b, n) ? n : 0; }
    bool SendAsync(const void*, size_t n) override
    {
        CHECK(magic == kAlive);
        bytes += n;
        ++frames;
        std::this_thread::yield();
        return true;
    }
    size_t Receive(void*, size_t) override { return 0; }
    bool Disconnect() override { return true; }
    bool IsConnected() const override { return true; }
};

static std::vector<uint8_t> unmasked_frame(size_t len, uint8_t fill)
{
    std::vector<uint8_t> f{uint8_t(0x82), uint8_t(len)};
    f.resize(2 + len, fill);
    return f;
}

// One thread feeds and flushes a receive batch; another swaps connections
// out of the table, Forgets them and deletes them at once.
static void test_receive_forget_while_flushing()
{
    WSReceiveBatch batch(nullptr);
    std::mutex table_lock;
    std::vector<Conn*> table;
    for (int i = 0; i < 12; ++i)
        table.push_back(new Conn);
    std::atomic<bool> stop{false};
    std::atomic<uint64_t> killed{0};
    std::thread killer([&] {
        std::mt19937 rng(7);
        while (!stop.load()) {
            Conn* victim;
            {
                std::lock_guard<std::mutex> g(table_lock);
                const size_t i = rng() % table.size();
                victim = table[i];
                table[i] = new Conn;
            }
            batch.Forget(*victim);   // returns once no flush will touch it
            delete victim;
            ++killed;
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    });
    const std::vector<uint8_t> f = unmasked_frame(40, 0x5A);
    size_t delivered = 0;
    for (int round = 0; round < 400; ++round) {
        {
            std::lock_guard<std::mutex> g(table_lock);
            for (Conn* c : table)
                for (int k = 0; k < 3; ++k)
                    batch.Feed(*c, f.data(), f.size());
        }
        delivered += batch.Flush();
    }
    stop = true;
    killer.join();
    CHECK(delivered > 0);
    CHECK(killed.load() > 0);
    std::lock_guard<std::mutex> g(table_lock);
    for (Conn* c : table)
        delete c;
}

// The same for a send batch: transports are forgotten and deleted while
// another thread's flush hands frames out.
static void test_send_forget_while_flushing()
{
    WSSendBatch batch(nullptr);
    std::mutex table_lock;
    std::vector<Sink*> table;
    for (int i = 0; i < 12; ++i)
        table.push_back(new Sink);
    std::atomic<bool> stop{false};
    std::atomic<uint64_t> killed{0};
    std::thread killer([&] {
        std::mt19937 rng(11);
        while (!stop.load()) {
            Sink* victim;
            {
                std::lock_guard<std::mutex> g(table_lock);
                const size_t i = rng() % table.size();
                victim = table[i];
                table[i] = new Sink;
            }
            batch.Forget(*victim);
            delete victim;
            ++killed;
            std::this_thread::sleep_for(std::chrono::microseconds(20));
        }
    });
    const uint8_t payload[32] = {1, 2, 3};
    size_t sent = 0;
    for (int round = 0; round < 400; ++round) {
        {
            std::lock_guard<std::mutex> g(table_lock);
            for (Sink* t : table)
                for (int k = 0; k < 3; ++k)
                    batch.Queue(*t, 0, 0x82, false, payload, sizeof payload);
        }
        sent += batch.Flush();
    }
    stop = true;
    killer.join();
    CHECK(sent > 0);
    CHECK(killed.load() > 0);
    std::lock_guard<std::mutex> g(table_lock);
    for (Sink* t : table)
        delete t;
}

// Frames a session queued into ANOTHER thread's BatchScope (a SendAsync
// from a worker): destroying the session on this thread drops them from that
// thread's batch (BatchScope::ForgetEverywhere), so the scope's end does not
// hand a frame to the destroyed transport.
static void test_session_destroyed_while_queued_elsewhere()
{
    constexpr int n = 6, victim = 2;
    std::vector<Sink*> sinks;
    std::vector<WSSession*> sessions;
    for (int i = 0; i < n; ++i) {
        sinks.push_back(new Sink);
        sessions.push_back(new WSSession(*sinks.back()));
    }
    std::mutex m;
    std::condition_variable cv;
    int phase = 0;
    std::thread worker([&] {
        BatchScope scope;   // e.g. an event-loop tick on a worker thread
        for (WSSession* s : sessions)
            CHECK(s->SendBinaryAsync("hello"));
        std::unique_lock<std::mutex> g(m);
        phase = 1;
        cv.notify_all();
        cv.wait(g, [&] { return phase == 2; });
        // the scope ends here: its flush hands out what is still queued
    });
    {
        std::unique_lock<std::mutex> g(m);
        cv.wait(g, [&] { return phase == 1; });
    }
    delete sessions[victim];   // ~WSSession: ForgetEverywhere
    delete sinks[victim];
    sessions[victim] = nullptr;
    sinks[victim] = nullptr;
    {
        std::lock_guard<std::mutex> g(m);
        phase = 2;
    }
    cv.notify_all();
    worker.join();
    for (int i = 0; i < n; ++i) {
        if (i == victim)
            continue;
        CHECK(sinks[i]->frames.load() == 1);
        CHECK(sinks[i]->bytes.load() == 2 + 5);   // 82 05 "hello"
        delete sessions[i];
        delete sinks[i];
    }
}

// Two threads flushing at once, each from inside a callback destroying a
// connection still queued in the OTHER thread's flush (a Forget
// that waited for the other flush's next record deadlocked here: each thread
// waited for the other, both inside a callback).  `automatic`: the batches
// are the threads' own BatchScope batches and the connections go through
// BatchScope::ForgetEverywhere, as ~WSSession / ~WSClient do.  A watchdog
// ends the process if the two flushes do not finish.
struct Trigger : Conn {
    std::function<void()> on_first;
    std::atomic<int> calls{0};

protected:
    void onWSReceived(const void* buffer, size_t size) override
    {
        Conn::onWSReceived(buffer, size);
        if (calls.fetch_add(1) == 0 && on_first)
            on_first();
    }
};

static void test_cross_thread_destroy_in_callbacks(bool automatic)
{
    for (int iter = 0; iter < 50; ++iter) {
        // per iteration on the heap (the sanitizers track a freed block; a
        // stack slot reused by the next iteration's mutex they do not)
        struct State {
            WSReceiveBatch x{nullptr}, y{nullptr};
            Trigger tx, ty;
            Conn* vx = new Conn;   // queued behind tx on thread A, destroyed by thread B's callback
            Conn* vy = new Conn;   // queued behind ty on thread B, destroyed by thread A's callback
            Sink dummy;
            std::mutex m;
            std::condition_variable cv;
            int inside = 0;
            std::atomic<int> done{0};
        };
        auto st = std::make_unique<State>();
        State& S = *st;
        auto both_inside = [&] {   // both flushes are inside a callback before either destroys
            std::unique_lock<std::mutex> g(S.m);
            ++S.inside;
            S.cv.notify_all();
            // no timed wait: this ThreadSanitizer does not intercept the
            // clock-based condition wait libstdc++ uses for wait_for (a false
            // "double lock"); the watchdog below bounds the test instead
            S.cv.wait(g, [&] { return S.inside == 2; });
        };
        auto destroy = [&](WSReceiveBatch& other, Conn*& victim) {
            if (automatic)
                BatchScope::ForgetEverywhere(*victim, S.dummy);
            else
                other.Forget(*victim);
            delete victim;
            victim = nullptr;
        };
        S.tx.on_first = [&] { both_inside(); destroy(S.y, S.vy); };
        S.ty.on_first = [&] { both_inside(); destroy(S.x, S.vx); };
        const std::vector<uint8_t> f = unmasked_frame(24, 0x33);
        auto run = [&](WSReceiveBatch& mine, Trigger& t, Conn* v) {
            if (automatic) {
                BatchScope scope;
                BatchScope::Receive().Feed(t, f.data(), f.size());
                BatchScope::Receive().Feed(*v, f.data(), f.size());
                // the scope's end flushes this thread's automatic batch
            } else {
                mine.Feed(t, f.data(), f.size());
                mine.Feed(*v, f.data(), f.size());
                mine.Flush();
            }
            ++S.done;
        };
        std::thread watchdog([&] {
            for (int i = 0; i < 200 && S.done.load() < 2; ++i)
                std::this_thread::sleep_for(std::chrono::milliseconds(100));
            if (S.done.load() < 2) {
                std::fprintf(stderr, "cross-thread destroy (%s): flushes blocked on each other\n",
                             automatic ? "automatic" : "explicit");
                std::_Exit(3);
            }
        });
        Conn* vx0 = S.vx;
        Conn* vy0 = S.vy;
        std::thread a([&] { run(S.x, S.tx, vx0); });
        std::thread b([&] { run(S.y, S.ty, vy0); });
        a.join();
        b.join();
        watchdog.join();
        CHECK(S.tx.calls.load() == 1 && S.ty.calls.load() == 1);
        CHECK(S.vx == nullptr && S.vy == nullptr);   // destroyed, and never delivered to after (Conn checks)
    }
}

// A session that counts what it is delivered and checks it is alive.
struct CountSession : WSSession {
    using WSSession::WSSession;
    uint64_t magic = kAlive;
    std::atomic<uint64_t> bytes{0};
    ~CountSession() override { magic = 0; }
    void Ready() { Handshaked(false); }   // upgraded (server side: key 0, no GPU pass)

protected:
    void onWSReceived(const void* buffer, size_t size) override
    {
        CHECK(magic == kAlive);
        bytes += size;
    }
};

// Two threads flushing at once, each from inside a callback moving a session
// off the batch the OTHER thread is flushing (SetReceiveBatch -> Drain), with
// the session's frames queued there after that flush began (Drain
// waited for the other thread's whole flush, so each waited for the other).
// Drain now waits only for the session's own frames in the running flush and
// delivers those still queued itself.  The moved session gets its frame
// exactly once, before SetReceiveBatch returns.  A watchdog ends the process
// if the flushes block on each other.
static void test_cross_thread_drain_in_callbacks()
{
    for (int iter = 0; iter < 50; ++iter) {
        struct State {
            WSReceiveBatch x{nullptr}, y{nullptr};
            Trigger tx, ty;
            Sink sink_x, sink_y;
            CountSession sx{sink_x}, sy{sink_y};   // attached to y / x, moved off them by thread A / B
            std::mutex m;
            std::condition_variable cv;
            int inside = 0;
            std::atomic<int> done{0};
        };
        auto st = std::make_unique<State>();
        State& S = *st;
        S.sx.Ready();
        S.sy.Ready();
        S.sx.SetReceiveBatch(&S.y);
        S.sy.SetReceiveBatch(&S.x);
        const std::vector<uint8_t> f = unmasked_frame(24, 0x33);
        auto both_inside = [&] {
            std::unique_lock<std::mutex> g(S.m);
            ++S.inside;
            S.cv.notify_all();
            S.cv.wait(g, [&] { return S.inside == 2; });
        };
        auto move_off = [&](CountSession& s) {
            s.onReceived(f.data(), f.size());   // queued in the batch the other thread is flushing
            s.SetReceiveBatch(nullptr);         // delivered before this returns
            CHECK(s.bytes.load() == 24);
        };
        S.tx.on_first = [&] { both_inside(); move_off(S.sx); };
        S.ty.on_first = [&] { both_inside(); move_off(S.sy); };
        auto run = [&](WSReceiveBatch& mine, Trigger& t) {
            mine.Feed(t, f.data(), f.size());
            mine.Flush();
            ++S.done;
        };
        std::thread watchdog([&] {
            for (int i = 0; i < 200 && S.done.load() < 2; ++i)
                std::this_thread::sleep_for(std::chrono::milliseconds(100));
            if (S.done.load() < 2) {
                std::fprintf(stderr, "cross-thread drain: flushes blocked on each other\n");
                std::_Exit(3);
            }
        });
        std::thread a([&] { run(S.x, S.tx); });
        std::thread b([&] { run(S.y, S.ty); });
        a.join();
        b.join();
        watchdog.join();
        CHECK(S.tx.calls.load() == 1 && S.ty.calls.load() == 1);
        // nothing of theirs left behind to deliver twice
        S.x.Flush();
        S.y.Flush();
        CHECK(S.sx.bytes.load() == 24 && S.sy.bytes.load() == 24);
    }
}

// IO threads feed their sessions' reads (RouteFrames) and send synchronously
// (SendFrame flushes the send batch) while another thread switches the
// server's batched receive and send on and off and a third flushes: no read
// may use a batch after the switch freed it, and every frame of every read is
// delivered exactly once (the frames a read put into a batch being switched
// off are flushed by the switch, not lost).
static void test_server_toggle_batches_while_reading()
{
    constexpr int kThreads = 4, kPerThread = 4, kReads = 3000, kFramesPerRead = 3, kLen = 24;
    WSServer server;
    std::vector<std::unique_ptr<Sink>> sinks;
    std::vector<std::shared_ptr<CountSession>> sessions;
    for (int i = 0; i < kThreads * kPerThread; ++i) {
        sinks.push_back(std::make_unique<Sink>());
        sessions.push_back(std::make_shared<CountSession>(*sinks.back()));
        sessions.back()->Ready();
        server.AddSession(sessions.back());
    }
    std::vector<uint8_t> read;
    for (int k = 0; k < kFramesPerRead; ++k) {
        const std::vector<uint8_t> f = unmasked_frame(kLen, uint8_t(0x40 + k));
        read.insert(read.end(), f.begin(), f.end());
    }
    std::atomic<int> running{kThreads};
    std::thread toggler([&] {
        for (uint32_t i = 0; running.load() > 0; ++i) {
            server.EnableBatchReceive(i & 1);
            server.EnableBatchSend(i & 2);
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
        server.EnableBatchReceive(false);
        server.EnableBatchSend(false);
    });
    std::thread flusher([&] {
        while (running.load() > 0) {
            server.FlushReceived();
            server.FlushSend();
            std::this_thread::yield();
        }
    });
    std::vector<std::thread> io;
    for (int t = 0; t < kThreads; ++t)
        io.emplace_back([&, t] {
            for (int r = 0; r < kReads; ++r) {
                CountSession& s = *sessions[size_t(t * kPerThread + r % kPerThread)];
                s.onReceived(read.data(), read.size());
                if (r % 64 == 0)
                    CHECK(s.SendBinary("sync", 4) == 6);   // 82 04 "sync"
            }
            --running;
        });
    for (auto& th : io)
        th.join();
    toggler.join();
    flusher.join();
    server.FlushReceived();
    uint64_t got = 0;
    for (auto& s : sessions)
        got += s->bytes.load();
    CHECK(got == uint64_t(kThreads) * kReads * kFramesPerRead * kLen);
    for (auto& s : sessions)
        server.RemoveSession(s);
}

int main()
{
    test_server_toggle_batches_while_reading();
    test_receive_forget_while_flushing();
    test_send_forget_while_flushing();
    test_session_destroyed_while_queued_elsewhere();
    if (!std::getenv("ONLY_AUTO"))
        test_cross_thread_destroy_in_callbacks(false);
    if (!std::getenv("ONLY_EXPLICIT"))
        test_cross_thread_destroy_in_callbacks(true);
    test_cross_thread_drain_in_callbacks();
    std::printf("%d checks, %d failures\n", g_checks.load(), g_failures.load());
    return g_failures.load() == 0 ? 0 : 1;
}
