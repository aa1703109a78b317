// echo_prof.cpp — where C1's time goes.  Linked into
// bench_echo as tools/_build/bench_echo_prof: the executable's definitions
// of these library entry points take the place of libwsg.so's (symbol
// interposition; the library's own calls go through its PLT) and forward to
// the real ones, timing each call:
//   WSReceiveBatch::Feed   host framing of a read
//   WSReceiveBatch::Flush  GPU unmask pass + delivery (the echo's callbacks,
//                          which queue the replies, run inside it)
//   WSSendBatch::Flush     GPU mask pass + hand-off to the transports
//   wsg_decode_batch_host / wsg_encode_batch_host   the GPU passes alone
// At exit: one JSON line on stderr, microseconds per call and totals.
#include "wsg_capi.h"

#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <initializer_list>

namespace {

struct Acc {
    const char* name;
    std::atomic<uint64_t> calls{0}, ns{0}, frames{0};
};
Acc g_feed{"rx_feed"}, g_rx{"rx_flush"}, g_tx{"tx_flush"}, g_dec{"gpu_decode_host"}, g_enc{"gpu_encode_host"};

uint64_t now_ns()
{
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch())
                        .count());
}

struct Timer {
    Acc& a;
    uint64_t t0 = now_ns();
    uint64_t frames = 0;
    ~Timer()
    {
        a.ns += now_ns() - t0;
        a.calls += 1;
        a.frames += frames;
    }
};

template <class F>
F real(const char* name)
{
    void* p = dlsym(RTLD_NEXT, name);
    if (!p) {
        std::fprintf(stderr, "echo_prof: %s not found\n", name);
        std::abort();
    }
    return reinterpret_cast<F>(p);
}

void report()
{
    std::fprintf(stderr, "ECHO_PROF {");
    bool first = true;
    for (Acc* a : {&g_feed, &g_rx, &g_tx, &g_dec, &g_enc}) {
        const double us = double(a->ns.load()) / 1e3;
        const uint64_t c = a->calls.load();
        std::fprintf(stderr, "%s\"%s\": {\"calls\": %llu, \"total_us\": %.1f, \"us_per_call\": %.3f, \"frames\": %llu}",
                     first ? "" : ", ", a->name, (unsigned long long)c, us, c ? us / double(c) : 0.0,
                     (unsigned long long)a->frames.load());
        first = false;
    }
    std::fprintf(stderr, "}\n");
}

struct AtExit {
    AtExit() { std::atexit(report); }
} g_at_exit;

} // namespace

extern "C" {

int wsg_decode_batch_host(wsg_ctx* c, const uint8_t* wire, uint64_t wire_len, const uint64_t* frame_start,
                          uint32_t n, uint8_t* out, wsg_recv_info* info)
{
    using F = int (*)(wsg_ctx*, const uint8_t*, uint64_t, const uint64_t*, uint32_t, uint8_t*, wsg_recv_info*);
    static F f = real<F>("wsg_decode_batch_host");
    Timer t{g_dec};
    t.frames = n;
    return f(c, wire, wire_len, frame_start, n, out, info);
}

int wsg_encode_batch_host(wsg_ctx* c, const uint8_t* payload, uint64_t payload_len, const wsg_send_desc* desc,
                          uint32_t n, uint8_t* wire, uint64_t wire_cap, uint64_t* wire_off)
{
    using F = int (*)(wsg_ctx*, const uint8_t*, uint64_t, const wsg_send_desc*, uint32_t, uint8_t*, uint64_t,
                      uint64_t*);
    static F f = real<F>("wsg_encode_batch_host");
    Timer t{g_enc};
    t.frames = n;
    return f(c, payload, payload_len, desc, n, wire, wire_cap, wire_off);
}

// CppServer::WS::WSReceiveBatch::Feed(WebSocket&, const void*, size_t)
void _ZN9CppServer2WS14WSReceiveBatch4FeedERNS0_9WebSocketEPKvm(void* self, void* ws, const void* b, size_t n)
{
    using F = void (*)(void*, void*, const void*, size_t);
    static F f = real<F>("_ZN9CppServer2WS14WSReceiveBatch4FeedERNS0_9WebSocketEPKvm");
    Timer t{g_feed};
    f(self, ws, b, n);
}

// CppServer::WS::WSReceiveBatch::Flush()
size_t _ZN9CppServer2WS14WSReceiveBatch5FlushEv(void* self)
{
    using F = size_t (*)(void*);
    static F f = real<F>("_ZN9CppServer2WS14WSReceiveBatch5FlushEv");
    Timer t{g_rx};
    const size_t r = f(self);
    t.frames = r;
    return r;
}

// CppServer::WS::WSSendBatch::Flush(Sink, void*)
size_t _ZN9CppServer2WS11WSSendBatch5FlushEPFvPvS2_PKhmES2_(void* self, void* sink, void* user)
{
    using F = size_t (*)(void*, void*, void*);
    static F f = real<F>("_ZN9CppServer2WS11WSSendBatch5FlushEPFvPvS2_PKhmES2_");
    Timer t{g_tx};
    const size_t r = f(self, sink, user);
    t.frames = r;
    return r;
}

} // extern "C"
