// bench_batch.cpp — end-to-end rate of the batched receive / send paths
// (WSReceiveBatch / WSSendBatch) against the
// per-call path (one PrepareReceiveFrame / PrepareSendFrame per frame, each
// with its own GPU XOR), on host buffers: host framing, PCIe both ways, the
// kernels and the callbacks are all inside the timed region.
//
//   bench_batch rx|tx SESSIONS FRAMES_PER_SESSION PAYLOAD [FEED_CHUNK] [REPS]
//
// Prints one JSON object.  Uses only the product library (libwsg.so).
#include "server/ws/ws_batch.h"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <vector>

using namespace CppServer::WS;
using Clock = std::chrono::steady_clock;

namespace {

struct Conn : WebSocket {
    uint64_t bytes = 0, messages = 0, sum = 0;
    void onWSReceived(const void* b, size_t n) override
    {
        bytes += n;
        ++messages;
        if (n)
            sum += static_cast<const uint8_t*>(b)[n - 1];
    }
    using WebSocket::PrepareReceiveFrame;
    using WebSocket::PrepareSendFrame;
    const std::vector<uint8_t>& sent() const { return _ws_send_buffer; }
};

double seconds(Clock::time_point a, Clock::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// client-style masked binary frames of random bytes (masking random bytes
// gives random bytes, so the wire is a valid stream without encoding it)
std::vector<uint8_t> make_stream(std::mt19937_64& g, int frames, size_t payload)
{
    std::vector<uint8_t> s;
    for (int f = 0; f < frames; ++f) {
        uint8_t h[16];
        const int n = wsg_header_pack(WSG_FIN | WSG_BINARY, 1, payload, 0, uint32_t(g()), h);
        s.insert(s.end(), h, h + n);
        const size_t at = s.size();
        s.resize(at + payload);
        for (size_t k = 0; k < payload; k += 8) {
            const uint64_t v = g();
            std::memcpy(&s[at + k], &v, std::min<size_t>(8, payload - k));
        }
    }
    return s;
}

int rx(int S, int F, size_t P, size_t chunk, int reps)
{
    std::mt19937_64 g(1);
    std::vector<std::vector<uint8_t>> streams(S);
    for (auto& s : streams)
        s = make_stream(g, F, P);
    std::vector<Conn> conns(S);
    WSReceiveBatch batch;
    auto feed_all = [&](auto&& feed) {
        std::vector<size_t> pos(S, 0);
        for (bool more = true; more;) {
            more = false;
            for (int i = 0; i < S; ++i) {
                const size_t n = std::min(chunk ? chunk : streams[i].size(), streams[i].size() - pos[i]);
                if (n) {
                    feed(i, streams[i].data() + pos[i], n);
                    pos[i] += n;
                    more = more || pos[i] < streams[i].size();
                }
            }
        }
    };
    double best_b = 1e30, best_p = 1e30;
    for (int r = 0; r <= reps; ++r) {
        auto t0 = Clock::now();
        feed_all([&](int i, const uint8_t* d, size_t n) { batch.Feed(conns[i], d, n); });
        batch.Flush();
        auto t1 = Clock::now();
        feed_all([&](int i, const uint8_t* d, size_t n) { conns[i].PrepareReceiveFrame(d, n); });
        auto t2 = Clock::now();
        if (r) {   // rep 0 warms up (pinned buffers, device scratch)
            best_b = std::min(best_b, seconds(t0, t1));
            best_p = std::min(best_p, seconds(t1, t2));
        }
    }
    uint64_t bytes = 0, msgs = 0;
    for (auto& c : conns) {
        bytes += c.bytes;
        msgs += c.messages;
    }
    const double payload = double(S) * F * P;
    const bool ok = bytes == uint64_t(payload) * 2 * (reps + 1) && msgs == uint64_t(S) * F * 2 * (reps + 1);
    if (!ok) {
        int shown = 0;
        for (int i = 0; i < S && shown < 5; ++i)
            if (conns[i].messages != uint64_t(F) * 2 * (reps + 1) || conns[i].bytes != uint64_t(F) * P * 2 * (reps + 1)) {
                std::fprintf(stderr, "rx: session %d got %llu messages / %llu bytes\n", i,
                             (unsigned long long)conns[i].messages, (unsigned long long)conns[i].bytes);
                ++shown;
            }
    }
    if (!ok)
        std::fprintf(stderr, "rx: delivered %llu bytes / %llu messages, expected %llu / %llu\n",
                     (unsigned long long)bytes, (unsigned long long)msgs,
                     (unsigned long long)(uint64_t(payload) * 2 * (reps + 1)),
                     (unsigned long long)(uint64_t(S) * F * 2 * (reps + 1)));
    std::printf("{\"mode\": \"rx\", \"sessions\": %d, \"frames_per_session\": %d, \"payload\": %zu, \"feed_chunk\": %zu, "
                "\"batched_GiBps\": %.3f, \"per_call_GiBps\": %.3f, \"batched_frames_per_s\": %.0f, "
                "\"per_call_frames_per_s\": %.0f, \"delivered_ok\": %s}\n",
                S, F, P, chunk, payload / best_b / (1 << 30), payload / best_p / (1 << 30), S * F / best_b,
                S * F / best_p, ok ? "true" : "false");
    return ok ? 0 : 1;
}

int tx(int S, int F, size_t P, int reps)
{
    std::mt19937_64 g(2);
    std::vector<uint8_t> payload(P);
    for (auto& b : payload)
        b = uint8_t(g());
    std::vector<Conn> conns(S);
    std::vector<uint32_t> keys(S);
    for (int i = 0; i < S; ++i) {
        keys[i] = uint32_t(g()) | 1u;
        conns[i].set_send_key(keys[i]);
    }
    WSSendBatch batch;
    uint64_t sunk = 0;
    auto sink = [](void* user, void*, const uint8_t*, size_t n) { *static_cast<uint64_t*>(user) += n; };
    double best_b = 1e30, best_p = 1e30;
    uint64_t per_call = 0;
    for (int r = 0; r <= reps; ++r) {
        auto t0 = Clock::now();
        for (int f = 0; f < F; ++f)
            for (int i = 0; i < S; ++i)
                batch.Queue(static_cast<void*>(&conns[i]), keys[i], WSG_FIN | WSG_BINARY, true, payload.data(), P);
        batch.Flush(sink, &sunk);
        auto t1 = Clock::now();
        for (int f = 0; f < F; ++f)
            for (int i = 0; i < S; ++i) {
                conns[i].PrepareSendFrame(WSG_FIN | WSG_BINARY, true, payload.data(), P);
                per_call += conns[i].sent().size();
            }
        auto t2 = Clock::now();
        if (r) {
            best_b = std::min(best_b, seconds(t0, t1));
            best_p = std::min(best_p, seconds(t1, t2));
        }
    }
    const double bytes = double(S) * F * P;
    const bool ok = sunk == per_call && sunk == uint64_t(S) * F * wsg_frame_size(WSG_FIN | WSG_BINARY, 1, P, 0) * (reps + 1);
    std::printf("{\"mode\": \"tx\", \"sessions\": %d, \"frames_per_session\": %d, \"payload\": %zu, "
                "\"batched_GiBps\": %.3f, \"per_call_GiBps\": %.3f, \"batched_frames_per_s\": %.0f, "
                "\"per_call_frames_per_s\": %.0f, \"delivered_ok\": %s}\n",
                S, F, P, bytes / best_b / (1 << 30), bytes / best_p / (1 << 30), S * F / best_b, S * F / best_p,
                ok ? "true" : "false");
    return ok ? 0 : 1;
}

} // namespace

int main(int argc, char** argv)
{
    if (argc < 5) {
        std::fprintf(stderr, "usage: %s rx|tx SESSIONS FRAMES PAYLOAD [FEED_CHUNK] [REPS]\n", argv[0]);
        return 2;
    }
    const std::string mode = argv[1];
    const int S = std::atoi(argv[2]), F = std::atoi(argv[3]);
    const size_t P = std::strtoull(argv[4], nullptr, 10);
    const size_t chunk = argc > 5 ? std::strtoull(argv[5], nullptr, 10) : 0;
    const int reps = argc > 6 ? std::atoi(argv[6]) : 3;
    try {
        return mode == "rx" ? rx(S, F, P, chunk, reps) : tx(S, F, P, reps);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "bench_batch: %s\n", e.what());
        return 3;
    }
}
