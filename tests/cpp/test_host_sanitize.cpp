// test_host_sanitize.cpp — host code under AddressSanitizer + UBSan
// ("-fsanitize=address,undefined CI target for the CPU
// restatement and shim").  Built by `make -C tests/cpp sanitize` from the
// sources themselves (the oracle's ws_oracle.cpp, the product's http.cpp),
// run by tests/test_sanitize.py on the CPU.  Exercises:
//   * the oracle (test infrastructure, oracle/ws_oracle.cpp): random frames of
//     every length class encoded, decoded whole, and fed to the streaming
//     parser in random splits (the reference's split-header behaviour, Q7,
//     included), plus garbage streams; batch encode/decode of random batches
//     with garbage frame tables;
//   * the HTTP request/response parser of the upgrade (http.cpp) on random,
//     truncated and mutated inputs, and the Base64 / accept-key helpers.
#include "server/http/http_request.h"
#include "server/http/http_response.h"
#include "server/ws/ws_handshake.h"

#include "../../oracle/ws_oracle.h"

#include <cstdio>
#include <cstring>
#include <exception>
#include <random>
#include <string>
#include <vector>

using namespace CppServer;

static int g_failures = 0, g_checks = 0;
#define CHECK(cond)                                                                    \
    do {                                                                               \
        ++g_checks;                                                                    \
        if (!(cond)) {                                                                 \
            ++g_failures;                                                              \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
        }                                                                              \
    } while (0)

static std::mt19937_64 g_rng(12345);

static size_t pick_len()
{
    static const size_t classes[] = {0, 1, 2, 15, 16, 17, 124, 125, 126, 127, 128, 1000, 65535, 65536, 70000};
    return (g_rng() % 3 == 0) ? classes[g_rng() % (sizeof(classes) / sizeof(classes[0]))] : size_t(g_rng() % 3000);
}

static void test_oracle_roundtrips()
{
    static const uint8_t ops[] = {0x81, 0x82, 0x01, 0x02, 0x00, 0x80, 0x88, 0x89, 0x8A, 0xC2, 0x83};
    for (int it = 0; it < 300; ++it) {
        wso_session* tx = wso_new();
        wso_session* rx = wso_new();
        const uint32_t key = uint32_t(g_rng());
        wso_set_send_key(tx, key);
        std::vector<uint8_t> stream;
        const int frames = 1 + int(g_rng() % 6);
        for (int f = 0; f < frames; ++f) {
            std::vector<uint8_t> payload(pick_len());
            for (auto& b : payload)
                b = uint8_t(g_rng());
            const uint8_t op = ops[g_rng() % sizeof(ops)];
            const int32_t status = (g_rng() % 4 == 0) ? int32_t(g_rng() % 70000) : 0;
            wso_prepare_send(tx, op, int(g_rng() & 1), payload.data(), payload.size(), status);
            size_t n = 0;
            const uint8_t* fr = wso_send_buffer(tx, &n);
            stream.insert(stream.end(), fr, fr + n);
        }
        // whole stream in one read, then in random splits on a fresh session
        wso_prepare_receive(rx, stream.data(), stream.size());
        const size_t whole = wso_event_count(rx);
        wso_session* rx2 = wso_new();
        for (size_t at = 0; at < stream.size();) {
            const size_t take = std::min<size_t>(stream.size() - at, 1 + g_rng() % 40);
            (void)wso_required(rx2);
            wso_prepare_receive(rx2, stream.data() + at, take);
            at += take;
        }
        CHECK(whole <= size_t(frames));
        for (size_t i = 0; i < wso_event_count(rx); ++i) {
            int kind = 0, status = 0;
            const uint8_t* d = nullptr;
            size_t len = 0;
            wso_event(rx, i, &kind, &status, &d, &len);
            CHECK(kind >= 1 && kind <= 4);
            if (len)
                CHECK(d != nullptr);
        }
        wso_free(rx2);
        wso_free(rx);
        wso_free(tx);
    }
}

static void test_oracle_garbage_streams()
{
    for (int it = 0; it < 2000; ++it) {
        std::vector<uint8_t> junk(g_rng() % 200);
        for (auto& b : junk)
            b = uint8_t(g_rng());
        // no byte reads as the 127 (64-bit length) form: a garbage 64-bit
        // length would ask for gigabytes (the reference's reserve() throws or
        // the allocator gives up); the 7- and 16-bit forms stay random
        for (auto& b : junk)
            if ((b & 0x7F) == 0x7F)
                b ^= 1;
        wso_session* s = wso_new();
        try {
            for (size_t at = 0; at < junk.size();) {
                const size_t take = std::min<size_t>(junk.size() - at, 1 + g_rng() % 9);
                wso_prepare_receive(s, junk.data() + at, take);
                at += take;
            }
        } catch (const std::exception&) {
            // a garbage 64-bit length makes the reference's reserve() throw
            // (ws.cpp:388-389, std::length_error / std::bad_alloc): that is
            // its behaviour, not a memory error
        }
        (void)wso_required(s);
        wso_clear(s);
        wso_free(s);
    }
    CHECK(true);
}

static void test_oracle_batches()
{
    for (int it = 0; it < 100; ++it) {
        const uint32_t n = 1 + uint32_t(g_rng() % 200);
        std::vector<wsg_send_desc> desc(n);
        uint64_t at = 0;
        for (auto& d : desc) {
            d = wsg_send_desc{};
            d.len = pick_len() % 5000;
            d.src_off = at;
            d.key = uint32_t(g_rng());
            d.opcode = (g_rng() % 5 == 0) ? 0x88 : 0x82;
            d.status = d.opcode == 0x88 ? 1000 : 0;
            d.mask = uint8_t(g_rng() & 1);
            at += d.len;
        }
        std::vector<uint8_t> payload(at + 1);
        for (auto& b : payload)
            b = uint8_t(g_rng());
        std::vector<uint8_t> wire(at + 16 * n + 16);
        std::vector<uint64_t> off(n + 1);
        CHECK(wso_encode_batch(payload.data(), desc.data(), n, wire.data(), wire.size(), off.data()) == 0);
        const uint64_t len = off[n];
        std::vector<uint8_t> out(len + 1);
        std::vector<wsg_recv_info> info(n);
        CHECK(wso_decode_batch(wire.data(), len, off.data(), n, out.data(), info.data()) == 0);
        for (uint32_t i = 0; i < n; ++i)
            CHECK(info[i].len == desc[i].len + (desc[i].opcode == 0x88 ? 2 : 0));
        // garbage frame tables: any status, no memory error
        std::vector<uint64_t> bad(off.begin(), off.end() - 1);
        for (auto& b : bad)
            if (g_rng() % 4 == 0)
                b = g_rng() % (len + 50);
        (void)wso_decode_batch(wire.data(), len, bad.data(), n, out.data(), info.data());
    }
}

static void test_http_parser()
{
    const std::string base = "GET /chat HTTP/1.1\r\nHost: server.example.com\r\nUpgrade: websocket\r\n"
                             "Connection: Upgrade\r\nSec-WebSocket-Key: dGhlIHNhbXBsZSBub25jZQ==\r\n"
                             "Sec-WebSocket-Version: 13\r\n\r\n";
    HTTP::HTTPRequest req;
    CHECK(req.Parse(base) == base.size());
    CHECK(!req.error());
    for (int it = 0; it < 5000; ++it) {
        std::string m = base;
        const int edits = 1 + int(g_rng() % 4);
        for (int e = 0; e < edits; ++e) {
            const size_t at = g_rng() % m.size();
            switch (g_rng() % 3) {
            case 0:
                m[at] = char(g_rng());
                break;
            case 1:
                m.erase(at, 1 + g_rng() % 5);
                break;
            default:
                m.insert(at, std::string(1 + g_rng() % 5, char(g_rng())));
                break;
            }
            if (m.empty())
                m = "\r\n";
        }
        m = m.substr(0, g_rng() % (m.size() + 1));
        HTTP::HTTPRequest r;
        const size_t used = r.Parse(m);
        CHECK(used <= m.size());
        HTTP::HTTPResponse resp;
        (void)resp.Parse(m);
    }
    const std::string ok = "HTTP/1.1 101 Switching Protocols\r\nUpgrade: websocket\r\nConnection: Upgrade\r\n"
                           "Sec-WebSocket-Accept: s3pPLMBiTxaQ9kYGzzhZRbK+xOo=\r\n\r\n";
    HTTP::HTTPResponse resp;
    CHECK(resp.Parse(ok) == ok.size());
    CHECK(resp.status() == 101);
}

static void test_base64()
{
    CHECK(WS::WSAcceptKey("dGhlIHNhbXBsZSBub25jZQ==") == "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=");
    for (int it = 0; it < 2000; ++it) {
        std::string s(g_rng() % 100, '\0');
        for (auto& c : s)
            c = char(g_rng());
        CHECK(WS::Base64Decode(WS::Base64Encode(s)) == s);
        std::string junk(g_rng() % 50, '\0');
        for (auto& c : junk)
            c = char(g_rng());
        (void)WS::Base64Decode(junk);
    }
}

int main()
{
    test_oracle_roundtrips();
    test_oracle_garbage_streams();
    test_oracle_batches();
    test_http_parser();
    test_base64();
    std::printf("%d checks, %d failures\n", g_checks, g_failures);
    return g_failures == 0 ? 0 : 1;
}
